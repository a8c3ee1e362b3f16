"""Keypoint undistortion (Frame::UndistortKeyPoints, Frame.cc:389-423 —
cv::undistortPoints restated from OpenCV 3.4; parity unpinned against OpenCV
itself, which is not in the container). CPU: the oracle's properties; GPU: the
kernel against the oracle bit for bit."""
import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd import synth

EUROC_K = (458.654, 457.296, 367.215, 248.375)
EUROC_D = (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05)       # EuRoC cam0
TUM2_K = (520.908620, 521.007327, 325.141442, 249.701764)
TUM2_D = (0.231222, -0.784899, -0.003257, -0.000105, 0.917205)        # TUM fr2


def _kps(n, seed, w=752, h=480):
    sc = synth.synth_scene("euroc", 1500, n, seed)
    k = sc["keypoints"].copy()
    rng = np.random.default_rng(seed)
    k["x"] = rng.uniform(0, w - 1, n).astype(np.float32)
    k["y"] = rng.uniform(0, h - 1, n).astype(np.float32)
    return k


def _distort(K, D, x, y):  # the forward radial-tangential model (double)
    fx, fy, cx, cy = K
    d = list(D) + [0.0] * (5 - len(D))
    k1, k2, p1, p2, k3 = d
    xn, yn = (x - cx) / fx, (y - cy) / fy
    r2 = xn * xn + yn * yn
    rad = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 ** 3
    xd = xn * rad + 2 * p1 * xn * yn + p2 * (r2 + 2 * xn * xn)
    yd = yn * rad + p1 * (r2 + 2 * yn * yn) + 2 * p2 * xn * yn
    return xd * fx + cx, yd * fy + cy


def test_oracle_copies_when_k1_is_zero():
    k = _kps(300, 1)
    u = O.undistort_keypoints(k, EUROC_K, (0.0, 0.1, 0.01, 0.01))
    assert u.tobytes() == k.tobytes()


@pytest.mark.parametrize("K,D", [(EUROC_K, EUROC_D), (TUM2_K, TUM2_D)])
def test_oracle_inverts_the_distortion(K, D):
    """Five fixed-point iterations: redistorting the result lands within a
    fraction of a pixel of the input over the central image."""
    k = _kps(500, 2)
    u = O.undistort_keypoints(k, K, D)
    assert np.array_equal(u["octave"], k["octave"]) and np.array_equal(u["angle"], k["angle"])
    x, y = _distort(K, D, u["x"].astype(np.float64), u["y"].astype(np.float64))
    central = (np.abs(k["x"] - K[2]) < 250) & (np.abs(k["y"] - K[3]) < 180)
    assert np.abs(x - k["x"])[central].max() < 0.05 and np.abs(y - k["y"])[central].max() < 0.05


@pytest.mark.gpu
@pytest.mark.parametrize("K,D", [(EUROC_K, EUROC_D), (TUM2_K, TUM2_D), (EUROC_K, (0.0, 0.0, 0.0, 0.0))])
def test_undistort_gpu_bit_exact(K, D):
    from gf_orb_slam_amd.matcher import undistort_keypoints

    k = _kps(1000, 3)
    g = undistort_keypoints(k, K, D)
    o = O.undistort_keypoints(k, K, D)
    assert g.tobytes() == o.tobytes()


def test_oracle_frame_bounds():
    """Frame::ComputeImageBounds (Frame.cc:425-493): with EuRoC's barrel
    distortion the undistorted corners lie outside the image, so the bounds
    widen; k1 = 0 gives the image."""
    import ctypes

    o = O.orc()
    b = (ctypes.c_int * 4)()
    K = (ctypes.c_float * 4)(*EUROC_K)
    D = (ctypes.c_float * 5)(*(list(EUROC_D) + [0.0]))
    assert o.orc_frame_bounds(K, D, 752, 480, b) == 0
    mnMinX, mnMaxX, mnMinY, mnMaxY = list(b)
    assert mnMinX < 0 and mnMaxX > 752 and mnMinY < 0 and mnMaxY > 480
    Z = (ctypes.c_float * 5)(0, 0.1, 0, 0, 0)
    assert o.orc_frame_bounds(K, Z, 752, 480, b) == 0 and list(b) == [0, 752, 0, 480]
