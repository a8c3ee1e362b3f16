"""GPU parity of ORB extraction against the CPU oracle:
bit-exact pyramid, blurred levels, keypoints (28-byte records, same order) and
256-bit descriptors."""
import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd import ORBextractor, synth

pytestmark = pytest.mark.gpu

CASES = [("euroc", 1000, 0), ("euroc", 1000, 7), ("tum", 1000, 3), ("tum", 2000, 5)]


def _frame(cam, seed):
    w, h = synth.CAMERAS[cam][:2]
    return synth.synth_frame(w, h, synth.frame_seed(0, seed))


@pytest.mark.parametrize("cam,nf,seed", CASES)
def test_pyramid_and_blur_bit_exact(cam, nf, seed):
    img = _frame(cam, seed)
    ex = ORBextractor(nf, 1.2, 8, 1, 20)
    ex(img)
    for lvl in range(8):
        np.testing.assert_array_equal(ex.debug_level(lvl, 0), O.level(img, lvl, 0, nfeatures=nf),
                                      err_msg=f"pyramid level {lvl}")
        np.testing.assert_array_equal(ex.debug_level(lvl, 1), O.level(img, lvl, 1, nfeatures=nf),
                                      err_msg=f"blurred level {lvl}")


@pytest.mark.parametrize("w,h,scale,nl", [(1241, 376, 1.2, 8), (1920, 1080, 1.2, 8), (640, 480, 1.5, 5),
                                          (752, 480, 2.0, 4), (800, 600, 3.0, 3), (320, 240, 1.1, 10)])
def test_pyramid_geometries(w, h, scale, nl):
    """k_pyramid's block plan (spans, column groups of 4 or 1) on other frame
    sizes and scale factors: every level and its blur bit-exact."""
    img = synth.synth_frame(w, h, synth.frame_seed(1, w + nl))
    ex = ORBextractor(1000, scale, nl, 1, 20)
    ex(img)
    for lvl in range(nl):
        np.testing.assert_array_equal(ex.debug_level(lvl, 0), O.level(img, lvl, 0, scale=scale, nlevels=nl),
                                      err_msg=f"pyramid level {lvl}")
        np.testing.assert_array_equal(ex.debug_level(lvl, 1), O.level(img, lvl, 1, scale=scale, nlevels=nl),
                                      err_msg=f"blurred level {lvl}")


def _diff_report(kg, ko):
    n = min(len(kg), len(ko))
    bad = np.nonzero(kg[:n].tobytes() != ko[:n].tobytes())
    for i in range(n):
        if kg[i].tobytes() != ko[i].tobytes():
            return f"first mismatch at {i}: gpu={kg[i]} oracle={ko[i]}"
    return f"len gpu={len(kg)} oracle={len(ko)}"


@pytest.mark.parametrize("cam,nf,seed", CASES)
def test_keypoints_descriptors_bit_exact(cam, nf, seed):
    img = _frame(cam, seed)
    ex = ORBextractor(nf, 1.2, 8, 1, 20)
    kg, dg = ex(img)
    ko, do = O.extract(img, nfeatures=nf)
    assert kg.tobytes() == ko.tobytes(), _diff_report(kg, ko)
    assert np.array_equal(dg, do), f"descriptor rows differ: {np.nonzero((dg != do).any(1))[0][:10]}"


def test_golden_frames_gpu():
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "extract_golden.json")))
    for case in g["cases"]:
        img = np.load(os.path.join(os.path.dirname(__file__), "golden", case["frame"]))
        ex = ORBextractor(case["nfeatures"], 1.2, 8, 1, 20)
        kg, dg = ex(img)
        ko, do = O.extract(img, nfeatures=case["nfeatures"])
        assert kg.tobytes() == ko.tobytes(), _diff_report(kg, ko)
        assert np.array_equal(dg, do)


def test_low_texture_threshold_fallback():
    """Flat image with a few weak corners: every cell falls back to the
    minimum threshold (ORBextractor.cc:623-628); quotas redistribute."""
    rng = np.random.default_rng(4)
    img = np.full((480, 640), 128, np.uint8)
    img += rng.integers(0, 12, img.shape, dtype=np.uint8)
    img[100:140, 200:260] = 40
    ex = ORBextractor(1000, 1.2, 8, 1, 20)
    kg, dg = ex(img)
    ko, do = O.extract(img)
    assert kg.tobytes() == ko.tobytes(), _diff_report(kg, ko)
    assert np.array_equal(dg, do)


@pytest.mark.parametrize("fast_th", [0, 5, 7, 40])
def test_fast_threshold_edges(fast_th):
    """Thresholds at and below the minimum one (7): the score map is built at
    min(fastTh, 7), where a threshold of 0 admits corners of score 0."""
    img = _frame("euroc", 11)
    kg, dg = ORBextractor(1000, 1.2, 8, 1, fast_th)(img)
    ko, do = O.extract(img, nfeatures=1000, fast_th=fast_th)
    assert kg.tobytes() == ko.tobytes(), _diff_report(kg, ko)
    assert np.array_equal(dg, do)


@pytest.mark.parametrize("cam", ["euroc", "tum"])
@pytest.mark.parametrize("score_type", [1, 0])
@pytest.mark.parametrize("nf", [150, 200, 250, 500, 1000, 2000])
def test_nfeatures_and_score_type(nf, score_type, cam):
    """The reference's nFeatures range and both score types (ORBextractor.h:57,
    ORBextractor.nScoreType in the settings, Tracking.cc:186): few features
    make few, large cells (752x480 at 200 features: windows of ~360x150 px at
    level 0) whose window runs k_fast_cells_band in row bands; HARRIS_SCORE (0)
    replaces each FAST corner's response by HarrisResponses (ORBextractor.cc
    :86-127, 667-670) before retainBest. Bit-exact keypoints (responses
    included) and descriptors. Harris: parity unpinned (no reference fixture;
    docs/ORACLE_ASSUMPTIONS.md A21)."""
    img = _frame(cam, 40 + nf % 7)
    kg, dg = ORBextractor(nf, 1.2, 8, score_type, 20)(img)
    ko, do = O.extract(img, nfeatures=nf, score_type=score_type)
    assert len(ko) > 0.8 * nf
    assert kg.tobytes() == ko.tobytes(), _diff_report(kg, ko)
    assert np.array_equal(dg, do)
    if score_type == 0:
        assert np.any(ko["response"] != np.round(ko["response"]))  # Harris responses, not FAST scores


@pytest.mark.parametrize("score_type", [1, 0])
def test_banded_cells_threshold_fallback(score_type):
    """Large cells (200 features) on a flat image with weak texture: every
    banded window falls back to the minimum threshold (the retry pass
    recomputes the scores band by band from the level) and quotas
    redistribute (ORBextractor.cc:623-628, 695-721)."""
    rng = np.random.default_rng(6)
    img = np.full((480, 752), 128, np.uint8)
    img += rng.integers(0, 12, img.shape, dtype=np.uint8)
    img[100:140, 200:260] = 40
    img[300:330, 500:600] = 200
    kg, dg = ORBextractor(200, 1.2, 8, score_type, 20)(img)
    ko, do = O.extract(img, nfeatures=200, score_type=score_type)
    assert kg.tobytes() == ko.tobytes(), _diff_report(kg, ko)
    assert np.array_equal(dg, do)


@pytest.mark.parametrize("nf", [200, 500, 1000])
def test_long_cell_lists(nf):
    """Dense corners: uniform noise whose contrast ramps across the image,
    so a cell's corner list after NMS spans from none to thousands (cells of
    twenty thousand pixels at 500 features). Lists longer than the
    selection's per-wave LDS buffers (k_select: SEL_BUF = SEL_BUF_CELL = 1024
    entries; with -DSEL_BUF_CELL=256 lists of 257..1024 wait for wave 0's
    buffer) take the sequential replay in global memory; the cut must match
    the oracle's retainBest either way (ORBextractor.cc:647-651, 750-752)."""
    rng = np.random.default_rng(21)
    h, w = 480, 752
    amp = np.linspace(0, 255, w)[None, :]
    img = (128 + (rng.random((h, w)) - 0.5) * amp).clip(0, 255).astype(np.uint8)
    kg, dg = ORBextractor(nf, 1.2, 8, 1, 20)(img)
    ko, do = O.extract(img, nfeatures=nf)
    assert kg.tobytes() == ko.tobytes(), _diff_report(kg, ko)
    assert np.array_equal(dg, do)


def test_flat_image_no_keypoints():
    img = np.full((480, 640), 77, np.uint8)
    kg, dg = ORBextractor(1000)(img)
    assert len(kg) == 0 and dg.shape == (0, 32)


def test_batch_device_matches_host():
    import torch
    frames = np.stack([_frame("euroc", s) for s in range(3)])
    ex = ORBextractor(1000, 1.2, 8, 1, 20, width=752, height=480, max_batch=3)
    imgs = torch.from_numpy(frames).cuda()
    cap = ex.capacity
    kps = torch.zeros((3, cap, 28), dtype=torch.uint8, device="cuda")
    desc = torch.zeros((3, cap, 32), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(3, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ex.extract_batch_dev(imgs, kps, desc, cnt)
    ex.ctx.sync()
    for f in range(3):
        ko, do = O.extract(frames[f])
        n = int(cnt[f])
        assert n == len(ko)
        assert kps[f, :n].cpu().numpy().tobytes() == ko.tobytes()
        assert np.array_equal(desc[f, :n].cpu().numpy(), do)
