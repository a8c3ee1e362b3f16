"""Host-side parts of the GF module in libgfslam (no GPU needed): the glibc
rand() port and the PWLS kinematics, against glibc and the oracle/KATs."""
import ctypes
import json
import os

import numpy as np

import oracle_lib as O
from gf_orb_slam_amd.observability import Observability, ObsCamera, Rng

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat_observability.json")))


def test_rng_port_matches_glibc():
    libc = ctypes.CDLL("libc.so.6")
    for seed in (1, 7, 12345, 2**31 + 5):
        libc.srand(ctypes.c_uint(seed))
        ref = [libc.rand() for _ in range(5000)]
        assert list(Rng.seeded(seed).next(5000)) == ref


def _obs():
    return Observability.__new__(Observability)


def test_predict_matches_oracle_bitwise():
    for case in ("kine1", "kine2"):
        c = KAT[case]
        ob = _obs()
        ob.Xv = np.array(c["Xv"])
        ob.predictPWLSVec(c["dt"], c["nseg"])
        ko = O.obs_predict(c["Xv"], c["dt"], c["nseg"])
        for a, b in zip(ob.kinematic, ko):
            assert bytes(a) == bytes(b)


def test_predict_kat():
    c = KAT["kine2"]
    ob = _obs()
    ob.Xv = np.array(c["Xv"])
    ob.predictPWLSVec(c["dt"], 3)
    for i, k in enumerate(ob.kinematic):
        assert np.abs(np.array(k.F_Q[:]).reshape(4, 4) - c["F_Q"][i]).sum(1).max() < 0.002
        assert np.abs(np.array(k.F_Omg[:]).reshape(4, 3) - c["F_Omg"][i]).sum(1).max() < 0.0002


def test_update_matches_oracle():
    rng = np.random.default_rng(3)
    from gf_orb_slam_amd import synth
    for _ in range(20):
        T0 = synth.look_pose(rng, 0.5, 20)
        T1 = synth.look_pose(rng, 0.5, 20)
        Twc1 = np.linalg.inv(T1.astype(np.float64)).astype(np.float32)
        ob = _obs()
        ob.updatePWLSVec(1.0, T0, 1.05, Twc1)
        np.testing.assert_array_equal(ob.Xv, O.obs_update(1.0, T0, 1.05, Twc1))
