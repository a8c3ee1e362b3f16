import sys
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import numpy as np, torch
rng = np.random.default_rng(0)
a = rng.normal(size=100000) * 1e3; b = rng.normal(size=100000) * 7 + 0.1
ga, gb = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
print("div mismatches", int(((ga / gb).cpu().numpy() != a / b).sum()))
print("sqrt mismatches", int((torch.sqrt(ga.abs()).cpu().numpy() != np.sqrt(np.abs(a))).sum()))
from gf_orb_slam_amd import synth
from gf_orb_slam_amd.observability import Observability, ObsCamera
import oracle_lib as O
sc = synth.synth_scene("euroc", 3000, 10, 21)
cam = ObsCamera.from_intrinsics(457.3, 457.3, 367.215, 248.375, 752, 480, bound=75)
ob = Observability(cam)
T = sc["Tcw"]
ob.updatePWLSVec(0.0, T, 0.05, np.linalg.inv(T.astype(np.float64)).astype(np.float32))
ob.predictPWLSVec(0.05, 2)
Hg, Ig, Ug, Vg = ob.build_info(sc["map"]["pos"], None, False, kine_idx=1)
Ho, Io, Uo, Vo = O.obs_build_info(cam, np.array(ob.kinematic[1].Xv[:]), sc["map"]["pos"], None, False)
print("H mismatch", int((Hg != Ho).sum()), "max rel", float(np.max(np.abs(Hg - Ho) / (np.abs(Ho) + 1e-300))))
print("uv mismatch", int((Ug != Uo).sum()))
i = int(np.nonzero((Ug != Uo).any(1))[0][0])
print("example", i, Ug[i], Uo[i], Hg[i][:3], Ho[i][:3])
