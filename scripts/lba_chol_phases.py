"""k_ba_solve Cholesky phase split (diagnostic; a BA_CHOL_PHASES build via GF_LIB):
s_memtime cycles of the diagonal + panel part and of the trailing-update part,
summed over the block steps of the last trial of one config-4 solve."""
import ctypes, sys
sys.path.insert(0, '.')
import numpy as np, torch
from gf_orb_slam_amd.optimizer import LocalBAPlan
from gf_orb_slam_amd.synth import synth_lba_problem
from gf_orb_slam_amd._lib import lib, check
plan = LocalBAPlan([synth_lba_problem(100, 20, 3000)])
st = torch.zeros(8, dtype=torch.int64, device='cuda')
lib().gf_ba_plan_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
check(lib().gf_ba_plan_debug_stamps(plan.handle, ctypes.c_void_p(st.data_ptr())))
plan.solve()
t = st.cpu().numpy().astype(np.float64)
chol_us = (t[2] - t[1]) / 100.0
a, b = t[5], t[6]
print("cholesky %.1f us: diagonal+panel %d cycles (%.0f%%), trailing %d cycles (%.0f%%)" % (chol_us, a, 100 * a / (a + b), b, 100 * b / (a + b)))
