"""k_ba_solve phase timing (diagnostic): stamps of the last trial of one config-4 solve."""
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
print("k_ba_solve phases (us): assemble %.1f  cholesky %.1f  trsv %.1f  tail %.1f" % tuple(np.diff(t[:5]) / 100.0))
print("trsv core cycles %d over %.1f us -> %.2f GHz" % (t[6] - t[5], (t[3] - t[2]) / 100.0, (t[6] - t[5]) / ((t[3] - t[2]) * 10.0)))
