import sys, ctypes, numpy as np, torch
sys.path.insert(0, '.')
from gf_orb_slam_amd._lib import lib
from gf_orb_slam_amd import synth
from gf_orb_slam_amd.pipeline import FrontEnd
B=64
fe = FrontEnd("euroc", 1000, B, 2000, seed=0)
w,h=fe.cam[:2]
fr=np.stack([synth.synth_frame(w,h,synth.frame_seed(b,0)) for b in range(8)])
fe.load_frames(fr[np.arange(B)%8]); fe.build_maps()
buf = torch.zeros(B*8, dtype=torch.int64, device='cuda')
l = lib(); l.gf_debug_active_timers.argtypes=[ctypes.c_void_p]
for i in range(3): fe.step()
fe.sync()
l.gf_debug_active_timers(ctypes.c_void_p(buf.data_ptr()))
fe.step(); fe.sync()
t = buf.cpu().numpy().reshape(B,8)
print("mean ticks [grid, draws, logdet, top, onepoint, removal, total, ntops]:", t.mean(0)); print("max total", t[:,6].max(), "min", t[:,6].min())
print("ntm", fe.num_to_match.cpu().numpy()[:8], "nactive", fe.n_active.cpu().numpy()[:8])
