import sys, ctypes
sys.path.insert(0, '.')
import numpy as np, torch
from gf_orb_slam_amd import ORBextractor, synth
from gf_orb_slam_amd._lib import lib
frames = np.stack([synth.synth_frame(752, 480, s) for s in range(3)])
imgs = torch.from_numpy(frames).cuda()
print("strides", imgs.stride(), imgs.is_contiguous(), imgs.dtype, imgs.device)
ex = ORBextractor(1000, 1.2, 8, 1, 20, width=752, height=480, max_batch=3)
print(lib().gf_orb_extract_batch_dev.argtypes)
