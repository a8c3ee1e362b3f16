"""Extraction alone: B rendered EuRoC frames through gf_orb_extract_batch_dev,
`steps` times on one stream (run it under rocprofv3 --kernel-trace --stats
for per-kernel device times without the bench's other groups).
Usage: python scripts/extract_times.py [B] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from gf_orb_slam_amd import ORBextractor, scene  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
W = scene.Workload("euroc", B, n_scenes=8, period=32, seed=0)
frames = W.render_all("cuda")
frames = frames.reshape(-1, frames.shape[-2], frames.shape[-1])
frames = frames.repeat((B + frames.shape[0] - 1) // frames.shape[0], 1, 1)[:B].contiguous()
ex = ORBextractor(1000, 1.2, 8, 1, 20, max_batch=B)
ex._bind(frames.shape[2], frames.shape[1])
cap = ex.capacity
kps = torch.zeros((B, cap, 28), dtype=torch.int8, device="cuda")
desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    ex.extract_batch_dev(frames, kps, desc, cnt, s)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    ex.extract_batch_dev(frames, kps, desc, cnt, s)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
print(f"B={B} extraction {dt * 1e3:.3f} ms per batch ({B / dt:.0f} frames/s), keypoints/frame {cnt.float().mean().item():.1f}")
