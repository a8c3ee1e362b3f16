"""Step-by-step driver of the batched pose path (debugging aid)."""
import faulthandler
import os
import sys

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import torch

from gf_orb_slam_amd._lib import check, lib, ptr
from gf_orb_slam_amd.optimizer import POSE_EDGE_DTYPE, Optimizer
from gf_orb_slam_amd.orb import default_context
from gf_orb_slam_amd.synth import synth_pose_problem

sizes = [int(s) for s in sys.argv[1].split(",")] if len(sys.argv) > 1 else [7, 64]
stride = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
print("sizes", sizes, "stride", stride, flush=True)
probs = [synth_pose_problem(500 + i, max(n, 1)) for i, n in enumerate(sizes)]
E = np.zeros((len(sizes), stride), POSE_EDGE_DTYPE)
T = np.zeros((len(sizes), 4, 4), np.float32)
for i, (n, (_, T0, edges, cam)) in enumerate(zip(sizes, probs)):
    E[i, :n] = edges[:n]
    T[i] = T0
_, _, fx, fy, cx, cy = probs[0][3]
dev = torch.device("cuda:0")
print("torch alloc", flush=True)
dE = torch.from_numpy(E.view(np.uint8).reshape(-1)).to(dev)
dT = torch.from_numpy(T).to(dev)
dN = torch.tensor(sizes, dtype=torch.int32, device=dev)
dO = torch.zeros(len(sizes) * stride, dtype=torch.uint8, device=dev)
dI = torch.zeros(len(sizes), dtype=torch.int32, device=dev)
dIt = torch.zeros(len(sizes), dtype=torch.int32, device=dev)
torch.cuda.synchronize()
ctx = default_context()
print("ctx", ctx.handle, "stream", hex(ctx.stream), flush=True)
Optimizer.pose_opt_batch_dev(dT, dE, dN, stride, fx, fy, cx, cy, dO, dI, dIt, ctx=ctx)
print("launched", flush=True)
check(lib().gf_ctx_sync(ctx.handle))
print("synced", dI.cpu().numpy(), dIt.cpu().numpy(), flush=True)
