"""Local BA on the device: wall time per solve for B copies of config 4 (diagnostic)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import numpy as np
from gf_orb_slam_amd.optimizer import LocalBAPlan
from gf_orb_slam_amd.synth import synth_lba_problem
from gf_orb_slam_amd._lib import lib, check
import oracle_lib as O

for B in [int(b) for b in os.environ.get('LBA_BATCHES', '1,8,64').split(',')]:
    probs = [synth_lba_problem(100 + i, 20, 3000) for i in range(B)]
    plan = LocalBAPlan(probs)
    plan.solve()
    t = time.perf_counter(); steps = plan.solve(); dt = time.perf_counter() - t
    res = plan.results()
    its = np.mean([sum(r[3]) for r in res])
    print(f"B={B} wall {dt*1e3:.2f} ms  steps {steps}  mean iterations {its:.1f}  -> {B/dt:.1f} solves/s", flush=True)
    check(lib().gf_prof_enable(plan.ctx.handle, 1)); check(lib().gf_prof_reset(plan.ctx.handle))
    plan.solve()
    import ctypes
    i = 0; name = ctypes.create_string_buffer(64)
    while True:
        ms, cnt = ctypes.c_double(), ctypes.c_int()
        if lib().gf_prof_report(plan.ctx.handle, i, name, 64, ctypes.byref(ms), ctypes.byref(cnt)) != 0: break
        print(f"   {name.value.decode():16s} {ms.value:8.3f} ms  {cnt.value} launches  {ms.value/cnt.value*1e3:8.1f} us avg")
        i += 1
    check(lib().gf_prof_enable(plan.ctx.handle, 0))
    plan.close()
t = time.perf_counter(); O.local_ba(probs[0]); print(f"oracle 1 solve {1e3*(time.perf_counter()-t):.1f} ms")
