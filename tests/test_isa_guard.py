"""A code-generation guard for k_active_match (CPU: hipcc -S, no GPU).

Round 6 traced the active matcher's layout-dependent parity break
(config2_active, `rng differs` at step 4 when the level sigma^2 came from an
LDS copy) to the compiler: under the kernel's register pressure, copies of
live-through values (spill copies of the wave's rand()-call counter to
AGPRs) were placed in a join block *before* that block's exec restore
(`s_or_b64 exec, exec, ...`), so they ran under the mask of the branch that
had just ended, and lanes outside it kept a stale counter: the RNG ring
index of the write-back then differed by lane. The kernel was
changed so that no such copy remains (the wide sorted-live-set loops off,
the recurrence row read from its table, the wave counters pinned to scalar
registers); this test compiles the product source and the LDS-sigma^2
variant that used to fail, and checks that no copy-type instruction
(v_mov, v_accvgpr_*) precedes an exec restore in any join block of the two
active-matching kernels."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wno-unused-function", "--cuda-device-only", "-S"]
COPY = ("v_mov_b32", "v_mov_b64", "v_accvgpr_write", "v_accvgpr_read", "v_accvgpr_mov")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("variant", [[], ["-DAM_LSIG"]], ids=["product", "lds_sigma2"])
def test_no_copy_before_exec_restore(tmp_path, variant):
    import isa_exec_check

    out = tmp_path / "gf.s"
    r = subprocess.run([HIPCC] + FLAGS + variant + [os.path.join(ROOT, "gf_orb_slam_amd", "csrc", "gf.hip"),
                                                    "-o", str(out)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    res = isa_exec_check.scan(str(out))
    kernels = [k for k in res if "k_active_match" in k]
    bad = {k: [b for b in res[k] if any(i.startswith(COPY) for i in b)] for k in kernels}
    assert not any(bad.values()), {k: v[:3] for k, v in bad.items() if v}
