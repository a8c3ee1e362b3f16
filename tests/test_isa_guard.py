"""A code-generation guard for every HIP kernel (CPU: hipcc -S, no GPU).

Round 6 traced the active matcher's layout-dependent parity break
(config2_active, `rng differs` at step 4 when the level sigma^2 came from an
LDS copy) to the compiler: under the kernel's register pressure, copies of
live-through values (spill copies to AGPRs of the wave's rand()-call
counter) were placed in a join block -- the target of an `s_cbranch_execz`
that skipped a masked region -- *before* that block's exec restore
(`s_or_b64 exec, exec, ...`). They ran under the mask of the region that had
just ended, so lanes outside it kept a stale counter and the RNG ring index
of the write-back differed by lane. The kernel's branchy loads
were made unconditional and its wave counters scalar; this test compiles
every kernel source (and the LDS-sigma^2 variant that used to fail) and
checks that no such join block holds a vector instruction other than the
EXEC-independent lane reads / writes of SGPR spills. scripts/isa_exec_check.py
flags the failing r05 build's block and nothing else in the library."""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wno-unused-function", "--cuda-device-only", "-S"]
SRCS = sorted(glob.glob(os.path.join(ROOT, "gf_orb_slam_amd", "csrc", "*.hip")))
JOBS = [(os.path.basename(s)[:-4], s, []) for s in SRCS] + \
       [("gf_lds_sigma2", os.path.join(ROOT, "gf_orb_slam_amd", "csrc", "gf.hip"), ["-DAM_LSIG"])]


def _compile(job, d):
    name, src, extra = job
    out = os.path.join(d, name + ".s")
    r = subprocess.run([HIPCC] + FLAGS + extra + [src, "-o", out], capture_output=True, text=True, timeout=900)
    return name, out, r.returncode, r.stderr[-2000:]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_no_masked_copy_before_exec_restore(tmp_path):
    import isa_exec_check

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = list(ex.map(lambda j: _compile(j, str(tmp_path)), JOBS))
    bad = {}
    for name, out, rc, err in res:
        assert rc == 0, f"{name}: {err}"
        for k, blocks in isa_exec_check.scan(out).items():
            bad[f"{name}:{k}"] = blocks[:3]
    assert not bad, bad


def test_scanner_flags_the_r05_pattern(tmp_path):
    """The scanner on a hand-made excerpt of the failing r05 build (gf.hip
    -DAM_LSIG): the join .LBB6_787 of the branch that loaded the live set's
    match flags holds the AGPR copies before its exec restore."""
    import isa_exec_check

    src = tmp_path / "x.s"
    src.write_text("""_ZN12_GLOBAL__N_114k_active_matchENS_10ActiveArgsE:
	v_cmp_lt_i32_e32 vcc, -1, v7
	s_and_saveexec_b64 s[0:1], vcc
	s_cbranch_execz .LBB6_787
; %bb.786:
	ds_read_u16 v4, v4 offset:784
	v_cndmask_b32_e64 v16, 0, 1, vcc
.LBB6_787:
	v_accvgpr_write_b32 a15, v178
	s_movk_i32 s95, 0x7d0
	s_or_b64 exec, exec, s[0:1]
	v_cmp_gt_i32_e32 vcc, s88, v226
	s_and_saveexec_b64 s[2:3], vcc
	s_cbranch_execz .LBB6_790
; %bb.789:
	v_mov_b32_e32 v1, 1
	s_or_b64 exec, exec, s[2:3]
.LBB6_790:
	s_or_saveexec_b64 s[100:101], -1
	v_accvgpr_read_b32 v255, a33
	s_mov_b64 exec, s[100:101]
	v_readlane_b32 s0, v255, 3
	s_or_b64 exec, exec, s[2:3]
	s_endpgm
""")
    res = isa_exec_check.scan(str(src))
    assert list(res.values()) == [[["v_accvgpr_write_b32 a15, v178"]]]
