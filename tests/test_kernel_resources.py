"""Register budget of the hand-written kernels (CPU: hipcc cross-compiles gfx950 here).

A spilled persistent kernel runs far slower, and a harmless-looking source edit can tip one
over: round 5's (reverted) compile-time removal of the timing-only knob branches let hipcc
re-schedule the config-5 BPTT (rnnrs_bwd_kernel<1, 12, 6, *>) into 70-112 spilled VGPRs,
22.2 -> 27.2 ms/step, which no functional test noticed. Every kernel that spills must be on
the allowlist below (diagnostic stamp builds and variants no default plan launches)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="needs hipcc")

# mangled-name prefixes allowed to spill (measured in round 4, unchanged since)
ALLOWED = {
    "rnn_xcd.hip": ("_ZN12_GLOBAL__N_115rnnw_fwd_kernelILi6ELi0ELb1E",      # stamps build
                    "_ZN12_GLOBAL__N_115rnne_fwd_kernelILi4ELi0ELb0ELb1E",  # stamps build
                    "_ZN12_GLOBAL__N_115rnnq_fwd_kernelILi1ELi7ELb1ELi0E",
                    "_ZN12_GLOBAL__N_115rnnq_fwd_kernelILi1ELi8ELb1ELi0E",
                    "_ZN12_GLOBAL__N_115rnnq_fwd_kernelILi1ELi8ELb0ELi0E"),
    "rnn_fp8.hip": None,            # allowlist = whatever spilled in round 4 (2 kernels), by count
    "gemm8.hip": ("_ZN12_GLOBAL__N_112gemm8_kernelILb0ELi1ELi0E",),        # row-col variant, unused
}


@pytest.mark.parametrize("src", ["rnn_xcd.hip", "gemm8.hip", "rnn_fp8.hip"])
def test_no_new_register_spills(src):
    import kernel_resources as KR
    rows = KR.analyse(os.path.join(ROOT, "deepspeech_amd", "csrc", src))
    assert rows, "no kernels found"
    spilled = [r["name"] for r in rows if r.get("VGPRs Spill", 0) or r.get("ScratchSize [bytes/lane]", 0)]
    allowed = ALLOWED[src]
    if allowed is None:
        assert len(spilled) <= 2, spilled
    else:
        bad = [n for n in spilled if not n.startswith(allowed)]
        assert not bad, bad
