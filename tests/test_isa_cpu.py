"""Static ISA check of the default training-path attention kernels (cross-compiled for gfx950 here, no GPU).

A `s_waitcnt vmcnt(N)` right before an MFMA in these kernels means the compiler could not prove that
operands loaded before the main loop had retired, and so drains the loop's own prefetch loads ahead of
MFMAs every iteration (found and fixed in the text dK/dV kernel, round 4; scripts/isa_vmcnt_check.py).
"""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not available")
def test_attention_kernels_have_no_vmcnt_wait_ahead_of_mfma():
    from isa_vmcnt_check import check

    res = {name: hits for hits, _, name in check(os.path.join(ROOT, "csrc", "kernels", "attention.hip"))}
    defaults = [n for n in res if ("attn_bwd_dkdv_text_kernelILi2ELi4E" in n or "attn_bwd_dq_kernelILi3ELb1ELb0EE" in n
                                   or "attn_fwd_kernelILi3ELb0ELi2E" in n)]
    assert len(defaults) == 3, sorted(res)
    assert all(res[n] == 0 for n in defaults), {n: res[n] for n in defaults}
