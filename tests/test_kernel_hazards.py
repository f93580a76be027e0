"""CPU-side disassembly check of the inline-asm launch-epoch add (scripts/check_epoch_hazard.py): nothing may touch
the atomic's destination VGPRs before the s_waitcnt vmcnt(0) that gran_epoch_wait places (csrc/mlp/granule.h)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import check_epoch_hazard as ceh  # noqa: E402

FAKE = """
0000000000001000 <good_kernel>:
    global_atomic_add_x2 v[2:3], v0, v[4:5], s[0:1] sc0
    v_mov_b32 v6, 0
    s_waitcnt vmcnt(0)
    v_mov_b32 v7, v2
    s_endpgm
0000000000002000 <bad_kernel>:
    global_atomic_add_x2 v[2:3], v0, v[4:5], s[0:1] sc0
    v_accvgpr_write_b32 a0, v3
    s_waitcnt vmcnt(0)
    s_endpgm
"""


def test_checker_flags_an_early_read_and_passes_a_clean_kernel():
    n, bad = ceh.check(FAKE)
    assert n == 2
    assert len(bad) == 1 and bad[0].startswith("bad_kernel") and "('v', 3)" in bad[0]


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="hipcc not installed")
@pytest.mark.timeout(600)
def test_epoch_add_results_untouched_before_their_wait():
    assert ceh.main([]) == 0
