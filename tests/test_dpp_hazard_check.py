"""tools/check_dpp_hazards.py (the build-time ISA check of ADVICE r2's inline-asm DPP
hazard) flags a VALU write followed by a DPP read of the same VGPR within 2 wait states,
and accepts the s_nop-separated and unrelated-register forms."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import check_dpp_hazards as H  # noqa: E402

BAD = """kern:
\tv_mov_b32_e32 v21, v40
\tv_fmac_f64_dpp v[10:11], v[20:21], v[30:31] row_newbcast:1 row_mask:0xf bank_mask:0xf
"""
BAD2 = """kern:
\tv_add_f64 v[20:21], v[2:3], v[4:5]
\ts_mov_b32 s0, 0
\tv_fmac_f64_dpp v[10:11], v[20:21], v[30:31] row_newbcast:1 row_mask:0xf bank_mask:0xf
"""
GOOD = """kern:
\tv_add_f64 v[20:21], v[2:3], v[4:5]
\ts_nop 1
\tv_fmac_f64_dpp v[10:11], v[20:21], v[30:31] row_newbcast:1 row_mask:0xf bank_mask:0xf
\tv_fmac_f64_dpp v[12:13], v[20:21], v[10:11] row_newbcast:2 row_mask:0xf bank_mask:0xf
"""


def _run(tmp_path, text):
    p = tmp_path / "k.s"
    p.write_text(text)
    return H.check(str(p))


def test_hazard_checker(tmp_path):
    assert len(_run(tmp_path, BAD)) == 1
    assert len(_run(tmp_path, BAD2)) == 1
    # the second DPP reads v[20:21] as src0 and v[10:11] (just written) only as src1: fine
    assert _run(tmp_path, GOOD) == []
