"""CPU-side checks of the C-ABI library: it loads and exports every symbol
include/ryd_engine.h declares, with matching layout constants.  No compute."""
import ctypes
import os
import re

import pytest

from noisyquantumsimulator_amd import _native as N

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header():
    with open(os.path.join(REPO, "include", "ryd_engine.h")) as f:
        return f.read()


def test_header_declares_exported_symbols():
    decl = set(re.findall(r"\b(ryd_[a-z0-9_]+)\s*\(", _header()))
    assert decl == set(N.EXPORTED)


def test_header_constants_match_binding():
    h = _header()
    defs = dict(re.findall(r"#define\s+(RYD_[A-Z0-9_]+)\s+(-?\d+)u?", h))
    for k, v in N.P.items():
        assert int(defs["RYD_P_" + k]) == v
    for k, v in N.S.items():
        assert int(defs["RYD_S_" + k]) == v
    assert int(defs["RYD_NPARAM"]) == N.NPARAM and int(defs["RYD_NSUMMARY"]) == N.NSUMMARY
    for k, v in N.C.items():
        assert int(defs["RYD_C_" + k]) == v
    assert int(defs["RYD_NCOH"]) == N.NCOH
    for k, v in N.PROTO.items():
        assert int(defs["RYD_PROTO_" + k.upper()]) == v
    assert ctypes.sizeof(N.BatchDesc) == 56 and ctypes.sizeof(N.Stats) == 48
    for k, v in N.T.items():
        assert int(defs["RYD_T_" + k]) == v
    for k, v in N.TS.items():
        assert int(defs["RYD_TS_" + k]) == v
    assert int(defs["RYD_T_NSUMMARY"]) == N.T_NSUMMARY
    assert int(defs["RYD_ABI_VERSION"]) == N.RYD_ABI_VERSION
    assert ctypes.sizeof(N.TrajDesc) == 472
    assert int(defs["RYD_T_FLAG_ROWS"]) == N.T_FLAG["rows"] and int(defs["RYD_T_FLAG_LANES"]) == N.T_FLAG["lanes"]
    for k, v in N.DV.items():
        assert int(defs["RYD_DV_" + k]) == v
    assert int(defs["RYD_DV_NFIELD"]) == N.DV_NFIELD and int(defs["RYD_DV_NSPC"]) == N.DV_NSPC
    assert int(defs["RYD_DV_MAX_SPECIES"]) == N.DV_MAX_SPECIES and len(N.DV_SPC) == N.DV_NSPC
    for k, v in N.DV_FLAG.items():
        assert int(defs["RYD_DV_" + k]) == v
    for k, v in N.DV_LEAK.items():
        assert int(defs["RYD_DV_LEAK_" + k.upper()]) == v
    assert int(defs["RYD_DV_LEAK_OTHER"]) == N.DV_LEAK_OTHER
    diag = {k: int(v) for k, v in defs.items() if k.startswith("RYD_DV_D_")}
    assert sorted(diag.values()) == list(range(N.DV_NDIAG)) and int(defs["RYD_DV_NDIAG"]) == N.DV_NDIAG
    # 8 int32 + 4 + 2 doubles + the species table + values + columns
    assert ctypes.sizeof(N.DeriveDesc) == 32 + 48 + 8 * 24 * 4 + 8 * 38 + 4 * 38 + 0


def test_library_loads_and_exports():
    if not os.path.exists(N.LIB_PATH):
        pytest.skip("libryd_engine.so not built (run make / __graft_entry__.build())")
    lib = N.load()
    for sym in N.EXPORTED:
        assert hasattr(lib, sym), sym
    assert lib.ryd_abi_version() == N.RYD_ABI_VERSION == 5
    assert lib.ryd_param_count() == N.NPARAM
    assert lib.ryd_summary_width() == N.NSUMMARY
    assert lib.ryd_state_width(0, 3) == 25 and lib.ryd_state_width(1, 3) == 18
    assert lib.ryd_state_width(0, 4) == 36 and lib.ryd_state_width(1, 4) == 32
    assert lib.ryd_state_width(0, 5) == -1


def test_evolve_generic_validates_before_any_gpu_call():
    """ryd_evolve_generic rejects a NULL handle and bad sizes without touching a device."""
    lib = N.load()
    assert lib.ryd_evolve_generic(None, 9, 1, 0, 1, 1, None, None, None, None, None, None) == -1   # RYD_ERR_INVALID
