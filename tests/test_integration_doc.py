"""INTEGRATION.md is executable: the Option A import block runs against the package,
and the Option B ctypes stub binds the in-tree libryd_engine.so (symbols and struct
layout; no compute -- ryd_create just reports that this container has no GPU)."""
import ctypes
import os
import re

import pytest

from noisyquantumsimulator_amd import _native as N

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _blocks():
    with open(os.path.join(REPO, "INTEGRATION.md")) as f:
        return re.findall(r"```python\n(.*?)```", f.read(), re.S)


def test_option_a_import_block():
    block = _blocks()[0]
    after = block.split("# after", 1)[1]
    ns = {}
    exec(compile(after, "INTEGRATION.md:option-A", "exec"), ns)
    for name in ("simulate_CZ_gate", "LPSimulationInputs", "SmoothJPSimulationInputs", "JPSimulationInputs",
                 "TwoPhotonExcitationConfig", "LaserParameters", "NoiseSourceConfig"):
        assert name in ns, name
    import noisyquantumsimulator_amd as pkg
    for name in pkg.__all__:
        assert hasattr(pkg, name), name


def test_option_b_stub_binds_the_library():
    if not os.path.exists(N.LIB_PATH):
        pytest.skip("libryd_engine.so not built")
    stub = next(b for b in _blocks() if "ctypes stub" in b)
    stub = stub.replace('ctypes.CDLL("libryd_engine.so")', f'ctypes.CDLL({N.LIB_PATH!r})')
    ns = {}
    exec(compile(stub, "INTEGRATION.md:option-B", "exec"), ns)
    assert ctypes.sizeof(ns["_Desc"]) == ctypes.sizeof(N.BatchDesc)
    for (fa, ta), (fb, tb) in zip(ns["_Desc"]._fields_, N.BatchDesc._fields_):
        assert fa == fb and ctypes.sizeof(ta) == ctypes.sizeof(tb)
        assert getattr(ns["_Desc"], fa).offset == getattr(N.BatchDesc, fb).offset
    assert callable(ns["lp_square_rho"])
    assert ns["_lib"].ryd_abi_version() == N.RYD_ABI_VERSION
