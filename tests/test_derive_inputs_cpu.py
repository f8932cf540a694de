"""Host side of the device derivation (physics.derive_inputs -> ryd_derive): every golden
configuration maps onto a descriptor + input block without a GPU, with the same protocol
key and validation as the host derivation; array arguments become input rows, scalars
descriptor values, None the NaN 'not given' marker.  The device results themselves are
checked against physics.derive_batch in tests/test_gpu_derive.py."""
import warnings

import numpy as np
import pytest

from golden_configs import simulate_kwargs, simulation_inputs
from noisyquantumsimulator_amd import _native as N
from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import physics as PH
from noisyquantumsimulator_amd import sweeps as SW


def test_golden_configurations_map(physics_golden):
    warnings.simplefilter("ignore")
    n = 0
    for e in physics_golden:
        cfg = e["config"]
        si, kw = simulation_inputs(cfg), simulate_kwargs(cfg)
        try:
            b = PH.derive_batch(si, **kw)
        except (TypeError, ValueError) as exc:
            with pytest.raises(type(exc)):
                PH.derive_inputs(si, **kw)
            continue
        inp = PH.derive_inputs(si, n=b.n, **kw)
        assert inp.protocol == E.protocol_key(b) and inp.dim == b.dim and inp.cols.shape == (0, 1)
        assert all(c == -1 for c in inp.desc.col)
        assert inp.desc.value[N.DV["DELTA_E"]] == si.excitation.Delta_e
        if b.protocol == "jandura_pupillo":
            nseg = b.bangbang_phases.shape[1]
            assert inp.desc.bb_nseg == nseg
            ph = [inp.desc.value[N.DV["BB_PHI0"] + k] for k in range(nseg)]
            np.testing.assert_array_equal(ph, b.bangbang_phases[0])
        n += 1
    assert n >= 50


def test_c4_inputs_carry_three_columns():
    inp = SW.species_temperature_power_inputs(point_slice=slice(499_990, 500_010))
    assert inp.cols.shape == (3, 20)
    sp, T, P = SW.c4_columns(point_slice=slice(499_990, 500_010))
    rows = {f: inp.desc.col[N.DV[f]] for f in ("SPECIES", "TEMPERATURE", "TW_POWER")}
    np.testing.assert_array_equal(inp.cols[rows["SPECIES"]], sp)
    np.testing.assert_array_equal(inp.cols[rows["TEMPERATURE"]], T)
    np.testing.assert_array_equal(inp.cols[rows["TW_POWER"]], P)
    assert set(inp.cols[rows["SPECIES"]]) == {0.0, 1.0}
    assert np.isnan(inp.desc.value[N.DV["TW_WL_NM"]]) and np.isnan(inp.desc.value[N.DV["BG_LOSS"]])
    assert inp.desc.flags & N.DV_FLAG["NOISE"] and inp.desc.flags & N.DV_FLAG["TRAP_ON"]


def test_species_by_name_and_by_index_agree():
    si = SW.CF.LPSimulationInputs(excitation=SW.medium_excitation())
    a = PH.derive_inputs(si, species=np.array(["Cs133", "Rb87", "Cs133"]))
    b = PH.derive_inputs(si, species=np.array([1, 0, 1]))
    np.testing.assert_array_equal(a.cols, b.cols)
    with pytest.raises(ValueError):
        PH.derive_inputs(si, species=np.array([0, 4]))
    with pytest.raises(ValueError):
        PH.derive_inputs(si, species="K39")
