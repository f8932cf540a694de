"""Per-point warning bits (include/ryd_engine.h RYD_STATUS_WEAK_BLOCKADE, _DARK_STATE_SIGN,
_OMEGA_RANGE): the reference's UserWarnings, evaluated point by point by the host
derivation (RG/protocols.py:615-619, RG/simulation.py:1631-1676, :2930-2946)."""
import warnings

import numpy as np

from noisyquantumsimulator_amd import _native as N
from noisyquantumsimulator_amd import configurations as CF
from noisyquantumsimulator_amd import physics as PH

KW = dict(species="Rb87", n_rydberg=70, tweezer_power=0.020, tweezer_waist=0.8e-6, temperature=2e-6,
          B_field=1e-4, NA=0.5)


def _exc(p2=0.3, Delta_e=2 * np.pi * 1e9):
    return CF.TwoPhotonExcitationConfig(
        laser_1=CF.LaserParameters(power=50e-6, waist=50e-6, polarization="pi"),
        laser_2=CF.LaserParameters(power=p2, waist=50e-6, polarization="sigma+"), Delta_e=Delta_e)


def test_weak_blockade_bit_straddles_v_over_omega_10_for_lp():
    warnings.simplefilter("ignore")
    sf = np.linspace(2.0, 9.0, 57)                        # V/Omega from ~1e3 down through 10
    b = PH.derive_batch(CF.LPSimulationInputs(excitation=_exc()), n=sf.size, spacing_factor=sf, **KW)
    vo = b["V_over_Omega"]
    assert vo.min() < 10 < vo.max()
    got = (b.status_bits & N.STATUS_WEAK_BLOCKADE) != 0
    np.testing.assert_array_equal(got, vo < 10)
    assert "weak_blockade" in b.warnings


def test_weak_blockade_threshold_is_5_for_smooth_jp():
    warnings.simplefilter("ignore")
    sf = np.linspace(2.0, 12.0, 61)
    b = PH.derive_batch(CF.SmoothJPSimulationInputs(excitation=_exc()), n=sf.size, spacing_factor=sf, **KW)
    vo = b["V_over_Omega"]
    assert vo.min() < 5 < vo.max()
    np.testing.assert_array_equal((b.status_bits & N.STATUS_WEAK_BLOCKADE) != 0, vo < 5)
    # bang-bang has no blockade warning in the reference
    bb = PH.derive_batch(CF.JPSimulationInputs(excitation=_exc()), n=sf.size, spacing_factor=sf, **KW)
    assert not np.any(bb.status_bits & N.STATUS_WEAK_BLOCKADE)


def test_omega_range_bit():
    warnings.simplefilter("ignore")
    p2 = np.array([1e-9, 1e-6, 0.3, 50.0, 5e4])          # Omega from far below 0.1 MHz to above 100 MHz
    b = PH.derive_batch(CF.LPSimulationInputs(excitation=_exc()), n=p2.size,
                        overrides=dict(laser_2_power=p2), **KW)
    om = b["Omega"] / (2 * np.pi)
    want = (om > 100e6) | (om < 0.1e6)
    assert want.any() and not want.all()
    np.testing.assert_array_equal((b.status_bits & N.STATUS_OMEGA_RANGE) != 0, want)


def test_dark_state_sign_bit():
    warnings.simplefilter("ignore")
    # the reference forces delta/Omega opposite to sign(Delta_e): never flagged through
    # simulate_CZ_gate ...
    for de in (2 * np.pi * 1e9, -2 * np.pi * 1e9):
        b = PH.derive_batch(CF.SmoothJPSimulationInputs(excitation=_exc(Delta_e=de)), **KW)
        assert not np.any(b.status_bits & N.STATUS_DARK_STATE_SIGN)
    # ... but an explicit signed value with the wrong sign is (evolve_smooth_sinusoidal_jp check)
    sd = np.array([-0.02, 0.0, 0.02])
    b = PH.derive_batch(CF.SmoothJPSimulationInputs(excitation=_exc()), n=3,
                        overrides=dict(smooth_delta_over_omega=sd), **KW)
    np.testing.assert_array_equal((b.status_bits & N.STATUS_DARK_STATE_SIGN) != 0, [False, False, True])
