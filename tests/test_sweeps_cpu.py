"""Host logic of the research_parameter_sweeps driver (no GPU): the rows a batch gets,
the reference's defaults and quirks, NaN rows where the reference raises."""
import numpy as np
import pytest

from noisyquantumsimulator_amd import research_sweeps as RS
from noisyquantumsimulator_amd import simulation as SIM


class _Fake:
    """Stands in for simulate_CZ_gate_batch: records the calls, returns a result whose
    avg fidelity encodes the point index."""
    def __init__(self):
        self.calls = []

    def __call__(self, si, n, include_noise=True, overrides=None, devices=None, gauge_copies=None, **kw):
        from noisyquantumsimulator_amd import physics as PH
        self.calls.append(dict(si=si, n=n, include_noise=include_noise, overrides=overrides, kw=kw,
                               gauge_copies=gauge_copies))
        b = PH.derive_batch(si, n, include_noise=include_noise, overrides=overrides, **kw)
        F = np.tile(np.arange(n, dtype=float)[:, None] / 100, (1, 4))
        return SIM.BatchResult(batch=b, avg_fidelity=F.mean(1), fidelities=F, populations=F,
                               controlled_phase=np.zeros(n), cz_phase_fidelity=np.ones(n),
                               status=np.zeros(n, np.uint32), is_mixed=np.ones(n, bool))


def test_defaults_quirks_and_nan_rows(monkeypatch):
    fake = _Fake()
    monkeypatch.setattr(SIM, "simulate_CZ_gate_batch", fake)
    vals = [2 * np.pi * 1e9, None, 2 * np.pi * 5e9]
    r = RS.run_sweep("Delta_e", vals, verbose=False)
    # Delta_e = None raises TypeError in the reference (two_photon_rabi) -> NaN row, {}
    assert np.isnan(r.fidelities_lp[1]) and np.isnan(r.fidelities_jp[1])
    assert np.isnan(r.gate_times_lp[1]) and r.noise_breakdowns_lp[1] == {} and r.noise_breakdowns_jp[1] == {}
    assert np.all(np.isfinite(r.fidelities_lp[[0, 2]])) and np.all(np.isfinite(r.gate_times_jp[[0, 2]]))
    assert len(fake.calls) == 2                     # one batch per protocol
    lp, jp = fake.calls
    assert lp["gauge_copies"] == RS.SWEEP_GAUGE_COPIES == 4    # fewer gauge probes
    assert lp["n"] == 2 and type(lp["si"]).__name__ == "LPSimulationInputs" and lp["si"].pulse_shape == "square"
    assert type(jp["si"]).__name__ == "JPSimulationInputs"
    np.testing.assert_allclose(lp["overrides"]["Delta_e"], [2 * np.pi * 1e9, 2 * np.pi * 5e9])
    # run_single_simulation's fixed inputs: laser waists 1 um / 10 um, DEFAULT_PARAMS
    ex = lp["si"].excitation
    assert ex.laser_1.waist == 1e-6 and ex.laser_2.waist == 10e-6
    assert lp["si"].noise.include_motional_dephasing
    np.testing.assert_array_equal(lp["overrides"]["laser_1_power"], [2.5e-3] * 2)
    np.testing.assert_array_equal(lp["overrides"]["laser_2_power"], [1.0] * 2)
    np.testing.assert_array_equal(lp["overrides"]["laser_1_linewidth_hz"], [100.0] * 2)
    kw = lp["kw"]
    assert list(kw["species"]) == ["Rb87"] * 2 and np.all(kw["spacing_factor"] == 1.5)
    assert np.all(kw["B_field"] == 0.0) and np.all(kw["temperature"] == 20e-6)
    assert np.all(kw["tweezer_power"] == 10e-3) and np.all(kw["tweezer_waist"] == 1e-6)


def test_bad_pulse_shape_is_nan_for_lp_only(monkeypatch):
    monkeypatch.setattr(SIM, "simulate_CZ_gate_batch", _Fake())
    r = RS.run_sweep("pulse_shape", ["square", "time_optimal", "drag", "cosine"], verbose=False)
    assert np.isfinite(r.fidelities_lp[[0, 3]]).all() and np.isnan(r.fidelities_lp[[1, 2]]).all()
    assert np.isfinite(r.fidelities_jp).all()          # JP ignores pulse_shape


def test_species_and_fixed_kwargs_batch(monkeypatch):
    fake = _Fake()
    monkeypatch.setattr(SIM, "simulate_CZ_gate_batch", fake)
    RS.run_sweep("temperature", np.array([10, 20]) * 1e-6, verbose=False, species="Cs133", n_rydberg=60)
    kw = fake.calls[0]["kw"]
    assert list(kw["species"]) == ["Cs133"] * 2 and np.all(kw["n_rydberg"] == 60)
    np.testing.assert_allclose(kw["temperature"], [10e-6, 20e-6])


def test_run_single_simulation_returns_none_on_reference_errors(capsys):
    assert RS.run_single_simulation("levine_pichler", Delta_e=None) is None
    assert "simulation failed" in capsys.readouterr().out
