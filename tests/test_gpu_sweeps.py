"""The research_parameter_sweeps driver on the GPU engine against the oracle
(examples/research_parameter_sweeps.py:81-195): a 5-value temperature sweep, one
engine call per protocol; a Delta_e=None row is NaN, not an exception."""
import warnings

import numpy as np
import pytest
import scipy.linalg as sla

from noisyquantumsimulator_amd import _native as N
from noisyquantumsimulator_amd import physics as PH
from noisyquantumsimulator_amd import research_sweeps as RS
from noisyquantumsimulator_amd import simulation as SIM
from oracle import lindblad_oracle as O
from oracle_evaluator import point_spec

pytestmark = pytest.mark.gpu


def test_temperature_sweep_against_oracle():
    warnings.simplefilter("ignore")
    temps = np.array([5, 10, 20, 40, 80]) * 1e-6
    r = RS.run_sweep("temperature", temps, verbose=False)
    assert np.all(np.isfinite(r.fidelities_lp)) and np.all(np.isfinite(r.fidelities_jp))
    for proto, F, T, VO, ST in (("levine_pichler", r.fidelities_lp, r.gate_times_lp, r.v_over_omega_lp, r.status_lp),
                                ("jandura_pupillo", r.fidelities_jp, r.gate_times_jp, r.v_over_omega_jp, r.status_jp)):
        for i, t in enumerate(temps):
            row = dict(RS.DEFAULT_PARAMS, temperature=t)
            si = RS._inputs(proto, row)
            b = PH.derive_batch(si, 1, species="Rb87", n_rydberg=70, temperature=t, spacing_factor=1.5,
                                tweezer_power=10e-3, tweezer_waist=1e-6, B_field=0.0, NA=0.5)
            assert T[i] == pytest.approx(b["tau_total"][0] * 1e6, rel=1e-12)
            assert VO[i] == pytest.approx(b["V_over_Omega"][0], rel=1e-12)
            res = {k: O.snap_structural_zeros(v) for k, v in O.run_point(point_spec(b, 0)).items()}
            # the engine's one-rho-at-a-time probes with the sweep's probe count
            unstable, _ = O.gauge_unstable(res, copies=RS.SWEEP_GAUGE_COPIES)
            fid, avg, info = O.cz_fidelity(res, eigh=lambda m: sla.eigh(m))
            assert bool(ST[i] & N.STATUS_GAUGE_UNSTABLE) == unstable, (proto, t)
            if not unstable:
                assert F[i] == pytest.approx(avg, abs=1e-8)
            # gauge-invariant part through the same engine path
            br = SIM.simulate_CZ_gate_batch(si, 1, species="Rb87", n_rydberg=70, temperature=t, spacing_factor=1.5,
                                            tweezer_power=10e-3, tweezer_waist=1e-6, B_field=0.0, NA=0.5)
            pops = [np.real(res[lab][O.initial_kets()[lab].argmax(), O.initial_kets()[lab].argmax()])
                    for lab in O.LABELS]
            np.testing.assert_allclose(br.populations[0], pops, atol=1e-10)
            assert br.avg_fidelity[0] == F[i]


def test_delta_e_none_row_is_nan():
    warnings.simplefilter("ignore")
    r = RS.run_sweep("Delta_e", [2 * np.pi * 1e9, None, 2 * np.pi * 5e9], verbose=False)
    assert np.isnan(r.fidelities_lp[1]) and np.isnan(r.fidelities_jp[1]) and r.noise_breakdowns_lp[1] == {}
    assert np.all(np.isfinite(r.fidelities_lp[[0, 2]])) and np.all(np.isfinite(r.fidelities_jp[[0, 2]]))
    assert r.noise_breakdowns_jp[0]["n_collapse_ops"] == 14
