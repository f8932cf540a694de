"""Pin the CPU oracle (oracle/lindblad_oracle.py) before trusting it.

* every published number of the reference notebooks
* the closed-form decay known-answer test (scripts/archive/test_mesolve_direct.py:34-51)
* the QuTiP-like ZVODE integrator agrees with the exact propagator
"""
import numpy as np
import pytest

from conftest import states_from_fixture
from oracle import lindblad_oracle as O


def _check_published(name, got, published):
    for key, (val, digits) in published.items():
        if key not in got:
            continue
        assert round(got[key], digits) == pytest.approx(val, abs=0.51 * 10 ** (-digits)), (name, key)


@pytest.mark.parametrize("name", ["lp_medium_nf", "smooth_medium_nf", "lp_high_nf", "lp_low_nf",
                                  "smooth_high_nf", "smooth_low_nf"])
def test_published_fidelities(evolution_golden, name):
    e = evolution_golden[name]
    fid, avg, info = O.cz_fidelity(states_from_fixture(e))
    d = e["derived"]
    got = dict(avg=avg, F11=fid["11"], cz_phase_fidelity=info["cz_phase_fidelity"],
               phase_error_deg=info["phase_error_from_pi_deg"],
               controlled_phase_deg=abs(info["controlled_phase_deg"]),
               gate_time_us=d["tau_total"] * 1e6, V_over_Omega=d["V_over_Omega"],
               Omega_MHz=d["Omega"] / (2 * np.pi * 1e6))
    _check_published(name, got, e["published"])


def test_published_row5(evolution_golden):
    e = evolution_golden["lp_row5_physics"]
    st = states_from_fixture(e)
    idx = {k: int(np.argmax(np.abs(v))) for k, v in O.initial_kets().items()}
    pops = {k: abs(st[k][idx[k]]) ** 2 for k in O.LABELS}
    got = dict(F00=pops["00"], F01=pops["01"], F10=pops["10"], F11=pops["11"],
               avg_no_penalty=float(np.mean(list(pops.values()))),
               phi_01_deg=float(np.degrees(np.angle(st["01"][idx["01"]]))))
    _check_published("row5", got, e["published"])


def test_oracle_reproduces_fixture_states(evolution_golden):
    """Re-run the (fast) LP square fixtures through the oracle."""
    e = evolution_golden["lp_medium_noisy"]
    d = e["derived"]
    cops = O.collapse_operators(d)
    assert len(cops) == 14    # the reference's default c_op count
    p = O.PointSpec(protocol="lp_square", Omega=d["Omega"], V=d["V"], Delta=d["Delta_gate"],
                    tau=d["tau_single"], xi=complex(d["xi_re"], d["xi_im"]),
                    delta_zeeman=d["delta_zeeman"], delta_stark=d["delta_stark"], c_ops=cops)
    res = O.run_point(p)
    ref = states_from_fixture(e)
    for k in O.LABELS:
        np.testing.assert_allclose(res[k], ref[k], atol=1e-12)


def test_decay_known_answer():
    g = 1.0 / 140e-6
    t = np.linspace(0, 50e-6, 6)
    np.testing.assert_allclose(O.decay_kat(g, t), np.exp(-g * t), rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(O.decay_kat(g, t[1:], method="zvode"), np.exp(-g * t[1:]), rtol=1e-7)


def test_zvode_matches_expm_lp(evolution_golden):
    """QuTiP-like Adams/ZVODE vs exact propagator: populations agree to ~1e-8
    (the reference tolerance), the whole rho to ~1e-6 (SURVEY.md hard part 1)."""
    e = evolution_golden["lp_medium_noisy"]
    d = e["derived"]
    p = O.PointSpec(protocol="lp_square", Omega=d["Omega"], V=d["V"], Delta=d["Delta_gate"],
                    tau=d["tau_single"], xi=complex(d["xi_re"], d["xi_im"]),
                    delta_zeeman=d["delta_zeeman"], delta_stark=d["delta_stark"],
                    c_ops=O.collapse_operators(d))
    zv = O.run_point(p, method="zvode")
    ex = states_from_fixture(e)
    for k in O.LABELS:
        i = int(np.argmax(np.abs(O.initial_kets()[k])))
        assert abs(zv[k][i, i] - ex[k][i, i]) < 1e-7
        assert np.abs(zv[k] - ex[k]).max() < 1e-5


def test_ket_rho_split():
    """No c_ops -> kets (pure branch); c_ops -> rho (scripts/archive/test_mesolve.py:17-31)."""
    H = O.two_atom_hamiltonian(2 * np.pi * 1e6, 0.0, 2 * np.pi * 50e6)
    psi = O.initial_kets()["11"]
    assert O.evolve_state(H, psi, np.array([0, 1e-7])).ndim == 1
    c = O.collapse_operators({"gamma_r": 1e4})
    assert O.evolve_state(H, psi, np.array([0, 1e-7]), c).ndim == 2
