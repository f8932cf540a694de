"""C2 (BASELINE configs[1]) on the bench's own grid: sweeps.omega_delta_grid (100 x 100
(Omega, Delta/Omega), LP square, medium apparatus, the full 8-channel noise model).
The whole 10k-point batch runs in one launch; its four corners and centre are checked
against the oracle (expm of the Lindbladian built from the same derived rates,
oracle/lindblad_oracle.py) to 1e-10, and the reference's phase penalty on those points
is either reproduced through ryd_mixed_phase or flagged GAUGE_UNSTABLE."""
import warnings

import numpy as np
import pytest
import scipy.linalg as sla
from threadpoolctl import threadpool_limits

from noisyquantumsimulator_amd import _native as N
from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import simulation as SIM
from noisyquantumsimulator_amd import sweeps as SW
from oracle import lindblad_oracle as O

pytestmark = pytest.mark.gpu

CHECK = (0, 99, 5050, 9900, 9999)     # (Omega, Delta/Omega) corners and centre


def _spec(c, i):
    return O.PointSpec(protocol="lp_square", Omega=c["Omega"][i], V=c["V"][i], Delta=c["Delta_gate"][i],
                       tau=c["tau_single"][i], xi=complex(c["xi_re"][i], c["xi_im"][i]),
                       delta_zeeman=c["delta_zeeman"][i], delta_stark=c["delta_stark"][i],
                       c_ops=O.collapse_operators({k: c[k][i] for k in O.RATE_KEYS}))


def test_c2_grid_corners_match_oracle():
    warnings.simplefilter("ignore")
    b = SW.omega_delta_grid()
    assert b.n == 10000
    r = SIM._engine().run(E.pack_params(b), "lp_square", "lindblad")
    assert np.all(r.status == 0)
    idx = np.array(CHECK)
    rho = r.rho()
    ph, flags = E.mixed_phase(r.state[:, (4 * idx[:, None] + np.arange(4)).ravel()], idx.size, 3, copies=64)
    _, pen = SIM._cp_penalty(ph)
    c = b.cols
    for k, i in enumerate(CHECK):
        with threadpool_limits(1):
            ref = {lab: O.snap_structural_zeros(v) for lab, v in O.run_point(_spec(c, i)).items()}
        for j, lab in enumerate(O.LABELS):
            np.testing.assert_allclose(rho[i, j], ref[lab], atol=1e-10, err_msg=f"point {i} {lab}")
        if not flags[k] & N.STATUS_GAUGE_UNSTABLE:
            _, _, info = O.cz_fidelity(ref, eigh=lambda m: sla.eigh(m))
            assert pen[k] == pytest.approx(info["cz_phase_fidelity"], abs=1e-8), i


def test_c2_grid_populations_across_sweep():
    """Size-independent properties over the whole grid: populations in [0, 1], trace 1
    (every channel of the model maps the 9 levels into themselves) to the parity
    tolerance, a Hermitian PSD sample, and populations that vary smoothly along Omega
    (no point-to-point scatter from a wrong shard or lane)."""
    warnings.simplefilter("ignore")
    b = SW.omega_delta_grid()
    r = SIM._engine().run(E.pack_params(b), "lp_square", "lindblad")
    pops = r.populations()
    assert np.all((pops >= -1e-12) & (pops <= 1 + 1e-12))
    rho = r.rho()[::97]
    tr = np.einsum("nkaa->nk", rho).real
    np.testing.assert_allclose(tr, 1.0, atol=1e-10)
    assert np.linalg.eigvalsh(rho).min() > -1e-11
    p11 = pops[:, 3].reshape(100, 100)
    assert np.max(np.abs(np.diff(p11, 2, axis=0))) < 0.05


def test_dopri5_at_full_c2_stiffness():
    """The reference-style adaptive stepper (RYD_METHOD_DOPRI5) on the bench's own
    corners, at the real blockade (V/2pi = 1234 MHz, V tau up to 5e3 rad) and the
    reference's mesolve tolerances (rtol 1e-8, atol 1e-10, RG/simulation.py:683-690):
    it agrees with the exact propagator to the stepper's own error, the ZVODE-level
    ~1e-7 of SURVEY.md section 7 hard part 1 (populations 1e-7, rho elements 1e-6), and
    needs orders of magnitude more generator applications."""
    warnings.simplefilter("ignore")
    b = SW.omega_delta_grid()
    p = E.pack_params(b)[:, np.array(CHECK)].copy()
    eng = SIM._engine()
    ex = eng.run(p, "lp_square", "lindblad")
    rk = eng.run(p, "lp_square", "lindblad", method="dopri5", rtol=1e-8, atol=1e-10, max_steps=10 ** 7)
    assert np.all(rk.status == 0) and np.all(ex.status == 0)
    np.testing.assert_allclose(rk.populations(), ex.populations(), atol=1e-7, rtol=0)
    np.testing.assert_allclose(rk.state, ex.state, atol=1e-6, rtol=0)
    assert rk.matvec_useful > 20 * ex.matvec_useful
