"""C4 (BASELINE.json configs[3]): the 1M-point species x temperature x tweezer-power
LP-square grid on the GPU, at full size.

* every point succeeds; size-independent properties of every rho (trace 1,
  Hermitian by construction, populations in [0, 1]);
* the 8-way range partition (what 8 ranks of bench.py --workload c4 run) reproduces
  the single-launch rows bit for bit;
* spot checks against the expm oracle for both species, at the grid's corners.
"""
import numpy as np
import pytest

from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import sweeps as SW
from oracle import lindblad_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-10


@pytest.fixture(scope="module")
def c4():
    b = SW.species_temperature_power_grid()
    p = E.pack_params(b)
    eng = E.Engine()
    r = eng.run(p, "lp_square", "lindblad")
    return b, p, eng, r


def test_c4_full_grid_properties(c4):
    b, p, eng, r = c4
    assert b.n == SW.C4_POINTS
    assert np.all(r.status == 0)
    tr = r.col("TRACE11")
    np.testing.assert_allclose(tr, 1.0, atol=1e-11)
    pops = r.populations()
    assert np.all((pops > -1e-12) & (pops < 1 + 1e-12))
    # diagonal sector coordinates of every input's rho sum to 1 (trace of each rho)
    S = r.state.reshape(25, -1)
    diag_sum = sum(S[5 * a + c] for a in range(3) for c in range(3))
    np.testing.assert_allclose(diag_sum, 1.0, atol=1e-11)


def test_c4_range_shards_match_single_launch(c4):
    b, p, eng, r = c4
    ws = 8
    for rank in (0, 3, 7):
        sl = SW.range_shard(SW.C4_POINTS, rank, ws)
        rs = eng.run(p[:, sl], "lp_square", "lindblad")
        np.testing.assert_array_equal(rs.state, r.state[:, 4 * sl.start:4 * sl.stop])
        np.testing.assert_array_equal(rs.summary, r.summary[:, sl])


@pytest.mark.parametrize("i", [0, 499_999, 500_000, 999_999, 250_123])
def test_c4_points_match_oracle(c4, i):
    b, p, eng, r = c4
    c = b.cols
    spec = O.PointSpec(protocol="lp_square", Omega=c["Omega"][i], V=c["V"][i],
                       Delta=c["Delta_gate"][i], tau=c["tau_single"][i],
                       xi=complex(c["xi_re"][i], c["xi_im"][i]), delta_zeeman=c["delta_zeeman"][i],
                       delta_stark=c["delta_stark"][i],
                       c_ops=O.collapse_operators({k: c[k][i] for k in O.RATE_KEYS}))
    ref = O.run_point(spec)
    rho = E.expand_rho(r.state[:, 4 * i:4 * i + 4], 1)[0]
    for k, lab in enumerate(O.LABELS):
        np.testing.assert_allclose(rho[k], ref[lab], atol=TOL, rtol=0, err_msg=f"point {i}/{lab}")
