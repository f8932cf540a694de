"""CPU checks of the three-atom (C5) oracle and host layer: Philox4x32-10 against the
Random123 known-answer vectors, the three-atom Liouvillian against the two-atom
oracle (third atom parked in |0>), the exact-jump-time MC unravelling against the
exact mean state, and the C5 grid derivation.  No GPU."""
import ctypes
import warnings

import numpy as np
import pytest

from noisyquantumsimulator_amd import _native as N
from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import sweeps as SW
from noisyquantumsimulator_amd import trajectories as TR
from oracle import lindblad_oracle as O2
from oracle import three_atom_oracle as O3


@pytest.mark.parametrize("ctr,key,out", [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
])
def test_philox_known_answers(ctr, key, out):
    """Random123 kat_vectors for philox4x32_10."""
    assert O3.philox4x32_10(ctr, key) == out


def test_draw_ranges():
    rs = np.array([O3.draws(t, c, 7, 99) for t in range(200) for c in range(3)])
    assert np.all(rs[:, 0] > 0) and np.all(rs[:, 0] <= 1) and np.all(rs[:, 1] >= 0) and np.all(rs[:, 1] < 1)
    assert abs(rs[:, 0].mean() - 0.5) < 0.05


def _point(i=100, scale=50.0):
    warnings.simplefilter("ignore")
    p = E.pack_params(SW.blockade_grid_3atom(point_slice=slice(i, i + 1)))[:, 0].copy()
    p[4:8] *= scale
    return p


@pytest.mark.parametrize("spectator", [0, 2])
def test_three_atom_reduces_to_two_atom_oracle(spectator):
    """Atom `spectator` in |0> never moves (no drive, every channel annihilates |0>),
    so rho_3 = rho_2 (x) |0><0| with rho_2 from the two-atom oracle that reproduces the
    reference's published numbers."""
    p = _point()
    g1, g0, gphi, gsc = O3.rates(p)
    one, zero = np.array([0, 1, 0]), np.array([1, 0, 0])
    kets = [one, one]
    kets.insert(spectator, zero)
    psi0 = TR.product_ket(*kets)
    r3 = O3.exact_rho(p, "lp_square", psi0)
    s = O3.single_ops()
    I = np.eye(3)

    def both(op, g):
        return [np.sqrt(g) * np.kron(op, I), np.sqrt(g) * np.kron(I, op)]
    c2 = both(s["s1r_down"], g1) + both(s["s0r"], g0) + both(s["Pr"], gphi) + both(s["P1"], gsc)
    k2 = np.kron(one, one).astype(complex)
    rho = np.outer(k2, k2.conj())
    for Om, Dl, dt in O3.schedule(p, "lp_square"):
        rho = O2.evolve_state(O2.two_atom_hamiltonian(Om, Dl, p[2], 3, delta_zeeman=p[3]), rho, [0, dt], c2)
    P0 = np.diag([1.0, 0, 0])
    ref = np.kron(P0, rho) if spectator == 0 else np.kron(rho, P0)
    np.testing.assert_allclose(r3, ref, atol=1e-12)


def test_pure_ket_is_zero_rate_limit():
    p = _point(scale=0.0)
    psi0 = TR.plus_state()
    psi = O3.pure_ket(p, "lp_square", psi0)
    np.testing.assert_allclose(O3.exact_rho(p, "lp_square", psi0), np.outer(psi, psi.conj()), atol=1e-11)


def test_mc_unravelling_matches_exact_rho():
    """Exact-jump-time trajectories (the GPU's Philox streams) average to the Lindblad state."""
    p = _point(i=5, scale=40.0)
    psi0 = TR.plus_state()
    ref = O3.exact_rho(p, "lp_square", psi0)
    n = 240
    kets, nj = [], 0
    for t in range(n):
        k, jumps = O3.mc_trajectory(p, "lp_square", psi0, point=5, traj=t, seed=11)
        kets.append(k)
        nj += len(jumps)
    K = np.array(kets)
    X = np.einsum("ta,tb->tab", K, K.conj())
    mean, sd = X.mean(0), np.sqrt((np.abs(X - X.mean(0)) ** 2).mean(0) / (n - 1))
    assert nj > 30                                   # the test exercises jumps
    # elements fed by rare jump channels can have no sampled event at all (sd = 0):
    # floor the standard error at the Poisson scale sqrt(|rho| / n)
    z = np.abs(mean - ref) / np.maximum(sd, np.sqrt(np.abs(ref) / n) + 1e-12)
    assert np.all((np.abs(mean - ref) < 1e-10) | (z < 5.5)), z.max()


def test_c5_grid_and_shards():
    warnings.simplefilter("ignore")
    b = SW.blockade_grid_3atom()
    assert b.n == SW.C5_POINTS == 4096
    # the default order: Omega-major, V/Omega fastest
    np.testing.assert_allclose(b["V_over_Omega"].reshape(64, 64)[0], np.logspace(1, 3, 64), rtol=1e-9)
    np.testing.assert_allclose(b["Omega"].reshape(64, 64)[:, 0] / (2e6 * np.pi), np.linspace(1, 10, 64), rtol=1e-12)
    # blocked order: [8 V/Omega blocks][64 Omega][8 V/Omega in the block]
    bb = SW.blockade_grid_3atom(order="blocked")
    vo = bb["V_over_Omega"].reshape(8, 64, 8)
    np.testing.assert_allclose(vo[:, 0, :].ravel(), np.logspace(1, 3, 64), rtol=1e-9)
    np.testing.assert_allclose(bb["Omega"].reshape(8, 64, 8)[0, :, 0] / (2e6 * np.pi), np.linspace(1, 10, 64),
                               rtol=1e-12)
    om = bb["Omega"].reshape(8, 64, 8)
    assert np.all(np.diff(om, axis=1) > 0)                  # low Omega first in a block
    # every N = 8 range shard of the blocked order spans the whole Omega axis
    for r in range(8):
        sl = SW.range_shard(4096, r, 8)
        np.testing.assert_allclose(np.unique(bb["Omega"][sl]) / (2e6 * np.pi), np.linspace(1, 10, 64), rtol=1e-12)
    # the same point set in every order
    key = lambda x: np.lexsort((x["V_over_Omega"], x["Omega"]))
    np.testing.assert_array_equal(b["Omega"][key(b)], bb["Omega"][key(bb)])
    p = E.pack_params(b)
    assert np.all(p[4:8] > 0)
    full = p
    parts = []
    for r in range(3):
        bb, off = SW.c5_rank_shard(r, 3)
        assert off == SW.range_shard(4096, r, 3).start
        parts.append(E.pack_params(bb))
    np.testing.assert_array_equal(np.concatenate(parts, axis=1), full)


def test_traj_desc_layout_and_states():
    assert ctypes.sizeof(N.TrajDesc) == 472                # ABI 5: flags + point_stride before the seed
    d = TR.make_traj_desc("lp_square", TR.plus_state(), 512, seed=3)
    v = np.array(d.psi0[:])
    assert abs((v ** 2).sum() - 1) < 1e-15 and d.n_traj == 512 and d.ladder_levels == N.T["EXACT"]
    # exact jump times by default; the ladder walk where they do not apply (shaped envelope)
    assert TR.make_traj_desc("lp_shaped", TR.plus_state(), 256, shape="cosine").ladder_levels == TR.LADDER_WALK
    assert TR.make_traj_desc("lp_shaped", TR.plus_state(), 256, shape="square").ladder_levels == N.T["EXACT"]
    assert TR.make_traj_desc("bangbang", TR.plus_state(), 256, ladder_levels=20).ladder_levels == 20
    assert TR.basis_index(1, 1, 1) == 13 and TR.QUBIT_INDEX3 == (0, 1, 3, 4, 9, 10, 12, 13)
    flat = np.arange(1458, dtype=float)[None]
    rho = TR.unpack_rho(flat)
    assert rho[0, 1, 0] == 2 + 3j and rho[0, 0, 1] == 54 + 55j    # vec index a + 27 b


def test_strided_shards_partition_the_grid():
    """sweeps.c5_strided_shard: rank r of N holds points r, r + N, ... (offset r, stride N);
    together the ranks hold every point of the Omega-major grid once, with its columns."""
    full = E.pack_params(SW.blockade_grid_3atom())
    seen = np.zeros(SW.C5_POINTS, int)
    for r in range(8):
        b, off, stride = SW.c5_strided_shard(r, 8)
        assert (off, stride) == (r, 8) and b.n == SW.C5_POINTS // 8
        np.testing.assert_array_equal(E.pack_params(b), full[:, r::8])
        seen[r::8] += 1
    assert np.all(seen == 1)
    d = TR.make_traj_desc("lp_square", TR.plus_state(), 256)
    assert d.point_stride == 0                     # contiguous unless a shard sets it
