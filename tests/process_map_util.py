"""Shared helpers for the process-map tests: oracle PointSpec from packed params and
the GPU output rows an exact map corresponds to (so host code is testable on CPU)."""
import numpy as np

from noisyquantumsimulator_amd import _native as N
from oracle import lindblad_oracle as O


def spec_from_params(p, i, protocol, n_steps=300):
    g = lambda k: p[N.P[k], i]
    I3 = np.eye(3)
    ops = []
    for atom in ("A", "B"):
        emb = (lambda o: np.kron(o, I3)) if atom == "A" else (lambda o: np.kron(I3, o))
        for key, op in (("G1", np.outer(I3[1], I3[2])), ("G0", np.outer(I3[0], I3[2])),
                        ("GPHI", np.diag([0, 0, 1.0])), ("GSC", np.diag([0, 1.0, 0]))):
            rate = g(f"{key}_{atom}")
            if rate > 0:
                ops.append(np.sqrt(rate) * emb(op.astype(complex)))
    kw = dict(Omega=g("OMEGA"), V=g("V"), delta_zeeman=g("DELTA1"), c_ops=ops)
    if protocol == "lp_square":
        return O.PointSpec(protocol="lp_square", Delta=g("DELTA"), tau=g("TAU"),
                           xi=complex(g("XI_RE"), g("XI_IM")), **kw)
    if protocol == "smooth_jp":
        return O.PointSpec(protocol="smooth_jp", Delta=g("DELTA"), tau=g("TAU"), A=g("A"),
                           omega_mod=g("OMEGA_MOD"), phi_offset=g("PHI_OFF"), n_steps=n_steps, **kw)
    nseg = int(g("NSEG"))
    return O.PointSpec(protocol="bangbang", omega_tau=g("OMEGA_TAU"),
                       switching_times=[p[N.P["SWT0"] + k, i] for k in range(nseg - 1)],
                       phases=[p[N.P["PHI0"] + k, i] for k in range(nseg)], **kw)


def rows_from_map(S):
    """(state (25, 4), coh (NCOH, 1)) rows that the engine returns for the map S."""
    state = np.zeros((25, 4))
    for x in range(4):
        for y in range(4):
            state[5 * (y >> 1) + (y & 1), x] = S[5 * y, 5 * x].real
    coh = np.zeros((N.NCOH, 1))

    def put(row, z):
        coh[row, 0], coh[row + 1, 0] = z.real, z.imag
    for base, units in ((N.C["K0"], ((0, 1), (2, 3))), (N.C["K1"], ((0, 2), (1, 3)))):
        for s, (a, b) in enumerate(units):
            for o, (c, d) in enumerate(units):
                put(base + 4 * s + 2 * o, S[4 * c + d, 4 * a + b])
    put(N.C["K2"], S[3, 3])
    put(N.C["K3"], S[6, 6])
    return state, coh


def unitary_map(U):
    S = np.zeros((16, 16), dtype=complex)
    for a in range(4):
        for b in range(4):
            X = np.zeros((4, 4), dtype=complex)
            X[a, b] = 1
            S[:, 4 * a + b] = (U @ X @ U.conj().T).reshape(-1)
    return S
