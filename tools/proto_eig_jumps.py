"""Round-4 feasibility probe (CPU, numpy; not product code): exact C5 jump times from an
eigendecomposition of the non-Hermitian H_eff instead of the ladder walk (DESIGN.md
section 10, "C5 exact jump times").

traj3s_kernel finds each jump time by walking a ladder of precomputed propagators
exp(-i H_eff dt 2^-k) (~90 wave-steps per point, latency-bound).  With
H_eff = W diag(lam) W^-1 once per segment, the no-jump norm

    n(t) = || W diag(exp(-i lam t)) W^-1 psi ||^2,   n'(t) = -<psi(t)| sum_k c_k^+ c_k |psi(t)>

costs one 27-long diagonal scale and one 27x27 product per evaluation, so a jump time is
a few Newton steps on n(t) = r.  This probe measures, over a sample of the C5 grid
(both LP segments): cond(W), the Newton iteration counts, and the jump-time / jump-ket
error against brentq on scipy expm (the oracle's own method, restated here so the
probe imports nothing under oracle/).
    python tools/proto_eig_jumps.py [--points 48] [--traj 16]"""
import argparse
import math
import os
import sys

import numpy as np
import scipy.linalg as sla
from scipy.optimize import brentq

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from noisyquantumsimulator_amd import engine as E          # noqa: E402
from noisyquantumsimulator_amd import sweeps as SW         # noqa: E402
from noisyquantumsimulator_amd import trajectories as TR   # noqa: E402

COL = dict(OMEGA=0, DELTA=1, V=2, DELTA1=3, G1=4, G0=5, GPHI=6, GSC=7, TAU=12, XI_RE=13, XI_IM=14)


def _single(Om, Dl, d1):
    h = np.zeros((3, 3), complex)
    h[2, 1], h[1, 2] = 0.5 * Om, 0.5 * np.conj(Om)
    h[2, 2], h[1, 1] = -Dl, d1
    return h


def _on(a, j):
    m = [np.eye(3, dtype=complex)] * 3
    m[j] = a
    return np.kron(np.kron(m[0], m[1]), m[2])


def heff_and_channels(p, Om):
    Dl, V, d1 = p[COL["DELTA"]], p[COL["V"]], p[COL["DELTA1"]]
    g1, g0, gphi, gsc = (p[COL[k]] for k in ("G1", "G0", "GPHI", "GSC"))
    e = lambda i, j: np.outer(np.eye(3)[i], np.eye(3)[j]).astype(complex)
    H = sum(_on(_single(Om, Dl, d1), j) for j in range(3))
    Pr = [_on(e(2, 2), j) for j in range(3)]
    H = H + V * (Pr[0] @ Pr[1] + Pr[0] @ Pr[2] + Pr[1] @ Pr[2])
    c = []
    for j in range(3):
        c += [math.sqrt(g1) * _on(e(1, 2), j), math.sqrt(g0) * _on(e(0, 2), j),
              math.sqrt(gphi) * Pr[j], math.sqrt(gsc) * _on(e(1, 1), j)]
    G = sum(x.conj().T @ x for x in c)
    return H - 0.5j * G, G, c


class EigenSegment:
    """H_eff = W diag(lam) W^-1; psi(t) = W (exp(-i lam t) * a), a = W^-1 psi."""

    def __init__(self, Heff, G):
        self.lam, self.W = np.linalg.eig(Heff)
        self.Wi = np.linalg.inv(self.W)
        self.G = G
        self.cond = np.linalg.cond(self.W)

    def coeffs(self, psi):
        return self.Wi @ psi

    def ket(self, a, t):
        return self.W @ (np.exp(-1j * self.lam * t) * a)

    def jump_time(self, a, r, t_hi, n0, n_hi):
        """Safeguarded Newton on log n(t) = log r, started from the average-rate guess
        through the segment-end norm n_hi = n(t_hi) the no-jump test already computed."""
        lo, hi = 0.0, t_hi
        t = t_hi * math.log(n0 / r) / math.log(n0 / n_hi)
        for it in range(1, 60):
            x = self.ket(a, t)
            n = np.vdot(x, x).real
            dn = -np.vdot(x, self.G @ x).real
            if n > r:
                lo = t
            else:
                hi = t
            f = math.log(n) - math.log(r)
            if abs(f) <= 2e-15:                       # at the rounding level of n itself
                return t, it
            step = f / (dn / n) if dn != 0 else 0.0
            tn = t - step
            if not (lo < tn < hi):
                tn = 0.5 * (lo + hi)
            if abs(tn - t) <= 4e-16 * max(t, 1e-300) or hi - lo <= 4e-16 * hi:
                return tn, it
            t = tn
        return t, it


def expm_jump_time(Heff, psi, r, t_hi):
    prop = lambda tau: sla.expm(-1j * Heff * tau) @ psi
    f = lambda tau: np.vdot(prop(tau), prop(tau)).real - r
    return brentq(f, 0.0, t_hi, xtol=1e-22, rtol=4 * np.finfo(float).eps, maxiter=200)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=48)
    ap.add_argument("--traj", type=int, default=16)
    ap.add_argument("--check", type=int, default=6, help="points also checked against expm+brentq")
    args = ap.parse_args()
    rng = np.random.default_rng(7)
    idx = np.sort(rng.choice(SW.C5_POINTS, args.points, replace=False))
    batch = SW.blockade_grid_3atom()
    params = E.pack_params(batch)
    params = params if params.shape[0] == SW.C5_POINTS else params.T
    psi0 = TR.plus_state()
    conds, iters, n_jumps, dt_err, ket_err, gaps = [], [], 0, [], [], []
    wave_trips = []                                   # per (point, segment, 64-lane wave): max lane evaluations
    for q, pi in enumerate(idx):
        p = params[pi]
        Om0 = float(p[COL["OMEGA"]])
        xi = complex(p[COL["XI_RE"]], p[COL["XI_IM"]])
        tau = float(p[COL["TAU"]])
        segs = []
        for Om in (complex(Om0), Om0 * xi):
            Heff, G, c = heff_and_channels(p, Om)
            seg = EigenSegment(Heff, G)
            conds.append(seg.cond)
            lam = np.sort_complex(seg.lam)
            gaps.append(np.min(np.abs(np.diff(lam))) / np.max(np.abs(lam)))
            segs.append((seg, Heff, c))
        lane_evals = np.zeros((args.traj, 2), int)
        for tr in range(args.traj):
            psi = psi0.astype(complex).copy()
            r = rng.uniform(1e-12, 1.0)
            for si, (seg, Heff, c) in enumerate(segs):
                t = 0.0
                while True:
                    a = seg.coeffs(psi)
                    end = seg.ket(a, tau - t)
                    if np.vdot(end, end).real > r:
                        psi = end
                        break
                    tj, it = seg.jump_time(a, r, tau - t, np.vdot(psi, psi).real, np.vdot(end, end).real)
                    iters.append(it)
                    lane_evals[tr, si] += it + 1              # + the jump-ket basis change
                    n_jumps += 1
                    if q < args.check:
                        tx = expm_jump_time(Heff, psi, r, tau - t)
                        dt_err.append(abs(tj - tx) / tau)
                        kx = sla.expm(-1j * Heff * tx) @ psi
                        ket_err.append(np.max(np.abs(seg.ket(a, tj) - kx)) / np.linalg.norm(kx))
                    psi = seg.ket(a, tj)
                    t += tj
                    w = np.array([np.vdot(x @ psi, x @ psi).real for x in c])
                    k = min(int(np.searchsorted(np.cumsum(w), rng.uniform() * w.sum(), side="right")), 11)
                    psi = c[k] @ psi
                    psi /= np.linalg.norm(psi)
                    r = rng.uniform(1e-12, 1.0)
        for w0 in range(0, args.traj, 64):
            wave_trips.extend(lane_evals[w0:w0 + 64].max(axis=0))
    conds, iters = np.array(conds), np.array(iters)
    print(f"points {args.points} x 2 segments: cond(W) median {np.median(conds):.3g} "
          f"max {conds.max():.3g}; min relative eigenvalue gap {np.min(gaps):.2e}")
    print(f"jumps {n_jumps} over {args.points * args.traj} trajectories; Newton iterations "
          f"mean {iters.mean():.2f} p99 {np.percentile(iters, 99):.0f} max {iters.max()}")
    wave_trips = np.array(wave_trips)
    print(f"jump-loop evaluations per (64-lane wave, segment) beyond the 2 no-jump matvecs: "
          f"mean {wave_trips.mean():.1f} max {wave_trips.max()} (lane-divergence bound)")
    if dt_err:
        print(f"vs expm+brentq ({len(dt_err)} jumps): |dt|/tau max {max(dt_err):.2e}, "
              f"ket rel err max {max(ket_err):.2e}")


if __name__ == "__main__":
    main()
