"""Round-3 feasibility probe (CPU, numpy; not product code): exact slow/fast
block-diagonalisation of the two-atom sector generator L = L0 + V R (DESIGN.md section
10).  The V term rotates only the |rr>-coherence coordinates; a similarity
T = [[I, Y], [0, I]] [[I, 0], [X, I]] found by two contracting fixed-point iterations
(rate ~ ||L0|| / V) splits L into an O(Omega) slow block and an O(V) fast block, so the
s = 11-14 squaring levels of the full propagator are needed only on the small fast block.
Prints the iteration counts, the block norms (squaring levels each block needs) and the
error of T^-1 diag(expm(Ls tau), expm(Lf tau)) T against expm(L tau).
    python tools/proto_blockdiag.py"""
import numpy as np
import scipy.linalg as sla

TWO_PI = 2 * np.pi


def single_atom(Om, Dl, d1, g0, g1, gphi, gsc):
    """5x5 real single-atom generator on (e00, e11, err, ex, ey)."""
    hx, hz, G = 0.5 * Om, 0.5 * (d1 + Dl), 0.5 * (g1 + g0 + gphi + gsc)
    return np.array([[0, 0, g0, 0, 0],
                     [0, 0, g1, 0, -2 * hx],
                     [0, 0, -(g0 + g1), 0, 2 * hx],
                     [0, 0, 0, -G, 2 * hz],
                     [0, hx, -hx, -2 * hz, -G]], dtype=float)


def sector_generator(Om, Dl, d1, V, rates):
    M = single_atom(Om, Dl, d1, *rates)
    S = np.diag([0.0, 0.0, 2.0, 1.0, 1.0])            # {P_r, .} on the basis
    D = np.zeros((5, 5)); D[4, 3], D[3, 4] = 1.0, -1.0  # -i[P_r, .]: ex -> ey, ey -> -ex
    I = np.eye(5)
    L0 = np.kron(M, I) + np.kron(I, M)
    R = 0.5 * (np.kron(S, D) + np.kron(D, S))
    return L0, R


def main():
    Om = TWO_PI * 5e6
    Dl, d1, V = 0.377 * Om, TWO_PI * 0.216e6, TWO_PI * 1233.8e6
    rates = (3.6e3, 3.6e3, 2.5e4, 2.7e5)               # g0, g1, gphi, gsc (s^-1)
    tau = 4.29268 / Om
    L0, R = sector_generator(Om, Dl, d1, V, rates)
    L = L0 + V * R
    # split: fast = range of R (the V-rotated coordinates), slow = its kernel
    u, sv, _ = np.linalg.svd(R)
    k = int((sv > 1e-12).sum())
    Q = np.hstack([u[:, k:], u[:, :k]])               # slow first, then fast
    Lq = Q.T @ L @ Q
    ns = 25 - k
    A, B, C, Dm = Lq[:ns, :ns], Lq[:ns, ns:], Lq[ns:, :ns], Lq[ns:, ns:]
    print(f"slow {ns} x fast {k};  ||A|| = {np.linalg.norm(A, 2):.3e}  ||D|| = {np.linalg.norm(Dm, 2):.3e}"
          f"  ||B|| = {np.linalg.norm(B, 2):.3e}  ||C|| = {np.linalg.norm(C, 2):.3e}")
    Dinv = np.linalg.inv(Dm)
    # X: lower-left zero after [[I,0],[X,I]]:  X A - D X + C - X B X = 0
    X = np.zeros((k, ns))
    for it in range(60):
        Xn = Dinv @ (X @ A + C - X @ B @ X)
        if np.max(np.abs(Xn - X)) <= 1e-17 * max(1.0, np.max(np.abs(Xn))):
            X = Xn
            break
        X = Xn
    itx = it + 1
    T1 = np.block([[np.eye(ns), np.zeros((ns, k))], [X, np.eye(k)]])
    L1 = T1 @ Lq @ np.linalg.inv(T1)
    As, Bs, Ds = L1[:ns, :ns], L1[:ns, ns:], L1[ns:, ns:]
    # Y: upper-right zero after [[I,Y],[0,I]]:  Y Ds - As Y + Bs = 0  ->  Y = (As Y - Bs) Ds^-1
    Y = np.zeros((ns, k))
    Dsinv = np.linalg.inv(Ds)
    for it in range(60):
        Yn = (As @ Y - Bs) @ Dsinv
        if np.max(np.abs(Yn - Y)) <= 1e-17 * max(1.0, np.max(np.abs(Yn))):
            Y = Yn
            break
        Y = Yn
    ity = it + 1
    T2 = np.block([[np.eye(ns), Y], [np.zeros((k, ns)), np.eye(k)]])
    Lb = T2 @ L1 @ np.linalg.inv(T2)
    off = max(np.abs(Lb[:ns, ns:]).max(), np.abs(Lb[ns:, :ns]).max())
    Ls, Lf = Lb[:ns, :ns], Lb[ns:, ns:]
    T = T2 @ T1
    Ub = np.linalg.inv(T) @ sla.block_diag(sla.expm(Ls * tau), sla.expm(Lf * tau)) @ T
    U = Q @ Ub @ Q.T
    Uex = sla.expm(L * tau)
    lv = lambda n: int(np.ceil(np.log2(max(n * tau / 0.5, 1.0))))
    print(f"fixed-point iterations: X {itx}, Y {ity};  residual off-diagonal {off:.2e} (scale {np.abs(Lq).max():.2e})")
    print(f"cond(T) = {np.linalg.cond(T):.4f};  squaring levels: full {lv(np.linalg.norm(L, 1))}, "
          f"slow {lv(np.linalg.norm(Ls, 1))} ({ns}x{ns}), fast {lv(np.linalg.norm(Lf, 1))} ({k}x{k})")
    print(f"max |U_block - expm(L tau)| = {np.abs(U - Uex).max():.2e}")


if __name__ == "__main__":
    main()
