"""CPU oracle for the Rydberg-CZ Lindblad path -- TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The product path (``noisyquantumsimulator_amd``) never routes through it.

It restates, in plain numpy/scipy, the reference solver path of
scottjones03/NoisyQuantumSimulator for the two-atom Rydberg CZ gate:

* two-atom Hamiltonian        RG/hamiltonians.py:584-1172 (build_laser/detuning/
                              interaction/zeeman/stark, build_full_hamiltonian) and
                              RG/hamiltonians.py:1179-1274 (phase-modulated H)
* collapse operators          RG/noise_models.py:1199-1620 (build_all_noise_operators)
* time evolution              RG/simulation.py:647-690 (evolve_state -> qutip.mesolve),
                              evolvers :693-776 (LP square), :1502-1760 (smooth JP),
                              :1795-1943 (bang-bang JP), :2099-2231 (shaped LP)
* CZ fidelity                 RG/simulation.py:186-633 (compute_state_fidelity,
                              compute_CZ_fidelity)

(RG = src/qpu_simulator/micro_physics/neutral_atoms/rydberg_gates.)

Two integrators are provided for every segment:

``method="expm"``   exact propagator exp(L dt) of the column-stacked Liouvillian
                    (scipy.linalg.expm) -- ground truth, used for parity.
``method="zvode"``  scipy ZVODE Adams at the reference's tolerances
                    (atol 1e-10, rtol 1e-8, reference nsteps), restarted per
                    segment and stepped through the reference's tlist -- the
                    "QuTiP-like" CPU baseline.  QuTiP itself is an unpinned
                    third-party dependency (qutip>=5.0.0, pyproject.toml:38) that
                    is absent here; QuTiP 5's default mesolve integrator wraps the
                    same scipy ZVODE Adams method on the same vectorised
                    Liouvillian.

Parity pins (tests/test_oracle_golden.py): the published noise-free fidelities
of the reference notebooks and the closed-form decay
known-answer test of scripts/archive/test_mesolve_direct.py:34-51.

Mixed-state phase penalty: ``cz_fidelity(..., eigh=scipy.linalg.eigh)`` is the
reference's procedure (QuTiP 5's eigensolver); ``snap_structural_zeros`` gives the
exact zeros QuTiP's integration keeps; ``gauge_unstable`` tells whether the penalty
is a function of rho at 1e-12 relative precision (mostly it is not).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import scipy.linalg as sla
from scipy.integrate import ode

LABELS = ("00", "01", "10", "11")

# --------------------------------------------------------------------------
# single-atom operators (RG/hamiltonians.py:424-522)
# --------------------------------------------------------------------------


def _ket(d: int, i: int) -> np.ndarray:
    v = np.zeros(d, dtype=complex)
    v[i] = 1.0
    return v


def _proj(d: int, i: int) -> np.ndarray:
    return np.outer(_ket(d, i), _ket(d, i))


def _trans(d: int, to: int, frm: int) -> np.ndarray:
    """|to><frm|"""
    return np.outer(_ket(d, to), _ket(d, frm))


def _two(op1: np.ndarray, op2: np.ndarray) -> np.ndarray:
    """op1 (x) op2 -- qutip.tensor ordering (atom 1 is the slow index)."""
    return np.kron(op1, op2)


# --------------------------------------------------------------------------
# Hamiltonian (RG/hamiltonians.py:584-1274)
# --------------------------------------------------------------------------


def two_atom_hamiltonian(Omega: complex, Delta: float, V: float, dim: int = 3,
                         delta_zeeman: float = 0.0, delta_stark: float = 0.0,
                         trap_laser_on: bool = True,
                         add_detuning: bool = True) -> np.ndarray:
    """H = sum_atoms [ (Omega/2)|r><1| + h.c. - Delta P_r + (dz + ds) P_1 ] + V P_rr.

    dim 4 follows the sigma+ default of RG/hamiltonians.py:655-663 (|r-> not
    driven), detuning -Delta on both r+ and r- (:741-753, zeeman_splitting=0) and
    V on every r(+-)r(+-) pair (:835-853).  ``add_detuning=False`` mirrors the
    phase-modulated builder's ``if Delta != 0`` guard (:1264-1265) -- numerically
    identical, kept for fidelity to the reference.
    """
    d = dim
    I = np.eye(d, dtype=complex)
    if d == 3:
        s1r = _trans(3, 2, 1)              # |r><1|
        Ha = 0.5 * (Omega * s1r + np.conj(Omega) * s1r.conj().T)
        Pr = [_proj(3, 2)]
    elif d == 4:
        s1rp = _trans(4, 2, 1)             # |r+><1|
        Ha = 0.5 * (Omega * s1rp + np.conj(Omega) * s1rp.conj().T)
        Pr = [_proj(4, 2), _proj(4, 3)]
    else:
        raise ValueError(f"Unsupported Hilbert space dimension: {dim}. Use 3 or 4.")
    H = _two(Ha, I) + _two(I, Ha)
    if add_detuning:
        for P in Pr:
            H = H - Delta * (_two(P, I) + _two(I, P))
    for Pa in Pr:
        for Pb in Pr:
            H = H + V * _two(Pa, Pb)
    P1 = _proj(d, 1)
    if delta_zeeman != 0:
        H = H + delta_zeeman * (_two(P1, I) + _two(I, P1))
    if delta_stark != 0 and trap_laser_on:
        H = H + delta_stark * (_two(P1, I) + _two(I, P1))
    return H


# --------------------------------------------------------------------------
# collapse operators (RG/noise_models.py:1199-1620)
# --------------------------------------------------------------------------

RATE_KEYS = ("gamma_r", "gamma_bbr", "gamma_phi_laser", "gamma_phi_thermal",
             "gamma_phi_zeeman", "gamma_loss_antitrap", "gamma_loss_background",
             "gamma_scatter_intermediate", "gamma_leakage", "mJ_leakage_rate")


def collapse_operators(rates: Dict[str, float], dim: int = 3,
                       branching_1: float = 0.5) -> List[np.ndarray]:
    """The reference's c_op list, in the reference's order and with its
    ``rate > 0`` guards (build_all_noise_operators, RG/noise_models.py:1575-1592)."""
    g = {k: float(rates.get(k, 0.0) or 0.0) for k in RATE_KEYS}
    d = dim
    I = np.eye(d, dtype=complex)
    c: List[np.ndarray] = []
    rys = [2] if d == 3 else [2, 3]

    def both(op, rate):
        return [math.sqrt(rate) * _two(op, I), math.sqrt(rate) * _two(I, op)]

    # 1. decay (build_decay_operators :1199-1297); per Rydberg state:
    #    [r->1 (atom1, atom2), r->0 (atom1, atom2)]
    if g["gamma_r"] > 0:
        for r in rys:
            c += both(_trans(d, 1, r), g["gamma_r"] * branching_1)
            c += both(_trans(d, 0, r), g["gamma_r"] * (1 - branching_1))
    if g["gamma_bbr"] > 0:
        for r in rys:
            c += both(_trans(d, 0, r), g["gamma_bbr"])
    if d == 4 and g["mJ_leakage_rate"] > 0:
        c += both(_trans(d, 3, 2), g["mJ_leakage_rate"])
        c += both(_trans(d, 2, 3), g["mJ_leakage_rate"])
    # 2. dephasing (:1300-1356)
    gphi = g["gamma_phi_laser"] + g["gamma_phi_thermal"] + g["gamma_phi_zeeman"]
    if gphi > 0:
        for r in rys:
            c += both(_proj(d, r), gphi)
    # 3./4./6. losses |r> -> |0>  (:1359-1412)
    for key in ("gamma_loss_antitrap", "gamma_loss_background"):
        if g[key] > 0:
            for r in rys:
                c += both(_trans(d, 0, r), g[key])
    # 5. scattering: dephasing of |1> (:1415-1446)
    if g["gamma_scatter_intermediate"] > 0:
        c += both(_proj(d, 1), g["gamma_scatter_intermediate"])
    if g["gamma_leakage"] > 0:
        for r in rys:
            c += both(_trans(d, 0, r), g["gamma_leakage"])
    return c


# --------------------------------------------------------------------------
# Liouvillian + integrators (qutip.mesolve restatement)
# --------------------------------------------------------------------------


def liouvillian(H: np.ndarray, c_ops: Sequence[np.ndarray]) -> np.ndarray:
    """Column-stacked (QuTiP) superoperator: vec(rho)[a + D*b] = rho[a, b]."""
    D = H.shape[0]
    Id = np.eye(D, dtype=complex)
    L = -1j * (np.kron(Id, H) - np.kron(H.T, Id))
    for c in c_ops:
        cdc = c.conj().T @ c
        L = L + np.kron(c.conj(), c) - 0.5 * np.kron(Id, cdc) - 0.5 * np.kron(cdc.T, Id)
    return L


def vec(rho: np.ndarray) -> np.ndarray:
    return rho.reshape(-1, order="F")


def unvec(v: np.ndarray, D: int) -> np.ndarray:
    return v.reshape(D, D, order="F")


def _zvode(f, y0: np.ndarray, tlist: np.ndarray, atol: float, rtol: float,
           nsteps: int) -> np.ndarray:
    r = ode(f)
    r.set_integrator("zvode", method="adams", atol=atol, rtol=rtol,
                     nsteps=nsteps, order=12)
    r.set_initial_value(y0, tlist[0])
    y = y0
    for t in tlist[1:]:
        y = r.integrate(t)
        if not r.successful():
            raise RuntimeError("ZVODE failed (excess work / nsteps cap) at t=%g" % t)
    return y


def evolve_state(H: np.ndarray, psi0: np.ndarray, tlist: np.ndarray,
                 c_ops: Sequence[np.ndarray] = (), method: str = "expm",
                 options: Optional[dict] = None) -> np.ndarray:
    """RG/simulation.py:647-690.  A ket with no c_ops stays a ket (Schrodinger);
    a ket with c_ops becomes rho0 = |psi><psi| (scripts/archive/test_mesolve.py:17-31)."""
    opts = {"atol": 1e-10, "rtol": 1e-8, "nsteps": 50000}
    if options:
        opts.update(options)
    tlist = np.asarray(tlist, dtype=float)
    T = tlist[-1] - tlist[0]
    D = H.shape[0]
    is_ket = psi0.ndim == 1
    if is_ket and len(c_ops) == 0:
        if method == "expm":
            return sla.expm(-1j * H * T) @ psi0
        return _zvode(lambda t, y: -1j * (H @ y), psi0.astype(complex), tlist,
                      opts["atol"], opts["rtol"], opts["nsteps"])
    rho = np.outer(psi0, psi0.conj()) if is_ket else psi0
    L = liouvillian(H, c_ops)
    if method == "expm":
        return unvec(sla.expm(L * T) @ vec(rho), D)
    y = _zvode(lambda t, y: L @ y, vec(rho).astype(complex), tlist,
               opts["atol"], opts["rtol"], opts["nsteps"])
    return unvec(y, D)


# --------------------------------------------------------------------------
# protocol schedules (RG/simulation.py evolvers)
# --------------------------------------------------------------------------


@dataclass
class PointSpec:
    """Physics-level inputs of one simulate_CZ_gate point (after host derivation)."""
    protocol: str                   # "lp_square" | "lp_shaped" | "bangbang" | "smooth_jp"
    Omega: float
    V: float
    Delta: float = 0.0              # LP static detuning / smooth-JP two-photon detuning
    delta_zeeman: float = 0.0
    delta_stark: float = 0.0
    trap_laser_on: bool = True
    dim: int = 3
    # LP
    tau: float = 0.0                # single pulse (LP) or total (JP) duration
    xi: complex = 1.0 + 0j
    pulse_shape: str = "square"
    area_correction: float = 1.0
    # bang-bang
    omega_tau: float = 0.0
    switching_times: Sequence[float] = ()
    phases: Sequence[float] = ()
    # smooth JP
    A: float = 0.0
    omega_mod: float = 0.0
    phi_offset: float = 0.0
    n_steps: int = 300
    # noise
    c_ops: List[np.ndarray] = field(default_factory=list)


def initial_kets(dim: int = 3) -> Dict[str, np.ndarray]:
    b0, b1 = _ket(dim, 0), _ket(dim, 1)
    return {"00": np.kron(b0, b0), "01": np.kron(b0, b1),
            "10": np.kron(b1, b0), "11": np.kron(b1, b1)}


def cosine_envelope(t: float, tau: float) -> float:
    """RG/pulse_shaping.py:191-236 (sin^2).  Gaussian and blackman normalise by
    their own max, so a scalar t gives exactly 1 (:183-186, :290-293)."""
    return math.sin(math.pi * t / tau) ** 2


def envelope(shape: str, t: float, tau: float) -> float:
    s = shape.lower()
    if s == "cosine":
        return float(np.sin(np.pi * t / tau) ** 2)
    if s in ("gaussian", "blackman", "square"):
        return 1.0
    if s == "drag":
        raise TypeError("pulse_envelope_drag() missing 1 required positional argument: 'Delta_leak'")
    raise ValueError(f"Unknown pulse shape: {shape}")


def segments(p: PointSpec) -> List[Tuple[np.ndarray, np.ndarray, Optional[dict]]]:
    """(H, tlist, options) per mesolve call, exactly as the reference evolvers."""
    dz, ds, tl = p.delta_zeeman, p.delta_stark, p.trap_laser_on
    segs = []
    if p.protocol == "lp_square":                       # :693-776
        H1 = two_atom_hamiltonian(p.Omega, p.Delta, p.V, p.dim, dz, ds, tl)
        H2 = two_atom_hamiltonian(p.Omega * p.xi, p.Delta, p.V, p.dim, dz, ds, tl)
        t = np.linspace(0, p.tau, 100)
        segs = [(H1, t, None), (H2, t, None)]
    elif p.protocol == "lp_shaped":                     # :2099-2231
        n = 500
        t_pulse = np.linspace(0, p.tau, n)
        dt = p.tau / n
        Om_peak = p.Omega * p.area_correction
        opts = {"atol": 1e-10, "rtol": 1e-8, "nsteps": 50000}
        for fac in (1.0, p.xi):
            for i in range(n - 1):
                t_mid = (t_pulse[i] + t_pulse[i + 1]) / 2
                Om_t = Om_peak * envelope(p.pulse_shape, t_mid, p.tau) * fac
                H = two_atom_hamiltonian(Om_t, p.Delta, p.V, p.dim, dz, ds, tl)
                segs.append((H, np.array([0.0, dt]), opts))
    elif p.protocol == "bangbang":                      # :1795-1943
        bounds = [b / p.Omega for b in [0.0] + list(p.switching_times) + [p.omega_tau]]
        opts = {"atol": 1e-10, "rtol": 1e-8, "nsteps": 10000}
        for k, ph in enumerate(p.phases):
            dts = bounds[k + 1] - bounds[k]
            if dts < 1e-18:
                continue
            H = two_atom_hamiltonian(p.Omega * np.exp(1j * ph), 0.0, p.V, p.dim, dz, ds, tl,
                                     add_detuning=False)
            segs.append((H, np.linspace(0, dts, 51), opts))
    elif p.protocol == "smooth_jp":                     # :1502-1760
        tl_full = np.linspace(0, p.tau, p.n_steps + 1)
        dt = p.tau / p.n_steps
        opts = {"atol": 1e-10, "rtol": 1e-8, "nsteps": 10000}
        for i in range(p.n_steps):
            t_mid = tl_full[i] + dt / 2
            ph = p.A * np.cos(p.omega_mod * t_mid - p.phi_offset)
            H = two_atom_hamiltonian(p.Omega * np.exp(1j * ph), p.Delta, p.V, p.dim, dz, ds, tl,
                                     add_detuning=(p.Delta != 0))
            segs.append((H, np.array([0.0, dt]), opts))
    else:
        raise ValueError(p.protocol)
    return segs


def run_point(p: PointSpec, method: str = "expm") -> Dict[str, np.ndarray]:
    """Final state per computational-basis input (kets if no c_ops, else rho)."""
    segs = segments(p)
    out = {}
    for lab, psi0 in initial_kets(p.dim).items():
        s = psi0
        for H, t, opts in segs:
            s = evolve_state(H, s, t, p.c_ops, method=method, options=opts)
        out[lab] = s
    return out


# --------------------------------------------------------------------------
# CZ fidelity (RG/simulation.py:186-633)
# --------------------------------------------------------------------------


def _angle(z: complex) -> float:
    return float(np.angle(z))


def cz_fidelity(results: Dict[str, np.ndarray], dim: int = 3,
                eigh=np.linalg.eigh) -> Tuple[Dict[str, float], float, Dict]:
    """Restatement of compute_CZ_fidelity(extract_global_phase=True).

    Mixed branch: F_x = <x|rho_x|x> (qutip.fidelity(rho, |t><t|)**2, the target
    sign is irrelevant); phase from the dominant eigenvector (gauge-dependent,
    SURVEY.md hard part 3).  Pure branch: F_x = |<x|psi_x>|^2, phases from
    overlaps.  F11 gets the cos^2(err/2) controlled-phase penalty in both.
    """
    kets = initial_kets(dim)
    idx = {k: int(np.argmax(np.abs(v))) for k, v in kets.items()}
    mixed = results["01"].ndim == 2
    info: Dict = {}
    fid: Dict[str, float] = {}
    if mixed:
        ph = {}
        for lab in LABELS:
            rho = results[lab]
            w, U = eigh(rho)
            vmax = U[:, int(np.argmax(w))]
            ph[lab] = _angle(vmax[idx[lab]])
            fid[lab] = float(np.real(rho[idx[lab], idx[lab]]))
        cp = ph["11"] - ph["01"] - ph["10"] + ph["00"]
        info.update(phi_01_rad=ph["01"], phi_11_rad=ph["11"], is_mixed_state=True)
    else:
        ov = {lab: complex(results[lab][idx[lab]]) for lab in LABELS}
        for lab in LABELS:
            fid[lab] = float(abs(ov[lab]) ** 2)
        cp = (_angle(ov["11"]) - _angle(ov["01"]) - _angle(ov["10"]) + _angle(ov["00"]))
        info.update(phi_01_rad=_angle(ov["01"]), phi_11_rad=_angle(-ov["11"]),
                    amp_01=abs(ov["01"]), amp_11=abs(ov["11"]), is_mixed_state=False)
    cp = (cp + np.pi) % (2 * np.pi) - np.pi
    err = min(abs(cp - np.pi), abs(cp + np.pi))
    pen = float(np.cos(err / 2) ** 2)
    info.update(controlled_phase_rad=cp, controlled_phase_deg=float(np.degrees(cp)),
                phase_error_from_pi_rad=err, phase_error_from_pi_deg=float(np.degrees(err)),
                cz_phase_fidelity=pen, F11_population=fid["11"])
    fid["11"] = fid["11"] * pen
    info["F11_with_phase"] = fid["11"]
    avg = float(np.mean([fid[k] for k in LABELS]))
    return fid, avg, info


def structural_support(dim: int = 3) -> np.ndarray:
    """Boolean D x D mask of the rho entries the four basis inputs can ever populate.
    H and every c_op conserve each atom's {1, r}-excitation number, so an output rho_x
    lives on e_i (x) e_j with e = {|0><0|, |1><1|, |r><r|, |1><r|, |r><1|} (dim 4: +
    |r-><r-|); everything else is exactly zero in QuTiP's sparse ZVODE integration."""
    single = np.zeros((dim, dim), dtype=bool)
    single[0, 0] = single[1, 1] = single[2, 2] = single[1, 2] = single[2, 1] = True
    if dim == 4:
        single[3, 3] = True
    return np.kron(single, single)


def snap_structural_zeros(rho: np.ndarray, dim: int = 3) -> np.ndarray:
    """rho with the entries outside structural_support set to exactly +0.0 (the dense
    expm propagator leaves ~1e-17 residues there; QuTiP's output has exact zeros)."""
    out = np.array(rho, dtype=complex, copy=True)
    out[~structural_support(dim)] = 0.0
    return out


def _splitmix64(x: int) -> int:
    M = (1 << 64) - 1
    x = (x + 0x9E3779B97F4A7C15) & M
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M
    return x ^ (x >> 31)


def probe_copy(rho: np.ndarray, c: int, x: int, rel_eps: float = 1e-12) -> np.ndarray:
    """Copy c (1-based) of rho_x as the engine's gauge check builds it: every entry of the
    lower triangle (what LAPACK reads) with its real and imaginary parts scaled
    independently by (1 +- rel_eps); copy 1 all +, copy 2 all -, then the signs of
    splitmix64((c << 32) ^ (x << 24) ^ e), e = 2 (row + D col) (bits 0 / 1)."""
    D = rho.shape[0]
    q = rho.copy()
    for col in range(D):
        for row in range(col, D):
            e = 2 * (row + D * col)
            h = _splitmix64((c << 32) ^ (x << 24) ^ e)
            s1 = 1.0 if c == 1 else (-1.0 if c == 2 else (1.0 if h & 1 else -1.0))
            s2 = 1.0 if c == 1 else (-1.0 if c == 2 else (1.0 if h & 2 else -1.0))
            q[row, col] = complex(rho[row, col].real * (1.0 + s1 * rel_eps),
                                  rho[row, col].imag * (1.0 + s2 * rel_eps))
    return np.tril(q) + np.tril(q, -1).conj().T


def gauge_unstable(results: Dict[str, np.ndarray], dim: int = 3, rel_eps: float = 1e-12,
                   copies: int = 64, tol: float = 1e-9, seed: int = 7,
                   scheme: str = "one_rho") -> Tuple[bool, float]:
    """Does the reference's mixed-state penalty (cz_fidelity with scipy.linalg.eigh, the
    eigensolver QuTiP 5 uses) stay put when the real and imaginary parts of the entries
    of rho's lower triangle (what LAPACK reads) are scaled independently by (1 +- rel_eps)?
    Returns (unstable, max |penalty change| over the probes made).  The LAPACK eigenvector
    phase is decided by rounding in the Householder reduction and the tridiagonal
    eigenvector normalisation, so for most noisy points it is not.

    scheme "one_rho" (the engine's ryd_mixed_phase, round 4): probe (x, c) perturbs copy c
    of rho_x alone (probe_copy) with the other three rho unperturbed; rho_11 first, then
    rho_00, rho_01, rho_10, copies 1..copies each; stops at the first probe that moves the
    penalty by more than tol.  scheme "all_at_once" (rounds 1-3; how
    tests/golden/evolution_golden.json's flags were made): copy c perturbs all four rho
    together, copy 1 all +, copy 2 all -, then numpy sign patterns from ``seed``."""
    eigh = lambda m: sla.eigh(m)
    _, _, info0 = cz_fidelity(results, dim, eigh=eigh)
    pen0 = info0["cz_phase_fidelity"]
    spread = 0.0
    if scheme == "one_rho":
        labs = list(LABELS)
        for x in (3, 0, 1, 2):
            for c in range(1, copies + 1):
                pert = dict(results)
                pert[labs[x]] = probe_copy(results[labs[x]], c, x, rel_eps)
                _, _, info = cz_fidelity(pert, dim, eigh=eigh)
                spread = max(spread, abs(info["cz_phase_fidelity"] - pen0))
                if spread > tol:
                    return True, spread
        return False, spread
    if scheme != "all_at_once":
        raise ValueError(f"unknown scheme {scheme!r}")
    rng = np.random.default_rng(seed)
    for c in range(copies):
        pert = {}
        for lab, rho in results.items():
            D = rho.shape[0]
            if c < 2:
                s1 = s2 = np.full((D, D), 1.0 if c == 0 else -1.0)
            else:
                s1 = rng.choice([-1.0, 1.0], size=(D, D))
                s2 = rng.choice([-1.0, 1.0], size=(D, D))
            q = rho.real * (1.0 + rel_eps * s1) + 1j * rho.imag * (1.0 + rel_eps * s2)
            pert[lab] = np.tril(q) + np.tril(q, -1).conj().T
        _, _, info = cz_fidelity(pert, dim, eigh=eigh)
        spread = max(spread, abs(info["cz_phase_fidelity"] - pen0))
    return spread > tol, spread


def decay_kat(gamma: float, t: np.ndarray, method: str = "expm") -> np.ndarray:
    """scripts/archive/test_mesolve_direct.py:34-51: H = 0, one decay op
    sqrt(gamma)|0><1| on a qubit starting in |1>: rho_11(t) = exp(-gamma t)."""
    H = np.zeros((2, 2), dtype=complex)
    c = [math.sqrt(gamma) * np.outer(_ket(2, 0), _ket(2, 1))]
    psi = _ket(2, 1)
    out = []
    for tt in t:
        rho = evolve_state(H, psi, np.array([0.0, tt]), c, method=method)
        out.append(np.real(rho[1, 1]))
    return np.array(out)


# --------------------------------------------------------------------------
# qubit process map.  The reference's Kraus/CPTP extraction
# (src/qpu_simulator/noise_models/__init__.py:1-22) is a stub, so there is no
# reference oracle: these are the textbook definitions the build is checked
# against, on the same exact propagators as run_point.
# --------------------------------------------------------------------------

QUBIT_INDEX = (0, 1, 3, 4)     # |00>, |01>, |10>, |11> in the dim-3 two-atom basis


def process_map(p: PointSpec) -> np.ndarray:
    """S[4c+d, 4a+b] = <c| E(|a><b|) |d>: every qubit matrix unit evolved through the
    full column-stacked Liouvillian of each reference segment (exact expm), projected
    on the qubit block (leakage to |r> is simply lost)."""
    if p.dim != 3:
        raise ValueError("process_map: dim 3 only")
    D = 9
    props = [sla.expm(liouvillian(H, p.c_ops) * float(t[-1])) for H, t, _ in segments(p)]
    S = np.zeros((16, 16), dtype=complex)
    for a in range(4):
        for b in range(4):
            rho = np.zeros((D, D), dtype=complex)
            rho[QUBIT_INDEX[a], QUBIT_INDEX[b]] = 1.0
            v = vec(rho)
            for P in props:
                v = P @ v
            r = unvec(v, D)
            for c in range(4):
                for d in range(4):
                    S[4 * c + d, 4 * a + b] = r[QUBIT_INDEX[c], QUBIT_INDEX[d]]
    return S


def apply_map(S: np.ndarray, X: np.ndarray) -> np.ndarray:
    """E(X) for a 4x4 operator X from the matrix-unit map S."""
    out = np.zeros((4, 4), dtype=complex)
    for a in range(4):
        for b in range(4):
            out += X[a, b] * S[:, 4 * a + b].reshape(4, 4)
    return out


def choi_matrix(S: np.ndarray) -> np.ndarray:
    """J = sum_ab |a><b| (x) E(|a><b|) (input factor first)."""
    J = np.zeros((16, 16), dtype=complex)
    for a in range(4):
        for b in range(4):
            Eab = np.zeros((4, 4), dtype=complex)
            Eab[a, b] = 1.0
            J += np.kron(Eab, apply_map(S, Eab))
    return J


_PAULI1 = (np.eye(2, dtype=complex), np.array([[0, 1], [1, 0]], dtype=complex),
           np.array([[0, -1j], [1j, 0]]), np.array([[1, 0], [0, -1]], dtype=complex))
PAULI2 = [np.kron(P, Q) for P in _PAULI1 for Q in _PAULI1]     # II, IX, ..., ZZ (atom A first)


def pauli_transfer_matrix(S: np.ndarray) -> np.ndarray:
    """R[i, j] = Tr(P_i E(P_j)) / 4."""
    R = np.zeros((16, 16))
    for j, Pj in enumerate(PAULI2):
        EPj = apply_map(S, Pj)
        for i, Pi in enumerate(PAULI2):
            R[i, j] = np.real(np.trace(Pi @ EPj)) / 4
    return R
