"""simulate_CZ_gate on the MI355X engine -- the drop-in for the reference's
point-level contract (RG/simulation.py:2534-3676) and its batched form.

``simulate_CZ_gate``        same signature / SimulationResult as the reference;
                            a batch of one through the engine.
``simulate_CZ_gate_batch``  the sweep form: any apparatus argument may be an
                            array; all points go through ONE engine launch per
                            evolution kind (kets for noise-free points, rho in the
                            25-dim sector otherwise), then the fidelity epilogue.
``compute_CZ_fidelity``     RG/simulation.py:225-633 on numpy states.

Fidelity epilogue.  Noise-free (ket) points: everything (populations, overlap
phases, controlled phase, cos^2 penalty, average) comes from the GPU summary.
Noisy (rho) points: populations come from the GPU; the reference's controlled
phase uses the dominant eigenvector of each 9x9 rho (:424-452), whose phase is
the eigensolver's gauge choice (SURVEY.md §7 hard part 3).  ``phase_penalty``:
  "reference" (default) -- the C-ABI host epilogue ryd_mixed_phase: LAPACK zheevr
                 (scipy's own, QuTiP 5's eigensolver) on every rho, threaded, phases
                 bit-identical to scipy.linalg.eigh + np.angle; with ``gauge_check``
                 each point whose penalty is not a function of rho at 1e-12 relative
                 precision gets RYD_STATUS_GAUGE_UNSTABLE.
                 ``eigh="numpy"`` or a callable: the per-matrix Python path instead;
  "none"       -- gauge-invariant population fidelity only (F11 unpenalised).
Status bits per point: kernel failures (RYD_STATUS_FAIL_MASK) plus the reference's
warnings (weak blockade, dark-state sign, Omega range) and the gauge flag.
"""
from __future__ import annotations

import math
import time
import warnings
from dataclasses import dataclass, field
from types import SimpleNamespace
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np

from . import _native as N
from . import operators as OPS
from . import physics as PH
from .configurations import (AtomicConfiguration, JPSimulationInputs, LPSimulationInputs,
                             SmoothJPSimulationInputs)
from .constants import KB

LABELS = ("00", "01", "10", "11")
_IDX = {"00": 0, "01": 1, "10": 3, "11": 4}        # basis index 3*a1 + a2 (dim 3)
_IDX_DIM = {3: _IDX, 4: {"00": 0, "01": 1, "10": 4, "11": 5}}   # d*a1 + a2


# ---------------------------------------------------------------------------
# fidelity (RG/simulation.py:186-633)
# ---------------------------------------------------------------------------

def _eigh_fn(eigh):
    if eigh is None or eigh == "scipy":
        import scipy.linalg as sla
        return lambda m: sla.eigh(m)
    if eigh == "numpy":
        return np.linalg.eigh
    return eigh


def _wrap(cp):
    return (cp + np.pi) % (2 * np.pi) - np.pi


def _penalty(cp):
    err = np.minimum(np.abs(cp - np.pi), np.abs(cp + np.pi))
    return err, np.cos(err / 2) ** 2


def compute_state_fidelity(psi_out: np.ndarray, psi_target: np.ndarray) -> float:
    """RG/simulation.py:186-222: |<t|psi>|^2 for two kets; otherwise the Uhlmann
    fidelity qutip.fidelity(rho, sigma) = Tr sqrt(sqrt(rho) sigma sqrt(rho)), squared."""
    a, b = np.asarray(psi_out), np.asarray(psi_target)
    if a.ndim == 1 and b.ndim == 1:
        return float(abs(np.vdot(b, a)) ** 2)
    rho = np.outer(a, a.conj()) if a.ndim == 1 else a
    sig = np.outer(b, b.conj()) if b.ndim == 1 else b
    w, V = np.linalg.eigh((rho + rho.conj().T) / 2)
    sq = (V * np.sqrt(np.clip(w, 0, None))) @ V.conj().T
    m = sq @ sig @ sq
    ev = np.linalg.eigvalsh((m + m.conj().T) / 2)
    return float(np.sum(np.sqrt(np.clip(ev, 0, None))) ** 2)


def compute_CZ_fidelity(results: Dict[str, np.ndarray], extract_global_phase: bool = True,
                        hilbert_space_dim: int = 3, eigh=None,
                        phases: Optional[Dict[str, float]] = None) -> Tuple[Dict[str, float], float, Dict]:
    """Per-state fidelities, average and phase_info, as RG/simulation.py:225-633.
    ``phases`` (mixed states): the dominant-eigenvector phases when they are already known
    (ryd_mixed_phase computes them with scipy's own zheevr, bit for bit the values eigh
    would give here), so the four eigendecompositions are not repeated."""
    d = hilbert_space_dim
    idx = {lab: int(np.argmax(np.abs(v))) for lab, v in OPS.basis_kets(d).items()}
    mixed = np.ndim(results["01"]) == 2
    phase_info: Dict[str, Any] = {}
    fid: Dict[str, float] = {}
    if mixed:
        pops = {lab: float(np.real(results[lab][idx[lab], idx[lab]])) for lab in LABELS}
        fid.update(pops)
        if extract_global_phase:
            ph = {}
            if phases is not None:
                ph = {lab: float(phases[lab]) for lab in LABELS}
            else:
                eg = _eigh_fn(eigh)
                for lab in LABELS:
                    try:
                        w, U = eg(results[lab])
                        ph[lab] = float(np.angle(U[idx[lab], int(np.argmax(w))]))
                    except Exception:
                        ph[lab] = 0.0
            cp = float(_wrap(ph["11"] - ph["01"] - ph["10"] + ph["00"]))
            err, pen = _penalty(cp)
            phase_info = {
                "phi_01_rad": ph["01"], "phi_01_deg": np.degrees(ph["01"]),
                "phi_11_rad": ph["11"], "phi_11_deg": np.degrees(ph["11"]),
                "expected_phi_11_rad": -np.pi, "controlled_phase_rad": cp,
                "controlled_phase_deg": np.degrees(cp), "phase_error_from_pi_rad": float(err),
                "phase_error_from_pi_deg": float(np.degrees(err)), "cz_phase_fidelity": float(pen),
                "amp_01": np.sqrt(max(0, pops["01"])), "amp_11": np.sqrt(max(0, pops["11"])),
                "pop_00": pops["00"], "pop_01": pops["01"], "pop_11": pops["11"],
                "is_mixed_state": True,
                "note": "Phase extracted from dominant eigenvector - penalty applied for CZ condition",
            }
    else:
        ov = {lab: complex(results[lab][idx[lab]]) for lab in LABELS}
        for lab in LABELS:
            fid[lab] = float(abs(ov[lab]) ** 2)
        if extract_global_phase:
            phi01 = float(np.angle(ov["01"]))
            phi11 = float(np.angle(-ov["11"]))
            amp11 = abs(ov["11"])
            perr = float(np.arccos(np.clip(amp11, 0, 1)))
            cp = float(_wrap(np.angle(ov["11"]) - np.angle(ov["01"]) - np.angle(ov["10"])
                             + np.angle(ov["00"])))
            err, pen = _penalty(cp)
            phase_info = {
                "phi_01_rad": phi01, "phi_01_deg": np.degrees(phi01),
                "phi_11_rad": phi11, "phi_11_deg": np.degrees(phi11),
                "phi_11_plus_rad": float(np.angle(ov["11"])),
                "phi_11_plus_deg": float(np.degrees(np.angle(ov["11"]))),
                "phase_error_rad": perr, "phase_error_deg": np.degrees(perr),
                "amp_01": abs(ov["01"]), "amp_11": amp11, "is_mixed_state": False,
                "controlled_phase_rad": cp, "controlled_phase_deg": np.degrees(cp),
                "phase_error_from_pi_rad": float(err), "phase_error_from_pi_deg": float(np.degrees(err)),
                "cz_phase_fidelity": float(pen),
            }
    if phase_info:
        pen = phase_info.get("cz_phase_fidelity", 1.0)
        phase_info["F11_population"] = fid["11"]
        phase_info["F11_with_phase"] = fid["11"] * pen
        phase_info["cz_phase_condition_met"] = phase_info.get("phase_error_from_pi_rad", 0) < 0.2
        fid["11"] = fid["11"] * pen
    return fid, float(np.mean([fid[k] for k in LABELS])), phase_info


def _cp_penalty(ph: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """(controlled phase, penalty) from phases ph[n, 4] (00, 01, 10, 11), with the
    reference's operation order (RG/simulation.py:444-452)."""
    cp = ph[:, 3] - ph[:, 1] - ph[:, 2] + ph[:, 0]
    cp = (cp + np.pi) % (2 * np.pi) - np.pi
    err = np.minimum(np.abs(cp - np.pi), np.abs(cp + np.pi))
    # the reference squares a numpy scalar: np.float64 ** 2 is libm pow(x, 2.0), which
    # differs from x * x (numpy's vectorised ** 2) in the last bit for ~0.1% of inputs
    c = np.cos(err / 2).tolist()
    return cp, np.fromiter((math.pow(v, 2.0) for v in c), dtype=np.float64, count=len(c))


def mixed_phase_penalty(rho: np.ndarray, eigh=None) -> Tuple[np.ndarray, np.ndarray]:
    """Vectorised dominant-eigenvector controlled phase for rho[n, 4, D, D] (D = 9 or 16)
    -> (controlled_phase[n], penalty[n])."""
    n, D = rho.shape[0], rho.shape[-1]
    idx = _IDX_DIM[3 if D == 9 else 4]
    ph = np.zeros((n, 4))
    if eigh == "numpy":
        w, U = np.linalg.eigh(rho.reshape(-1, D, D))
        k = np.argmax(w, axis=1)
        vmax = U[np.arange(U.shape[0]), :, k]                    # (4n, D)
        comp = np.array([idx[l] for l in LABELS] * n)
        ph = np.angle(vmax[np.arange(4 * n), comp]).reshape(n, 4)
    else:
        eg = _eigh_fn(eigh)
        for i in range(n):
            for k, lab in enumerate(LABELS):
                w, U = eg(rho[i, k])
                ph[i, k] = np.angle(U[idx[lab], int(np.argmax(w))])
    cp = _wrap(ph[:, 3] - ph[:, 1] - ph[:, 2] + ph[:, 0])
    return cp, _penalty(cp)[1]


# ---------------------------------------------------------------------------
# results
# ---------------------------------------------------------------------------

@dataclass
class SimulationResult:
    """Same fields and properties as RG/simulation.py:2238-2531, with one drop-in
    difference in the types of four fields: the reference fills ``results`` (label ->
    final state), ``H1``, ``H2`` and ``c_ops`` with ``qutip.Qobj`` objects
    (RG/simulation.py:689-690, :3589-3676); here they are numpy ``ndarray``s holding the
    same matrices -- ``results[label]`` a (D, D) complex128 density matrix (noisy runs)
    or a (D,) ket (noise-free runs), ``H1``/``H2`` (D, D) complex128, ``c_ops`` a list
    of (D, D) complex128 -- in the same basis order and QuTiP's dense layout
    (``Qobj.full()`` of the reference's objects).  qutip is not a dependency of this
    package; a caller that needs Qobj methods wraps them with ``qutip.Qobj(arr,
    dims=[[d, d], [d, d]])``.  No caller inside the reference uses Qobj methods on these
    fields."""
    avg_fidelity: float
    fidelities: Dict[str, float]
    phase_info: Dict
    protocol: str
    n_pulses: int
    hilbert_space_dim: int
    Omega: float
    V: float
    Delta: float
    V_over_Omega: float
    tau_single: float
    tau_total: float
    R: float
    Delta_over_Omega: float = 0.0
    xi: complex = 1.0
    spacing_factor: float = 2.8
    U0_mK: float = 0.0
    omega_r_kHz: float = 0.0
    sigma_r_nm: float = 0.0
    trap_wavelength_nm: float = 1064.0
    magic_wavelength_analysis: Dict = None
    noise_breakdown: Dict = None
    include_noise: bool = True
    include_motional_dephasing: bool = True
    pulse_info: Dict = None
    config: AtomicConfiguration = None
    species: str = "Rb87"
    n_rydberg: int = 70
    qubit_0: Tuple[int, int] = (1, 0)
    qubit_1: Tuple[int, int] = (2, 0)
    temperature_K: float = 2e-6
    B_field_T: float = 1e-4
    delta_zeeman: float = 0.0
    delta_stark: float = 0.0
    trap_laser_on: bool = True
    results: Dict = None
    H1: Any = None
    H2: Any = None
    c_ops: List = None
    hs: Any = None
    # not in the reference's record: the gauge-invariant process / average gate fidelity
    # to CZ up to local Z phases (simulate_CZ_gate(..., process_fidelity=True)), None if
    # not requested; unlike avg_fidelity's noisy phase penalty they do not depend on the
    # eigensolver's gauge
    process_fidelity: Optional[float] = None
    avg_gate_fidelity: Optional[float] = None

    def __post_init__(self):
        for k in ("magic_wavelength_analysis", "noise_breakdown", "pulse_info", "results"):
            if getattr(self, k) is None:
                setattr(self, k, {})
        if self.c_ops is None:
            self.c_ops = []

    Omega_MHz = property(lambda s: s.Omega / (2 * np.pi * 1e6))
    V_MHz = property(lambda s: s.V / (2 * np.pi * 1e6))
    Delta_MHz = property(lambda s: s.Delta / (2 * np.pi * 1e6))
    gate_time_us = property(lambda s: s.tau_total * 1e6)
    R_um = property(lambda s: s.R * 1e6)
    xi_rad = property(lambda s: float(np.angle(s.xi)))
    xi_deg = property(lambda s: float(np.degrees(np.angle(s.xi))))
    temperature_uK = property(lambda s: s.temperature_K * 1e6)
    B_field_Gauss = property(lambda s: s.B_field_T * 1e4)

    def print_summary(self):
        print("=" * 70)
        print("CZ GATE SIMULATION RESULTS")
        print("=" * 70)
        print(f"Average fidelity: {self.avg_fidelity:.6f} ({(1 - self.avg_fidelity) * 100:.4f}% error)")
        for state, f in self.fidelities.items():
            print(f"  |{state}⟩ → {f:.6f}")
        print(f"Protocol: {self.protocol}   pulses: {self.n_pulses}   dim: {self.hilbert_space_dim}")
        print(f"Ω/(2π): {self.Omega_MHz:.3f} MHz   V/(2π): {self.V_MHz:.2f} MHz   V/Ω: {self.V_over_Omega:.2f}")
        print(f"Total gate: {self.gate_time_us:.3f} μs   R: {self.R_um:.2f} μm   U0: {self.U0_mK:.2f} mK")
        print("=" * 70)


@dataclass
class BatchResult:
    """SoA outputs of simulate_CZ_gate_batch (one row per point)."""
    batch: PH.DerivedBatch
    avg_fidelity: np.ndarray
    fidelities: np.ndarray            # (n, 4): F00, F01, F10, F11 (F11 penalised)
    populations: np.ndarray           # (n, 4)
    controlled_phase: np.ndarray
    cz_phase_fidelity: np.ndarray
    status: np.ndarray
    is_mixed: np.ndarray
    states: Optional[np.ndarray] = None   # rho (n,4,9,9) or kets (n,4,9) (complex)
    kernel_ms: float = 0.0
    # gauge-invariant figures of merit (``process_fidelity=True``; NaN otherwise, and for
    # dim 4 Lindblad points): process / average gate fidelity to CZ up to local Z phases
    process_fidelity: Optional[np.ndarray] = None
    avg_gate_fidelity: Optional[np.ndarray] = None
    timings: Dict[str, float] = field(default_factory=dict)   # host wall ms per stage
    # (n, 4) dominant-eigenvector phases of the mixed points' rho_00..rho_11 as the reference
    # forms them (ryd_mixed_phase with scipy's zheevr; NaN for kets and host-eigh runs)
    phases: Optional[np.ndarray] = None

    @property
    def n(self):
        return self.batch.n

    @property
    def ok(self) -> np.ndarray:
        """Points the engine evolved without failure (warning bits do not count)."""
        return (self.status & N.STATUS_FAIL_MASK) == 0

    @property
    def gauge_unstable(self) -> np.ndarray:
        return (self.status & N.STATUS_GAUGE_UNSTABLE) != 0

    def __len__(self):
        return self.n

    def point(self, i: int) -> Dict[str, Any]:
        return dict(avg_fidelity=float(self.avg_fidelity[i]),
                    fidelities=dict(zip(LABELS, map(float, self.fidelities[i]))),
                    controlled_phase=float(self.controlled_phase[i]),
                    cz_phase_fidelity=float(self.cz_phase_fidelity[i]),
                    status=int(self.status[i]))


_ENGINES: Dict[Tuple[int, ...], Any] = {}


def _engine(devices=None):
    from .engine import Engine
    key = tuple(devices) if devices is not None else (0,)
    if key not in _ENGINES:
        _ENGINES[key] = Engine(list(key))
    return _ENGINES[key]


def _as_array(x) -> np.ndarray:
    """A dense complex array from an ndarray or a Qobj-like object (anything with .full())."""
    return np.asarray(x.full() if hasattr(x, "full") else x, dtype=np.complex128)


def evolve_state(H, psi0, tlist, c_ops=None, options=None, *, devices=None) -> np.ndarray:
    """The reference's generic time-evolution helper (RG/simulation.py:647-690:
    ``mesolve(H, psi0, tlist, c_ops=c_ops, options=options).states[-1]``) on the GPU
    (``ryd_evolve_generic``): H constant from tlist[0] to tlist[-1], any jump operators.
    Like mesolve, a ket without collapse operators evolves as a ket (its phase kept) and
    otherwise the result is the density matrix.  ``options`` (atol / rtol / nsteps) is
    accepted for signature compatibility and unused: each segment is propagated exactly
    (Chebyshev series, tail < 1e-17).  H, psi0, c_ops: arrays or Qobj-like objects;
    returns an ndarray ((d,) ket or (d, d) density matrix)."""
    del options
    Hm = _as_array(H)
    v = _as_array(psi0)
    if v.ndim == 2 and v.shape != Hm.shape[-2:] and 1 in v.shape:
        v = v.ravel()                       # a Qobj ket's .full() is a (d, 1) column
    tl = np.asarray(tlist, dtype=np.float64)
    T = float(tl[-1] - tl[0]) if tl.size else 0.0
    ops = [_as_array(c) for c in (c_ops or [])]
    return evolve_state_batch(Hm[None], v[None], np.array([T]), [ops] if ops else None, devices=devices)[0]


def evolve_state_batch(H, psi0, T, c_ops=None, *, devices=None) -> np.ndarray:
    """Many independent evolve_state problems in one launch.  H (n, d, d) or, for
    piecewise-constant schedules, (n, n_seg, d, d) with T (n, n_seg) segment lengths;
    psi0 (n, d) kets or (n, d, d) density matrices; c_ops None or (n, K, d, d) (or a list of
    per-problem lists of K operators).  Kets with c_ops are evolved as |psi><psi|.  Raises
    EngineError for a failed problem (step cap: omega * dt > 2e6 rad in one segment;
    non-finite) and ValueError for inputs this engine does not evolve: a segment length
    that is negative or not finite, and a Hamiltonian that is not finite or not Hermitian
    (to 1e-12 of its largest entry).  The reference's mesolve WOULD evolve a non-Hermitian
    H through its Liouvillian; this engine does not support it (its Gershgorin series
    bound assumes a real diagonal), so such inputs are refused rather than evolved
    inexactly.  Column kets (n, d, 1) are taken as kets."""
    from ._native import EngineError, STATUS_FAIL_MASK
    H = np.asarray(H, dtype=np.complex128)
    if H.ndim == 3:
        H = H[:, None]
    n, n_seg, d = H.shape[0], H.shape[1], H.shape[2]
    T = np.asarray(T, dtype=np.float64).reshape(n, -1)
    if T.shape[1] != n_seg:
        raise ValueError("T must hold one length per segment")
    if not np.all(np.isfinite(T)) or np.any(T < 0):
        raise ValueError("segment lengths must be finite and non-negative")
    scale = np.abs(H).max(axis=(2, 3), initial=0.0)
    if not np.all(np.isfinite(H)) or np.any(np.abs(H - np.conj(np.swapaxes(H, 2, 3))).max(axis=(2, 3), initial=0.0)
                                            > 1e-12 * scale):
        raise ValueError("H must be finite and Hermitian: this engine does not evolve a non-Hermitian H "
                         "(the reference's mesolve would, through its Liouvillian)")
    v = np.asarray(psi0, dtype=np.complex128)
    if v.ndim == 3 and v.shape[1:] in ((d, 1), (1, d)) and d > 1:
        v = v.reshape(n, d)
    ops = None
    if c_ops is not None and len(c_ops) > 0:
        ops = np.asarray(c_ops, dtype=np.complex128)
        if ops.ndim == 3:
            ops = ops[None]
        if ops.shape[1] == 0:
            ops = None
    if ops is not None and v.ndim == 2:                     # mesolve: a ket with c_ops -> rho
        v = np.einsum("ni,nj->nij", v, v.conj())
    out, status = _engine(devices).evolve_generic(H, T, v, ops)
    bad = np.nonzero(status & STATUS_FAIL_MASK)[0]
    if bad.size:
        raise EngineError(f"evolve_state: problem {int(bad[0])} failed (status {int(status[bad[0]])})")
    return out


# gauge-check probes of the batch API, counted PER RHO (round 4 scheme: probe (x, c) perturbs
# rho_x alone, rho_11 first, so `copies` = 4 means up to 16 zheevr calls per point, and an
# unstable point stops at its first moving probe); the optimiser and sweep drivers use the
# same 4, direct engine.mixed_phase calls engine.GAUGE_COPIES.  Miss rates under this scheme
# on a 300-point sample of the C2 grid (all 300 unstable at 64 probes; tools/gauge_miss_rate.py,
# profiles/r05/gauge_miss_rate.json): 1 probe per rho misses 14.7 %, 2 miss 1.7 %, 4 and more
# none.  Ask for more with gauge_copies when the flag itself is the result being studied.
BATCH_GAUGE_COPIES = 4

# simulate_CZ_gate_batch's pipeline: up to PIPELINE_CHUNKS chunks of at least
# PIPELINE_MIN_CHUNK points when the native epilogue runs (fewer points: one chunk)
PIPELINE_CHUNKS = 4
PIPELINE_MIN_CHUNK = 2048


def simulate_CZ_gate_batch(simulation_inputs, n: Optional[int] = None, *, species="Rb87",
                           n_rydberg=70, qubit_0=(1, 0), qubit_1=(2, 0), hilbert_space_dim: int = 3,
                           tweezer_power=30e-3, tweezer_waist=1.0e-6, tweezer_wavelength_nm=None,
                           temperature=2e-6, B_field=1e-4, NA=0.5, spacing_factor=2.8,
                           include_noise: bool = True, background_loss_rate_hz=None,
                           trap_laser_on: bool = True, overrides: Optional[Dict[str, Any]] = None,
                           phase_penalty: str = "reference", eigh=None, return_states: bool = False,
                           devices=None, method: str = "chebyshev", gauge_check: bool = True,
                           gauge_copies: Optional[int] = None, process_fidelity: bool = False) -> BatchResult:
    """Evaluate many simulate_CZ_gate points in one GPU pass (see module doc).

    ``process_fidelity``: also compute the gauge-invariant process fidelity and average
    gate fidelity to CZ up to local Z phases (noise_models.gate_fidelity) -- from the
    kets for noise-free points, from the Lindblad state plus one ryd_run_coherences pass
    (the 6 qubit coherences) for noisy dim-3 points."""
    if hilbert_space_dim not in (3, 4):
        raise ValueError(f"Unsupported Hilbert space dimension: {hilbert_space_dim}. Use 3 or 4.")
    dim = hilbert_space_dim
    D = dim * dim
    from concurrent.futures import ThreadPoolExecutor
    from . import engine as E
    t_start = time.perf_counter()
    dkw = dict(species=species, n_rydberg=n_rydberg, qubit_0=qubit_0, qubit_1=qubit_1,
               hilbert_space_dim=hilbert_space_dim, tweezer_power=tweezer_power,
               tweezer_waist=tweezer_waist, tweezer_wavelength_nm=tweezer_wavelength_nm,
               temperature=temperature, B_field=B_field, NA=NA, spacing_factor=spacing_factor,
               include_noise=include_noise, background_loss_rate_hz=background_loss_rate_hz,
               trap_laser_on=trap_laser_on, overrides=overrides)
    nn = n if n is not None else PH.batch_size(**{k: v for k, v in dkw.items()
                                                   if k in PH.POINT_ARGS or k == "overrides"})
    host_eigh = phase_penalty == "reference" and eigh not in (None, "scipy")
    native_epilogue = phase_penalty == "reference" and not host_eigh
    # chunks: derivation and the GPU pass of chunk k + 1 run on this thread while the host
    # LAPACK epilogue of chunk k runs on its pool (one ryd_mixed_phase call at a time, in
    # chunk order; each rho's zheevr calls are the same as in one call, so the phases and
    # flags are too).  The derivation is elementwise, so the chunks' columns are the
    # whole call's (tests/test_pipeline_cpu.py).
    k = min(PIPELINE_CHUNKS, nn // PIPELINE_MIN_CHUNK) if native_epilogue else 1
    bounds = [(0, nn)]
    if k > 1:
        # the first chunk is half the others: the epilogue pool starts sooner
        f = nn // (2 * k - 1)
        bounds = [(0, f)] + [(f + (nn - f) * c // (k - 1), f + (nn - f) * (c + 1) // (k - 1)) for c in range(k - 1)]
    fids = np.zeros((nn, 4))
    pops = np.zeros((nn, 4))
    cp = np.full(nn, np.nan)
    pen = np.ones(nn)
    fpro = np.full(nn, np.nan)
    fgate = np.full(nn, np.nan)
    phases = np.full((nn, 4), np.nan)
    status = np.zeros(nn, np.uint32)
    ket_all = np.zeros(nn, bool)
    states = None
    if return_states:
        states = {"ket": np.zeros((nn, 4, D), complex), "rho": np.zeros((nn, 4, D, D), complex)}
    eng = _engine(devices)
    kms = 0.0
    derive_s = engine_s = 0.0
    parts: List[PH.DerivedBatch] = []
    pending = []                                    # (rows, future) of the epilogue calls
    copies = gauge_copies if gauge_copies is not None else BATCH_GAUGE_COPIES

    def epilogue(st, m):
        t0 = time.perf_counter()
        out = E.mixed_phase(st, m, dim, gauge_check=gauge_check, copies=copies)
        return out, time.perf_counter() - t0

    with ThreadPoolExecutor(max_workers=1) as ex:
        for lo, hi in bounds:
            t0 = time.perf_counter()
            b = PH.derive_batch(simulation_inputs, hi - lo, **(PH.slice_inputs(dkw, nn, lo, hi) if k > 1 else dkw))
            derive_s += time.perf_counter() - t0
            parts.append(b)
            key = E.protocol_key(b)
            shape = b.pulse_shape.lower() if key == "lp_shaped" else "square"
            g = b.channel_rates()
            # mesolve with an empty c_op list evolves kets (RG/simulation.py:683-690)
            ket_mask = (np.all([x == 0 for x in g], axis=0) & (b.mj_rate() == 0)) if include_noise \
                else np.ones(b.n, bool)
            ket_all[lo:hi] = ket_mask
            if b.status_bits is not None:
                status[lo:hi] |= b.status_bits
            for evol, mask in (("ket", ket_mask), ("lindblad", ~ket_mask)):
                loc = np.nonzero(mask)[0]
                if loc.size == 0:
                    continue
                idx = lo + loc
                t0 = time.perf_counter()
                prm = E.pack_params(b, loc)
                r = eng.run(prm, key, evol, shape=shape, method=method if dim == 3 else "chebyshev", dim=dim)
                coh = None
                if process_fidelity and evol == "lindblad" and dim == 3:
                    coh, cst = eng.run_coherences(prm, key, shape=shape)
                    status[idx] |= cst
                engine_s += time.perf_counter() - t0
                if process_fidelity and (evol == "ket" or coh is not None):
                    from . import noise_models as NM
                    S = NM.ket_maps(r.kets(), dim) if evol == "ket" else NM.assemble_maps(r.state, coh)
                    fpro[idx], fgate[idx] = NM.gate_fidelity(S)
                kms += r.kernel_ms
                status[idx] |= r.status
                pops[idx] = r.populations()
                if evol == "ket":
                    cp[idx] = r.col("CTRL_PHASE")
                    pen[idx] = r.col("PENALTY")
                    if return_states:
                        states["ket"][idx] = r.kets()
                    continue
                if native_epilogue:
                    pending.append((idx, ex.submit(epilogue, r.state, idx.size)))
                if return_states or host_eigh:
                    for s0 in range(0, idx.size, 65536):
                        sl = slice(s0, s0 + 65536)
                        rho = E.expand_rho(r.state[:, 4 * s0:4 * (s0 + 65536)], min(65536, idx.size - s0), dim)
                        if host_eigh:
                            cp[idx[sl]], pen[idx[sl]] = mixed_phase_penalty(rho, eigh)
                        if return_states:
                            states["rho"][idx[sl]] = rho
        b = PH.concat_batches(parts)                # (while the last epilogue runs)
        epi_s = 0.0
        for idx, fut in pending:
            (ph, gflags), dt = fut.result()
            epi_s += dt
            cp[idx], pen[idx] = _cp_penalty(ph)
            phases[idx] = ph
            status[idx] |= gflags
    fids[:] = pops
    fids[:, 3] = pops[:, 3] * pen
    avg = fids.mean(axis=1)
    t_end = time.perf_counter()
    # derive / engine / epilogue: each stage's own time (they overlap when chunked);
    # total: the call's wall clock
    timings = {"derive_ms": derive_s * 1e3, "engine_ms": engine_s * 1e3,
               "epilogue_ms": (epi_s if native_epilogue else t_end - t_start - derive_s - engine_s) * 1e3,
               "total_ms": (t_end - t_start) * 1e3, "chunks": len(bounds)}
    return BatchResult(batch=b, avg_fidelity=avg, fidelities=fids, populations=pops,
                       controlled_phase=cp, cz_phase_fidelity=pen, status=status,
                       is_mixed=~ket_all, states=states, kernel_ms=kms, timings=timings,
                       process_fidelity=fpro, avg_gate_fidelity=fgate, phases=phases)


def noise_breakdown_row(b: PH.DerivedBatch, i: int, n_collapse_ops: Optional[int] = None) -> Dict[str, Any]:
    """SimulationResult.noise_breakdown of point i of a derived batch
    (RG/simulation.py:3230-3334 and the dict it returns)."""
    c = {k: (v[i] if np.ndim(v) > 0 else v) for k, v in b.cols.items()}
    motional = b.noise_config.include_motional_dephasing if b.noise_config is not None else True
    nb = {"total_decay_rate": 0.0, "total_dephasing_rate": 0.0, "total_loss_rate": 0.0,
          "n_collapse_ops": 0, "motional_dephasing_included": motional,
          "gamma_scatter_intermediate": c["g_scatter"], "Omega1_MHz": c["Omega1"] / (2 * np.pi * 1e6)}
    if not b.include_noise:
        return nb
    rates = {k: c[k] for k in PH.RATE_FIELDS}
    if n_collapse_ops is None:
        n_collapse_ops = len(OPS.collapse_operators(rates, b.dim))
    gphi = rates["gamma_phi_laser"] + rates["gamma_phi_thermal"] + rates["gamma_phi_zeeman"]
    nb.update(rates)
    nb.update(
        branching_1=0.5, gamma_phi_total=gphi, total_decay_rate=rates["gamma_r"] + rates["gamma_bbr"],
        total_dephasing_rate=gphi,
        total_loss_rate=rates["gamma_loss_antitrap"] + rates["gamma_loss_background"] + rates["gamma_leakage"],
        dim=b.dim, n_collapse_ops=n_collapse_ops,
        gamma_blockade_fluct=c["g_thermal"] if motional else 0.0,
        gamma_doppler=c["g_doppler"], gamma_intensity_noise=c["g_intensity"],
        gamma_thermal_total=rates["gamma_phi_thermal"],
        delta_V_over_V_percent=c["dVV"] * 100, anti_trap_time_factor=c.get("anti_trap_time_factor", 0.0),
        magic_enhancement=c["enhancement"], alpha_ratio=c["alpha_ratio"],
        k_eff_rad_per_m=c["k_eff"], v_thermal_m_per_s=c["v_thermal"],
        gamma_mJ_leakage=rates["mJ_leakage_rate"])
    return nb


def _protocol_name(protocol: str) -> str:
    return {"levine_pichler": "levine_pichler", "smooth_jp": "smooth_jp",
            "jandura_pupillo": "jandura_pupillo"}[protocol]


def simulate_CZ_gate(
    simulation_inputs: Union[LPSimulationInputs, JPSimulationInputs, SmoothJPSimulationInputs],
    config: AtomicConfiguration = None, species: str = "Rb87", n_rydberg: int = 70,
    qubit_0: Tuple[int, int] = (1, 0), qubit_1: Tuple[int, int] = (2, 0),
    hilbert_space_dim: int = 3, tweezer_power: float = 30e-3, tweezer_waist: float = 1.0e-6,
    tweezer_wavelength_nm: float = None, temperature: float = 2e-6, B_field: float = 1e-4,
    NA: float = 0.5, spacing_factor: float = 2.8, include_noise: bool = True,
    background_loss_rate_hz: float = None, trap_laser_on: bool = True, verbose: bool = False,
    return_dataclass: bool = True, *, eigh=None, process_fidelity: bool = False,
) -> Union[SimulationResult, Dict]:
    """Drop-in for RG/simulation.py:2534 (same arguments, same outputs) on the GPU engine.
    ``process_fidelity=True`` also fills the gauge-invariant ``process_fidelity`` and
    ``avg_gate_fidelity`` (dim 3; noise-free points in dim 4)."""
    if config is None:
        config = AtomicConfiguration(species=species, qubit_0=qubit_0, qubit_1=qubit_1,
                                     n_rydberg=n_rydberg, L_rydberg="S")
    br = simulate_CZ_gate_batch(
        simulation_inputs, 1, species=config.species, n_rydberg=config.n_rydberg,
        qubit_0=config.qubit_0, qubit_1=config.qubit_1, hilbert_space_dim=hilbert_space_dim,
        tweezer_power=tweezer_power, tweezer_waist=tweezer_waist,
        tweezer_wavelength_nm=tweezer_wavelength_nm, temperature=temperature, B_field=B_field,
        NA=NA, spacing_factor=spacing_factor, include_noise=include_noise,
        background_loss_rate_hz=background_loss_rate_hz, trap_laser_on=trap_laser_on,
        phase_penalty="reference", eigh=eigh, return_states=True, process_fidelity=process_fidelity)
    if not br.ok[0]:
        raise RuntimeError(f"GPU engine failed for this point (status bits {int(br.status[0])})")
    b = br.batch
    c = {k: (v[0] if np.ndim(v) > 0 else v) for k, v in b.cols.items()}
    mixed = bool(br.is_mixed[0])
    st = br.states["rho" if mixed else "ket"][0]
    results = {lab: st[k] for k, lab in enumerate(LABELS)}
    known = None
    if mixed and br.phases is not None and np.all(np.isfinite(br.phases[0])):
        known = dict(zip(LABELS, br.phases[0]))        # the epilogue's scipy-zheevr phases
    fidelities, avg, phase_info = compute_CZ_fidelity(results, True, hilbert_space_dim, eigh=eigh, phases=known)
    protocol = b.protocol
    is_lp = protocol == "levine_pichler"
    d1 = c["delta_zeeman"] + (c["delta_stark"] if trap_laser_on else 0.0)
    H1 = H2 = None
    xi = 1.0
    if is_lp:
        xi = complex(c["xi_re"], c["xi_im"])
        H1 = OPS.hamiltonian(c["Omega"], c["Delta_gate"], c["V"], hilbert_space_dim, d1)
        H2 = OPS.hamiltonian(c["Omega"] * xi, c["Delta_gate"], c["V"], hilbert_space_dim, d1)
    rates = {k: c[k] for k in PH.RATE_FIELDS}
    c_ops = OPS.collapse_operators(rates, hilbert_space_dim) if include_noise else []
    noise_breakdown = noise_breakdown_row(b, 0, len(c_ops))
    A0 = 0.529e-10
    from .constants import EPS0
    au = 4 * np.pi * EPS0 * A0 ** 3
    magic = {"alpha_ratio": c["alpha_ratio"], "alpha_ground_au": c["alpha_g"] / au,
             "alpha_rydberg_au": c["alpha_r"] / au, "gamma_antitrap_Hz": c["g_antitrap_raw"],
             "differential_shift_Hz": c["diff_shift"], "magic_enhancement": c["enhancement"],
             "wavelength_nm": c["wavelength_nm"]}
    if protocol == "levine_pichler":
        pulse_info = {"shape": b.pulse_shape, "implementation": "constant_hamiltonian"}
        n_pulses = 2
    elif protocol == "smooth_jp":
        pulse_info = {"shape": "smooth_sinusoidal", "implementation": "time_dependent_hamiltonian",
                      "protocol_variant": "bluvstein_evered_dark_state", "A": c["A"],
                      "omega_mod_ratio": c["omega_mod"] / c["Omega"], "phi_offset": c["phi_offset"],
                      "delta_over_omega": c["smooth_delta_over_omega"]}
        n_pulses = 1
    else:
        pulse_info = {"shape": "bangbang", "implementation": "piecewise_constant_hamiltonian",
                      "protocol_variant": "jandura_pupillo_bangbang",
                      "switching_times": list(b.bangbang_times[0]), "phases": list(b.bangbang_phases[0]),
                      "n_segments": b.bangbang_phases.shape[1], "omega_tau": c["omega_tau"]}
        n_pulses = 1
    pulse_info.update(delta_zeeman=c["delta_zeeman"], delta_stark=c["delta_stark"] if trap_laser_on else 0.0,
                      trap_laser_on=trap_laser_on)
    hs = SimpleNamespace(dim=hilbert_space_dim, basis=OPS.basis_kets(hilbert_space_dim))
    rd = dict(
        avg_fidelity=avg, fidelities=fidelities, phase_info=phase_info,
        protocol=_protocol_name(protocol), n_pulses=n_pulses, hilbert_space_dim=hilbert_space_dim,
        Omega=c["Omega"], V=c["V"], Delta=c["Delta_gate"], V_over_Omega=c["V_over_Omega"],
        Delta_over_Omega=c["delta_over_omega"], tau_single=c["tau_single"], tau_total=c["tau_total"],
        xi=xi, R=c["R"], spacing_factor=spacing_factor, U0_mK=c["U0"] / KB * 1e3,
        omega_r_kHz=c["omega_r"] / (2 * np.pi * 1e3), sigma_r_nm=c["sigma_r"] * 1e9,
        trap_wavelength_nm=c["wavelength_nm"], magic_wavelength_analysis=magic,
        noise_breakdown=noise_breakdown, include_noise=include_noise,
        include_motional_dephasing=simulation_inputs.noise.include_motional_dephasing, pulse_info=pulse_info,
        config=config, species=config.species, n_rydberg=config.n_rydberg, qubit_0=config.qubit_0,
        qubit_1=config.qubit_1, temperature_K=temperature, B_field_T=B_field,
        delta_zeeman=c["delta_zeeman"], delta_stark=c["delta_stark"] if trap_laser_on else 0.0,
        trap_laser_on=trap_laser_on, results=results, H1=H1, H2=H2, c_ops=c_ops, hs=hs)
    if process_fidelity and np.isfinite(br.process_fidelity[0]):
        rd.update(process_fidelity=float(br.process_fidelity[0]),
                  avg_gate_fidelity=float(br.avg_gate_fidelity[0]))
    if verbose:
        print(f"  V/Ω = {rd['V_over_Omega']:.1f}; τ_total = {rd['tau_total'] * 1e6:.3f} µs; "
              f"avg F = {avg:.6f}")
    if return_dataclass:
        return SimulationResult(**rd)
    rd.update(Omega_rad_per_s=rd["Omega"], Omega_MHz=rd["Omega"] / (2 * np.pi * 1e6),
              V_rad_per_s=rd["V"], V_MHz=rd["V"] / (2 * np.pi * 1e6), Delta_rad_per_s=rd["Delta"],
              Delta_MHz=rd["Delta"] / (2 * np.pi * 1e6),
              xi_rad=float(np.angle(xi)) if n_pulses == 2 else 0.0,
              xi_deg=float(np.degrees(np.angle(xi))) if n_pulses == 2 else 0.0,
              tau_single_us=rd["tau_single"] * 1e6, tau_total_us=rd["tau_total"] * 1e6,
              gate_time_us=rd["tau_total"] * 1e6, R_meters=rd["R"], R_um=rd["R"] * 1e6,
              temperature_uK=temperature * 1e6, B_field_Gauss=B_field * 1e4)
    return rd
