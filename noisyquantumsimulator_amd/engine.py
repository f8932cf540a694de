"""Batched evolution engine: the host side of the ryd_engine C-ABI.

``Engine.run`` is the batched replacement for every ``evolve_state`` /
``qutip.mesolve`` call the reference evolvers make
(RG/simulation.py:647-2231): one call propagates all 4 computational-basis
inputs of every parameter point through every segment of the protocol.

State rows come back in the compact sector form of include/ryd_engine.h;
``expand_rho`` / ``expand_ket`` rebuild the QuTiP-layout 9x9 density matrices
(structural zeros exact) and kets for the fidelity epilogue and callers that
want ``SimulationResult.results``.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Any, Dict, Optional, Sequence, Tuple

import numpy as np

from . import _native as N
from .physics import DerivedBatch

def _sector_basis(d: int) -> np.ndarray:
    """Single-atom Hermitian basis of the sector: e00, e11, err, ex, ey (dim 3), plus
    e-- = |r-><r-| (dim 4, where r = r+)."""
    E = np.zeros((5 if d == 3 else 6, d, d), dtype=complex)
    E[0, 0, 0] = E[1, 1, 1] = E[2, 2, 2] = 1
    E[3, 1, 2] = E[3, 2, 1] = 1
    E[4, 1, 2], E[4, 2, 1] = 1j, -1j
    if d == 4:
        E[5, 3, 3] = 1
    # B[k i + j] = e_i (x) e_j  (atom 1 = slow index, as qutip.tensor)
    k = E.shape[0]
    return np.stack([np.kron(E[i], E[j]) for i in range(k) for j in range(k)]).reshape(k * k, d ** 4)


_BFLAT = {3: _sector_basis(3), 4: _sector_basis(4)}


def expand_rho(state: np.ndarray, n: int, dim: int = 3) -> np.ndarray:
    """Compact Lindblad rows (25 or 36, >=4n) -> rho[n, 4, D, D] (complex128), D = dim^2."""
    B = _BFLAT[dim]
    R = np.ascontiguousarray(state[:B.shape[0], :4 * n].T)     # (4n, 25 | 36)
    D = dim * dim
    return (R @ B).reshape(n, 4, D, D)


def expand_ket(state: np.ndarray, n: int, dim: int = 3) -> np.ndarray:
    """Ket rows (2 D, >=4n) -> psi[n, 4, D] (complex128)."""
    D = dim * dim
    s = state[:2 * D, :4 * n]
    return (s[0::2] + 1j * s[1::2]).T.reshape(n, 4, D)


GAUGE_REL_EPS = 1e-12       # relative perturbation of the sector coordinates (gauge check)
GAUGE_TOL = 1e-9            # penalty change that flags RYD_STATUS_GAUGE_UNSTABLE
GAUGE_COPIES = 16          # probes (an unstable point usually stops after a few); see ryd_mixed_phase


def mixed_phase(state: np.ndarray, n: int, dim: int = 3, gauge_check: bool = True,
                n_threads: int = 0, rel_eps: float = GAUGE_REL_EPS, tol: float = GAUGE_TOL,
                copies: int = GAUGE_COPIES) -> Tuple[np.ndarray, np.ndarray]:
    """The reference's mixed-state controlled phase (RG/simulation.py:424-452) for every
    point of a Lindblad state block (sector rows, >= 4n columns), through the C-ABI host
    epilogue ryd_mixed_phase on scipy's own LAPACK zheevr (so each phase equals
    scipy.linalg.eigh's -- QuTiP 5's eigensolver -- on the same rho).  Returns
    (phases[n, 4], flags[n]): phi_x = np.angle(<x|v_max>) exactly as the reference forms
    it, and RYD_STATUS_GAUGE_UNSTABLE where the penalty is not a function of rho at
    relative precision rel_eps."""
    lib = N.load()
    if n_threads <= 0:          # the GPU box's CPU share is 16 cores per GPU (os.cpu_count() shows more)
        n_threads = int(os.environ.get("RYD_HOST_THREADS", min(16, os.cpu_count() or 1)))
    pool = N.lapack_pool_copies(n_threads)
    if n_threads > 1 and n >= 64 and pool > 1:
        N.scipy_lapack_pool(pool)
    st = np.ascontiguousarray(state, dtype=np.float64)
    out = np.zeros((N.MP_WIDTH, max(n, 1)), dtype=np.float64)
    flags = np.zeros(max(n, 1), dtype=np.uint32)
    dptr = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    N.check(lib.ryd_mixed_phase(N.scipy_zheevr(), dim, dptr(st), n, st.shape[1],
                                copies if gauge_check else 0, rel_eps, tol, n_threads,
                                dptr(out), out.shape[1], flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))
    v = out[N.MP["V0"]:N.MP["V0"] + 8:2, :n] + 1j * out[N.MP["V0"] + 1:N.MP["V0"] + 8:2, :n]
    return np.angle(v).T.copy(), flags[:n]


@dataclass
class EngineResult:
    evolution: str
    n: int
    state: np.ndarray       # (width, 4n)
    summary: np.ndarray     # (NSUMMARY, n)
    status: np.ndarray      # (n,) uint32
    kernel_ms: float
    h2d_ms: float
    d2h_ms: float
    matvec_useful: float
    matvec_exec: float
    dim: int = 3

    def col(self, name: str) -> np.ndarray:
        return self.summary[N.S[name]]

    def populations(self) -> np.ndarray:
        return self.summary[N.S["POP0"]:N.S["POP0"] + 4].T

    def rho(self) -> np.ndarray:
        assert self.evolution == "lindblad"
        return expand_rho(self.state, self.n, self.dim)

    def kets(self) -> np.ndarray:
        assert self.evolution == "ket"
        return expand_ket(self.state, self.n, self.dim)


def protocol_key(batch: DerivedBatch) -> str:
    if batch.protocol == "levine_pichler":
        shape = batch.pulse_shape.lower()
        if shape == "square":
            return "lp_square"
        if shape == "drag":
            # RG/simulation.py:2170 -> area_correction_factor('drag') -> envelope without Delta_leak
            raise TypeError("pulse_envelope_drag() missing 1 required positional argument: 'Delta_leak'")
        if shape not in N.SHAPE:
            raise ValueError(f"Unknown pulse shape: {batch.pulse_shape}. "
                             f"Available shapes: ['square', 'gaussian', 'cosine', 'blackman', 'drag']")
        return "lp_shaped"
    if batch.protocol == "smooth_jp":
        return "smooth_jp"
    return "bangbang"


def pack_params(batch: DerivedBatch, idx: Optional[np.ndarray] = None) -> np.ndarray:
    """DerivedBatch -> SoA parameter block (NPARAM, n) for the kernel."""
    sel = slice(None) if idx is None else idx
    c = batch.cols
    n = batch.n if idx is None else len(idx)
    p = np.zeros((N.NPARAM, n), dtype=np.float64)
    P = N.P
    p[P["OMEGA"]] = c["Omega"][sel]
    p[P["DELTA"]] = c["Delta_seg"][sel]
    p[P["V"]] = c["V"][sel]
    p[P["DELTA1"]] = (c["delta_zeeman"] + (c["delta_stark"] if batch.trap_laser_on else 0.0))[sel]
    g1, g0, gphi, gsc = (g[sel] for g in batch.channel_rates())
    for key, g in (("G1", g1), ("G0", g0), ("GPHI", gphi), ("GSC", gsc)):
        p[P[key + "_A"]] = g
        p[P[key + "_B"]] = g
    if batch.dim == 4:
        gm = batch.mj_rate()[sel]
        p[P["GMJ_A"]] = gm
        p[P["GMJ_B"]] = gm
    key = protocol_key(batch)
    if key in ("lp_square", "lp_shaped"):
        p[P["TAU"]] = c["tau_single"][sel]
        p[P["XI_RE"]] = c["xi_re"][sel]
        p[P["XI_IM"]] = c["xi_im"][sel]
        if key == "lp_shaped":
            from .physics import area_correction_factor
            p[P["AREA_CORR"]] = area_correction_factor(batch.pulse_shape.lower(), c["tau_single"][sel])
    elif key == "smooth_jp":
        p[P["TAU"]] = c["tau_total"][sel]
        p[P["A"]] = c["A"][sel]
        p[P["OMEGA_MOD"]] = c["omega_mod"][sel]
        p[P["PHI_OFF"]] = c["phi_offset"][sel]
    else:
        t = batch.bangbang_times[sel]
        ph = batch.bangbang_phases[sel]
        nseg = ph.shape[1]
        if nseg > 8:
            raise ValueError("bang-bang schedules with more than 8 segments are not supported")
        p[P["OMEGA_TAU"]] = c["omega_tau"][sel]
        p[P["NSEG"]] = nseg
        p[P["SWT0"]:P["SWT0"] + nseg - 1] = t.T
        p[P["PHI0"]:P["PHI0"] + nseg] = ph.T
    return p


def make_desc(protocol: str, evolution: str, n_steps: int = 0, shape: str = "square",
              symmetric: bool = True, method: str = "chebyshev", dim: int = 3,
              rtol: float = 1e-10, atol: float = 1e-12, max_steps: int = 10 ** 7) -> N.BatchDesc:
    d = N.BatchDesc()
    d.abi_version = N.RYD_ABI_VERSION
    d.dim = dim
    d.protocol = N.PROTO[protocol]
    d.evolution = N.EVOL[evolution]
    d.method = N.METHOD[method]
    d.shape = N.SHAPE[shape]
    d.n_steps = n_steps
    d.flags = N.FLAG_SYMMETRIC_ATOMS if symmetric else 0
    d.rtol, d.atol, d.max_steps = rtol, atol, max_steps
    return d


def default_n_steps(protocol: str, params: np.ndarray) -> int:
    if protocol == "smooth_jp":
        return 300                       # RG/simulation.py:3496
    if protocol == "lp_shaped":
        return 500                       # evolve_shaped_pulse n_time_steps (:2113)
    if protocol == "bangbang":
        return int(params[N.P["NSEG"]].max()) if params.shape[1] else 1
    return 0


def symmetric_atoms(params: np.ndarray) -> bool:
    P = N.P
    return all(np.array_equal(params[P[k + "_A"]], params[P[k + "_B"]])
               for k in ("G1", "G0", "GPHI", "GSC", "GMJ"))


def device_count() -> int:
    """GPUs visible to the HIP runtime (ryd_device_count)."""
    lib = N.load()
    cnt = ctypes.c_int(0)
    N.check(lib.ryd_device_count(ctypes.byref(cnt)))
    return cnt.value


class Engine:
    """A handle on one or more GPUs (points are range-partitioned across them)."""

    def __init__(self, devices: Optional[Sequence[int]] = None):
        self.lib = N.load()
        cnt = ctypes.c_int(0)
        N.check(self.lib.ryd_device_count(ctypes.byref(cnt)))
        if cnt.value == 0:
            raise N.EngineError("no GPU visible to the HIP runtime")
        devs = list(devices) if devices is not None else [0]
        arr = (ctypes.c_int * len(devs))(*devs)
        h = ctypes.c_void_p()
        N.check(self.lib.ryd_create(arr, len(devs), ctypes.byref(h)))
        self.handle = h
        self.devices = devs

    def close(self):
        if getattr(self, "handle", None):
            self.lib.ryd_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, params: np.ndarray, protocol: str, evolution: str, n_steps: Optional[int] = None,
            shape: str = "square", method: str = "chebyshev", rtol: float = 1e-10,
            atol: float = 1e-12, max_steps: int = 10 ** 7, dim: int = 3) -> EngineResult:
        params = np.ascontiguousarray(params, dtype=np.float64)
        if params.shape[0] != N.NPARAM:
            raise ValueError(f"params must have shape ({N.NPARAM}, n)")
        n = params.shape[1]
        if n_steps is None:
            n_steps = default_n_steps(protocol, params)
        desc = make_desc(protocol, evolution, n_steps, shape, symmetric_atoms(params), method,
                         dim=dim, rtol=rtol, atol=atol, max_steps=max_steps)
        w = N.STATE_WIDTH_DIM[dim][evolution]
        # every kernel writes every state row and summary column of every point, so the
        # outputs need no zero fill (np.zeros of the 8 MB C2 state costs ~0.3 ms of page
        # zeroing per call; tools/unpack_probe.py)
        state = np.empty((w, 4 * n), dtype=np.float64)
        summ = np.empty((N.NSUMMARY, n), dtype=np.float64)
        status = np.zeros(n, dtype=np.uint32)
        st = N.Stats()
        dptr = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        N.check(self.lib.ryd_run_batch(
            self.handle, ctypes.byref(desc), dptr(params), n, n, dptr(state), 4 * n, dptr(summ), n,
            status.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(st)))
        return EngineResult(evolution, n, state, summ, status, st.kernel_ms, st.h2d_ms, st.d2h_ms,
                            st.matvec_useful, st.matvec_exec, dim)

    def last_timeline(self) -> Dict[str, Any]:
        """ryd_last_timeline: host staging times and the per-slot HIP-event timeline of the
        last host-buffer call (ms; slot times relative to the first slot on its device)."""
        buf = np.zeros(N.TL_HEAD + N.TL_SLOT * len(self.devices))
        N.check(self.lib.ryd_last_timeline(self.handle, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                           buf.size))
        slots = []
        for k in range(int(buf[0])):
            t = buf[N.TL_HEAD + N.TL_SLOT * k: N.TL_HEAD + N.TL_SLOT * (k + 1)]
            slots.append(dict(device=int(t[0]), h2d_start=t[1], kernel_start=t[2], kernel_end=t[3],
                              d2h_end=t[4], points=int(t[5]), host_enqueued=t[6], host_wait=t[7]))
        return dict(pack_ms=buf[1], unpack_ms=buf[2], wall_ms=buf[3], slots=slots)

    def run_coherences(self, params: np.ndarray, protocol: str, n_steps: Optional[int] = None,
                       shape: str = "square") -> Tuple[np.ndarray, np.ndarray]:
        """The 6 upper off-diagonal qubit matrix units through the gate
        (ryd_run_coherences): returns (coh (NCOH, n) float64, status (n,) uint32)."""
        params = np.ascontiguousarray(params, dtype=np.float64)
        if params.shape[0] != N.NPARAM:
            raise ValueError(f"params must have shape ({N.NPARAM}, n)")
        n = params.shape[1]
        if n_steps is None:
            n_steps = default_n_steps(protocol, params)
        desc = make_desc(protocol, "lindblad", n_steps, shape, symmetric_atoms(params), "cheb_vector")
        coh = np.zeros((N.NCOH, n), dtype=np.float64)
        status = np.zeros(n, dtype=np.uint32)
        st = N.Stats()
        dptr = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        N.check(self.lib.ryd_run_coherences(
            self.handle, ctypes.byref(desc), dptr(params), n, n, dptr(coh), n,
            status.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(st)))
        return coh, status


    def derive(self, inp, diag: bool = False) -> Tuple[np.ndarray, np.ndarray, Optional[np.ndarray]]:
        """Hot-path row a1 on the GPU (ryd_derive): ``physics.derive_inputs(...)`` ->
        (params (NPARAM, n) as pack_params builds them, warning bits (n,) uint32, and with
        ``diag`` the (DV_NDIAG, n) derived columns named by _native.DV_DIAG)."""
        n = inp.n
        cols = np.ascontiguousarray(inp.cols, dtype=np.float64)
        params = np.empty((N.NPARAM, n), dtype=np.float64)
        warn = np.zeros(n, dtype=np.uint32)
        dg = np.empty((N.DV_NDIAG, n), dtype=np.float64) if diag else None
        dptr = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        N.check(self.lib.ryd_derive(self.handle, ctypes.byref(inp.desc), dptr(cols) if cols.shape[0] else None,
                                    cols.shape[0], n, n, dptr(params), n,
                                    warn.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                    dptr(dg) if diag else None, n))
        return params, warn, dg

    def evolve_generic(self, H: np.ndarray, dt: np.ndarray, state0: np.ndarray,
                       ops: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
        """The generic evolve_state seam (ryd_evolve_generic; RG/simulation.py:647-690) for
        a batch: H (n, n_seg, d, d) piecewise-constant Hamiltonians, dt (n, n_seg), state0
        (n, d) kets or (n, d, d) density matrices, ops (n, K, d, d) jump operators (kets
        only without them).  Returns (final states, status (n,) uint32)."""
        H = np.ascontiguousarray(H, dtype=np.complex128)
        if H.ndim != 4 or H.shape[2] != H.shape[3]:
            raise ValueError("H must have shape (n, n_seg, d, d)")
        n, n_seg, d = H.shape[0], H.shape[1], H.shape[2]
        dt = np.ascontiguousarray(np.broadcast_to(np.asarray(dt, dtype=np.float64), (n, n_seg)))
        state0 = np.ascontiguousarray(state0, dtype=np.complex128)
        ket = state0.shape == (n, d)
        if not ket and state0.shape != (n, d, d):
            raise ValueError("state0 must have shape (n, d) or (n, d, d)")
        K = 0
        if ops is not None:
            ops = np.ascontiguousarray(ops, dtype=np.complex128)
            if ops.ndim != 4 or ops.shape[0] != n or ops.shape[2:] != (d, d):
                raise ValueError("ops must have shape (n, K, d, d)")
            K = ops.shape[1]
        out = np.zeros_like(state0)
        status = np.zeros(n, dtype=np.uint32)
        dptr = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        N.check(self.lib.ryd_evolve_generic(
            self.handle, d, n_seg, K, n, 1 if ket else 0, dptr(H), dptr(dt),
            dptr(ops) if K > 0 else None, dptr(state0), dptr(out),
            status.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))
        return out, status


class DeviceBatch:
    """Inputs resident in HBM on one device slot, for timed re-runs (bench.py)."""

    def __init__(self, engine: Engine, params: np.ndarray, protocol: str, evolution: str,
                 n_steps: Optional[int] = None, shape: str = "square", slot: int = 0,
                 method: str = "chebyshev", dim: int = 3):
        self.eng, self.slot = engine, slot
        lib = engine.lib
        params = np.ascontiguousarray(params, dtype=np.float64)
        self.n = n = params.shape[1]
        if n_steps is None:
            n_steps = default_n_steps(protocol, params)
        self.desc = make_desc(protocol, evolution, n_steps, shape, symmetric_atoms(params), method, dim=dim)
        self.dim = dim
        self.width = N.STATE_WIDTH_DIM[dim][evolution]
        self.evolution = evolution
        self._bufs = []

        def alloc(nbytes):
            p = ctypes.c_void_p()
            N.check(lib.ryd_malloc(engine.handle, slot, nbytes, ctypes.byref(p)))
            self._bufs.append(p)
            return p
        self.d_params = alloc(params.nbytes)
        self.d_state = alloc(8 * self.width * 4 * n)
        self.d_summary = alloc(8 * N.NSUMMARY * n)
        self.d_status = alloc(4 * n)
        N.check(lib.ryd_memcpy_h2d(engine.handle, slot, self.d_params, params.ctypes.data, params.nbytes))

    def launch(self, timed: bool = False) -> float:
        """Enqueue one propagation of the whole batch; with ``timed`` wait and return
        the kernel's device time (HIP events on the launch stream)."""
        ms = ctypes.c_float(0.0)
        N.check(self.eng.lib.ryd_run_batch_device(
            self.eng.handle, self.slot, ctypes.byref(self.desc), self.d_params, self.n, self.n,
            self.d_state, 4 * self.n, self.d_summary, self.n, self.d_status, None,
            ctypes.byref(ms) if timed else None))
        return float(ms.value)

    def mark(self, which: int):
        """Record HIP event `which` (0 = region start, 1 = region end) on the launch stream."""
        N.check(self.eng.lib.ryd_mark(self.eng.handle, self.slot, which))

    def mark_elapsed(self) -> float:
        """Device ms between marks 0 and 1 (waits for mark 1)."""
        ms = ctypes.c_float(0.0)
        N.check(self.eng.lib.ryd_mark_elapsed(self.eng.handle, self.slot, ctypes.byref(ms)))
        return float(ms.value)

    def synchronize(self):
        N.check(self.eng.lib.ryd_synchronize(self.eng.handle))

    def fetch(self) -> EngineResult:
        lib, h, s = self.eng.lib, self.eng.handle, self.slot
        state = np.zeros((self.width, 4 * self.n))
        summ = np.zeros((N.NSUMMARY, self.n))
        status = np.zeros(self.n, dtype=np.uint32)
        N.check(lib.ryd_memcpy_d2h(h, s, state.ctypes.data, self.d_state, state.nbytes))
        N.check(lib.ryd_memcpy_d2h(h, s, summ.ctypes.data, self.d_summary, summ.nbytes))
        N.check(lib.ryd_memcpy_d2h(h, s, status.ctypes.data, self.d_status, status.nbytes))
        return EngineResult(self.evolution, self.n, state, summ, status, 0.0, 0.0, 0.0,
                            summ[N.S["NMV_USEFUL"]].sum(), summ[N.S["NMV_EXEC"]].sum(), self.dim)

    def free(self):
        for p in self._bufs:
            self.eng.lib.ryd_free(self.eng.handle, self.slot, p)
        self._bufs = []


class DeviceSweep:
    """A sweep whose parameters never exist on the host: its varying input fields are
    resident on one device slot (``upload``), ``ryd_derive_device`` writes the parameter
    block in HBM and the propagation kernel reads it there (C4: 1M species x T x
    P_tweezer points -> derive + engine on the device).  ``launch`` enqueues derive then
    engine on the slot's stream."""

    def __init__(self, engine: Engine, inp, evolution: str = "lindblad", slot: int = 0,
                 n_steps: Optional[int] = None, method: str = "chebyshev"):
        self.eng, self.slot, self.inp = engine, slot, inp
        lib = engine.lib
        self.n = n = inp.n
        self.dim = inp.dim
        self.width = N.STATE_WIDTH_DIM[inp.dim][evolution]
        self.evolution = evolution
        if n_steps is None:
            n_steps = {"smooth_jp": 300, "lp_shaped": 500}.get(inp.protocol, 0)
            if inp.protocol == "bangbang":
                n_steps = int(inp.desc.bb_nseg)
        # every shared rate is equal on both atoms (the derivation writes atom B = atom A)
        self.desc = make_desc(inp.protocol, evolution, n_steps, inp.shape, True, method, dim=inp.dim)
        self._bufs = []

        def alloc(nbytes):
            p = ctypes.c_void_p()
            N.check(lib.ryd_malloc(engine.handle, slot, max(nbytes, 16), ctypes.byref(p)))
            self._bufs.append(p)
            return p
        self.k = inp.cols.shape[0]
        self.d_in = alloc(8 * self.k * n)
        self.d_params = alloc(8 * N.NPARAM * n)
        self.d_warn = alloc(4 * n)
        self.d_state = alloc(8 * self.width * 4 * n)
        self.d_summary = alloc(8 * N.NSUMMARY * n)
        self.d_status = alloc(4 * n)
        self.upload()

    def upload(self):
        """H2D of the varying input fields (the only per-point host data)."""
        cols = np.ascontiguousarray(self.inp.cols, dtype=np.float64)
        if self.k:
            N.check(self.eng.lib.ryd_memcpy_h2d(self.eng.handle, self.slot, self.d_in, cols.ctypes.data, cols.nbytes))

    def derive(self, timed: bool = False) -> float:
        ms = ctypes.c_float(0.0)
        N.check(self.eng.lib.ryd_derive_device(
            self.eng.handle, self.slot, ctypes.byref(self.inp.desc), self.d_in if self.k else None, self.n,
            self.n, self.d_params, self.n, self.d_warn, None, self.n, None, ctypes.byref(ms) if timed else None))
        return float(ms.value)

    def propagate(self, timed: bool = False) -> float:
        ms = ctypes.c_float(0.0)
        N.check(self.eng.lib.ryd_run_batch_device(
            self.eng.handle, self.slot, ctypes.byref(self.desc), self.d_params, self.n, self.n,
            self.d_state, 4 * self.n, self.d_summary, self.n, self.d_status, None,
            ctypes.byref(ms) if timed else None))
        return float(ms.value)

    def launch(self):
        self.derive()
        self.propagate()

    def mark(self, which: int):
        N.check(self.eng.lib.ryd_mark(self.eng.handle, self.slot, which))

    def mark_elapsed(self) -> float:
        ms = ctypes.c_float(0.0)
        N.check(self.eng.lib.ryd_mark_elapsed(self.eng.handle, self.slot, ctypes.byref(ms)))
        return float(ms.value)

    def synchronize(self):
        N.check(self.eng.lib.ryd_synchronize(self.eng.handle))

    def fetch_params(self) -> Tuple[np.ndarray, np.ndarray]:
        lib, h, s = self.eng.lib, self.eng.handle, self.slot
        p = np.zeros((N.NPARAM, self.n))
        w = np.zeros(self.n, dtype=np.uint32)
        N.check(lib.ryd_memcpy_d2h(h, s, p.ctypes.data, self.d_params, p.nbytes))
        N.check(lib.ryd_memcpy_d2h(h, s, w.ctypes.data, self.d_warn, w.nbytes))
        return p, w

    def fetch(self) -> EngineResult:
        lib, h, s = self.eng.lib, self.eng.handle, self.slot
        state = np.zeros((self.width, 4 * self.n))
        summ = np.zeros((N.NSUMMARY, self.n))
        status = np.zeros(self.n, dtype=np.uint32)
        N.check(lib.ryd_memcpy_d2h(h, s, state.ctypes.data, self.d_state, state.nbytes))
        N.check(lib.ryd_memcpy_d2h(h, s, summ.ctypes.data, self.d_summary, summ.nbytes))
        N.check(lib.ryd_memcpy_d2h(h, s, status.ctypes.data, self.d_status, status.nbytes))
        _, warn = self.fetch_params()
        return EngineResult(self.evolution, self.n, state, summ, status | warn, 0.0, 0.0, 0.0,
                            summ[N.S["NMV_USEFUL"]].sum(), summ[N.S["NMV_EXEC"]].sum(), self.dim)

    def free(self):
        for p in self._bufs:
            self.eng.lib.ryd_free(self.eng.handle, self.slot, p)
        self._bufs = []


class CoherenceDeviceBatch:
    """Process-map coherence sectors (ryd_run_coherences_device: the four
    coherence_cheb_kernel launches) with inputs resident in HBM, for timed re-runs."""

    def __init__(self, engine: Engine, params: np.ndarray, protocol: str, n_steps: Optional[int] = None,
                 shape: str = "square", slot: int = 0):
        self.eng, self.slot = engine, slot
        lib = engine.lib
        params = np.ascontiguousarray(params, dtype=np.float64)
        self.n = n = params.shape[1]
        if n_steps is None:
            n_steps = default_n_steps(protocol, params)
        self.desc = make_desc(protocol, "lindblad", n_steps, shape, symmetric_atoms(params), "cheb_vector")
        self._bufs = []

        def alloc(nbytes):
            p = ctypes.c_void_p()
            N.check(lib.ryd_malloc(engine.handle, slot, nbytes, ctypes.byref(p)))
            self._bufs.append(p)
            return p
        self.d_params = alloc(params.nbytes)
        self.d_coh = alloc(8 * N.NCOH * n)
        self.d_status = alloc(4 * n)
        N.check(lib.ryd_memcpy_h2d(engine.handle, slot, self.d_params, params.ctypes.data, params.nbytes))

    def launch(self, timed: bool = False) -> float:
        ms = ctypes.c_float(0.0)
        N.check(self.eng.lib.ryd_run_coherences_device(
            self.eng.handle, self.slot, ctypes.byref(self.desc), self.d_params, self.n, self.n,
            self.d_coh, self.n, self.d_status, None, ctypes.byref(ms) if timed else None))
        return float(ms.value)

    def mark(self, which: int):
        N.check(self.eng.lib.ryd_mark(self.eng.handle, self.slot, which))

    def mark_elapsed(self) -> float:
        ms = ctypes.c_float(0.0)
        N.check(self.eng.lib.ryd_mark_elapsed(self.eng.handle, self.slot, ctypes.byref(ms)))
        return float(ms.value)

    def synchronize(self):
        N.check(self.eng.lib.ryd_synchronize(self.eng.handle))

    def fetch(self) -> Tuple[np.ndarray, np.ndarray]:
        lib, h, s = self.eng.lib, self.eng.handle, self.slot
        coh = np.zeros((N.NCOH, self.n))
        status = np.zeros(self.n, dtype=np.uint32)
        N.check(lib.ryd_memcpy_d2h(h, s, coh.ctypes.data, self.d_coh, coh.nbytes))
        N.check(lib.ryd_memcpy_d2h(h, s, status.ctypes.data, self.d_status, status.nbytes))
        return coh, status

    def free(self):
        for p in self._bufs:
            self.eng.lib.ryd_free(self.eng.handle, self.slot, p)
        self._bufs = []
