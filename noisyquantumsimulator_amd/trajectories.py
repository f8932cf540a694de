"""Three-atom Rydberg blockade with quantum-jump trajectories on the GPU
(BASELINE configs[4]).

The reference has no three-atom model (RG/hamiltonians.py:381-1274 builds two
atoms), so this module defines it as the natural extension of the two-atom
path and runs it through ``ryd_run_trajectories`` (include/ryd_engine.h):

* three identical atoms on an equilateral triangle: V P_r (x) P_r on each pair,
  the single-atom Hamiltonian of RG/hamiltonians.py:584-1274,
* the same 4 collapse channels per atom as the two-atom engine (the default
  c_ops of RG/noise_models.py:1449-1620 collapsed: |1><r|, |0><r|, P_r, P_1),
* the same protocol schedules (``pack_params`` columns of a two-atom batch),
* waiting-time Monte-Carlo wave functions, Philox4x32-10 streams keyed by
  (seed, global point index, trajectory), the mean rho (27x27) and the standard
  error of every element reduced on the GPU.

Kets use the basis index 9 a0 + 3 a1 + a2 with a in {0, 1, 2 = r}.  The product
path has no CPU fallback: ``Engine()`` raises without the HIP library or a GPU.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _native as N
from .engine import Engine, default_n_steps

DIM = 27
LABELS3 = tuple(f"{a}{b}{c}" for a in "01" for b in "01" for c in "01")
QUBIT_INDEX3 = tuple(9 * a + 3 * b + c for a in (0, 1) for b in (0, 1) for c in (0, 1))
CHANNELS = ("|1><r|", "|0><r|", "P_r", "P_1")       # channel code = 4 * atom + c
# Jump times.  ladder_levels = N.T["EXACT"] (0): the root of ||psi(t)||^2 = r, by Newton on
# the eigen-decomposed H_eff (traj3e_kernel) -- the oracle's own definition, and the
# fastest C5 kernel; it needs |Omega| and Delta constant over a point's
# segments.  ladder_levels = L >= 1: the binary ladder walk (traj3s_kernel), jump times
# resolved to segment / 2^L; at L = 16 the delay shifts the conditional state by
# ~Omega tau / 2^(L+1) = 3e-5 per jump on the C5 points, against a standard error of
# ~1e-2 at 256 trajectories.  DEFAULT_LADDER (None) picks exact times wherever they
# apply and the L = 16 ladder for a shaped LP envelope.  In exact mode the library itself
# sends a point whose |Omega| or Delta changes between segments (an LP square with
# |xi| != 1), or whose H_eff eigenbasis is unconverged or ill-conditioned (near an
# exceptional point), through the L = 16 ladder and marks it N.STATUS_EXACT_FALLBACK
# (round 4: such points used to come back BAD_INPUT).
DEFAULT_LADDER = None
LADDER_WALK = 16


def resolve_ladder(ladder_levels: Optional[int], protocol: str, shape: str = "square") -> int:
    """The ladder_levels a descriptor gets: ``None`` -> exact jump times, or the L = 16
    ladder where exact mode cannot apply to any point (a shaped LP envelope)."""
    if ladder_levels is not None:
        return int(ladder_levels)
    return LADDER_WALK if (protocol == "lp_shaped" and shape != "square") else N.T["EXACT"]


def basis_index(a0: int, a1: int, a2: int) -> int:
    return 9 * a0 + 3 * a1 + a2


def product_ket(*single) -> np.ndarray:
    """Tensor product of three single-atom kets (length-3 vectors over |0>, |1>, |r>)."""
    if len(single) != 3:
        raise ValueError("three single-atom kets are needed")
    v = np.ones(1, dtype=complex)
    for s in single:
        v = np.kron(v, np.asarray(s, dtype=complex))
    return v / np.linalg.norm(v)


def plus_state() -> np.ndarray:
    """|+>^3 on the qubit levels: every computational input of the gate at once."""
    s = np.array([1.0, 1.0, 0.0]) / np.sqrt(2.0)
    return product_ket(s, s, s)


def _psi_array(psi0: np.ndarray) -> np.ndarray:
    psi0 = np.asarray(psi0, dtype=complex).ravel()
    if psi0.shape != (DIM,):
        raise ValueError("psi0 must have 27 amplitudes")
    nrm = np.linalg.norm(psi0)
    if not np.isfinite(nrm) or nrm == 0:
        raise ValueError("psi0 must be a finite, nonzero ket")
    psi0 = psi0 / nrm
    out = np.empty(2 * DIM)
    out[0::2], out[1::2] = psi0.real, psi0.imag
    return out


def make_traj_desc(protocol: str, psi0: np.ndarray, n_traj: int = 256, seed: int = 0,
                   ladder_levels: Optional[int] = DEFAULT_LADDER, n_steps: int = 0,
                   shape: str = "square", kernel: str = "auto") -> N.TrajDesc:
    """``kernel`` picks the exact-mode kernel (include/ryd_engine.h RYD_T_FLAG_*): "rows"
    (one trajectory per 16-lane DPP row, pass 1 once per point), "lanes" (one trajectory per
    lane, traj3e), or "auto" (the library's default, lanes; env RYD_T_ROWS=1 -> rows)."""
    if kernel not in N.T_FLAG:
        raise ValueError(f"kernel must be one of {sorted(N.T_FLAG)}")
    d = N.TrajDesc()
    d.flags = N.T_FLAG[kernel]
    d.abi_version = N.RYD_ABI_VERSION
    d.protocol = N.PROTO[protocol]
    d.shape = N.SHAPE[shape]
    d.n_steps = n_steps
    d.n_traj = n_traj
    d.ladder_levels = resolve_ladder(ladder_levels, protocol, shape)
    d.seed = seed & 0xFFFFFFFFFFFFFFFF
    d.psi0[:] = list(_psi_array(psi0))
    return d


def unpack_rho(flat: np.ndarray) -> np.ndarray:
    """(n, 1458) column-stacked (re, im) rows -> rho[n, 27, 27]."""
    v = flat[:, 0::2] + 1j * flat[:, 1::2]
    return v.reshape(-1, DIM, DIM).transpose(0, 2, 1)


def unpack_se(flat: np.ndarray) -> np.ndarray:
    return flat.reshape(-1, DIM, DIM).transpose(0, 2, 1)


@dataclass
class TrajectoryResult:
    n: int
    n_traj: int
    rho: np.ndarray             # (n, 27, 27) complex: mean over trajectories
    se: np.ndarray              # (n, 27, 27): standard error of each element
    summary: np.ndarray         # (T_NSUMMARY, n)
    status: np.ndarray          # (n,) uint32
    records: Optional[np.ndarray]   # (n, n_traj, 64) or None
    kernel_ms: float = 0.0
    h2d_ms: float = 0.0
    d2h_ms: float = 0.0

    def col(self, name: str) -> np.ndarray:
        return self.summary[N.TS[name]]

    def kets(self) -> np.ndarray:
        """Final normalised ket of every trajectory (records mode)."""
        r = self._rec()
        return r[..., 0:54:2] + 1j * r[..., 1:54:2]

    def n_jumps(self) -> np.ndarray:
        return self._rec()[..., N.T["REC_NJUMPS"]].astype(int)

    def jump_times(self) -> np.ndarray:
        j0 = N.T["REC_JUMP0"]
        return self._rec()[..., j0:j0 + 2 * N.T["REC_JUMPS"]:2]

    def jump_channels(self) -> np.ndarray:
        j0 = N.T["REC_JUMP0"]
        return self._rec()[..., j0 + 1:j0 + 2 * N.T["REC_JUMPS"]:2].astype(int)

    def _rec(self) -> np.ndarray:
        if self.records is None:
            raise ValueError("run with records=True to keep per-trajectory records")
        return self.records


def run_trajectories(engine: Engine, params: np.ndarray, protocol: str, psi0: Optional[np.ndarray] = None,
                     n_traj: int = 256, seed: int = 0, ladder_levels: Optional[int] = DEFAULT_LADDER,
                     n_steps: Optional[int] = None, shape: str = "square",
                     records: bool = False, kernel: str = "auto") -> TrajectoryResult:
    """Host-buffer form: every point of ``params`` (``pack_params`` columns; atom-A
    rates are used for all three atoms) through ``n_traj`` trajectories."""
    params = np.ascontiguousarray(params, dtype=np.float64)
    if params.shape[0] != N.NPARAM:
        raise ValueError(f"params must have shape ({N.NPARAM}, n)")
    n = params.shape[1]
    if n_steps is None:
        n_steps = default_n_steps(protocol, params)
    desc = make_traj_desc(protocol, plus_state() if psi0 is None else psi0, n_traj, seed, ladder_levels,
                          n_steps, shape, kernel)
    rho = np.zeros((n, N.T["RHO_WIDTH"]))
    se = np.zeros((n, N.T["SE_WIDTH"]))
    summ = np.zeros((N.T_NSUMMARY, n))
    status = np.zeros(n, dtype=np.uint32)
    rec = np.zeros((n, n_traj, N.T["REC_WIDTH"])) if records else None
    st = N.Stats()
    dptr = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    N.check(engine.lib.ryd_run_trajectories(
        engine.handle, ctypes.byref(desc), dptr(params), n, n, dptr(rho), dptr(se), dptr(summ), n,
        dptr(rec) if records else None, status.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
        ctypes.byref(st)))
    return TrajectoryResult(n, n_traj, unpack_rho(rho), unpack_se(se), summ, status, rec,
                            st.kernel_ms, st.h2d_ms, st.d2h_ms)


class TrajectoryDeviceBatch:
    """Inputs resident in HBM on one device slot, for timed re-runs (bench.py) and
    shards launched with their global point indices: point i of the batch is global point
    ``point_offset + point_stride * i`` (a range shard: stride 1; rank r of a strided split
    over N ranks: offset r, stride N), which keys its trajectories' random streams."""

    def __init__(self, engine: Engine, params: np.ndarray, protocol: str, psi0: Optional[np.ndarray] = None,
                 n_traj: int = 256, seed: int = 0, ladder_levels: Optional[int] = DEFAULT_LADDER,
                 n_steps: Optional[int] = None, shape: str = "square", slot: int = 0,
                 point_offset: int = 0, records: bool = False, kernel: str = "auto", point_stride: int = 1):
        if point_stride < 1 or point_offset < 0:
            raise ValueError("point_stride must be >= 1 and point_offset >= 0")
        self.eng, self.slot, self.point_offset = engine, slot, point_offset
        lib = engine.lib
        params = np.ascontiguousarray(params, dtype=np.float64)
        self.n = n = params.shape[1]
        if n_steps is None:
            n_steps = default_n_steps(protocol, params)
        self.n_traj = n_traj
        self.desc = make_traj_desc(protocol, plus_state() if psi0 is None else psi0, n_traj, seed,
                                   ladder_levels, n_steps, shape, kernel)
        self.desc.point_stride = point_stride
        self._bufs = []

        def alloc(nbytes):
            p = ctypes.c_void_p()
            N.check(lib.ryd_malloc(engine.handle, slot, nbytes, ctypes.byref(p)))
            self._bufs.append(p)
            return p
        self.d_params = alloc(params.nbytes)
        self.d_rho = alloc(8 * N.T["RHO_WIDTH"] * n)
        self.d_se = alloc(8 * N.T["SE_WIDTH"] * n)
        self.d_summary = alloc(8 * N.T_NSUMMARY * n)
        self.d_status = alloc(4 * n)
        self.d_rec = alloc(8 * N.T["REC_WIDTH"] * n_traj * n) if records else None
        N.check(lib.ryd_memcpy_h2d(engine.handle, slot, self.d_params, params.ctypes.data, params.nbytes))

    def launch(self, timed: bool = False) -> float:
        ms = ctypes.c_float(0.0)
        N.check(self.eng.lib.ryd_run_trajectories_device(
            self.eng.handle, self.slot, ctypes.byref(self.desc), self.d_params, self.n, self.n,
            self.point_offset, self.d_rho, N.T["RHO_WIDTH"], self.d_se, N.T["SE_WIDTH"], self.d_summary,
            self.n, self.d_rec, self.d_status, None, ctypes.byref(ms) if timed else None))
        return float(ms.value)

    def mark(self, which: int):
        """Record HIP event `which` (0 = region start, 1 = region end) on the launch stream."""
        N.check(self.eng.lib.ryd_mark(self.eng.handle, self.slot, which))

    def mark_elapsed(self) -> float:
        ms = ctypes.c_float(0.0)
        N.check(self.eng.lib.ryd_mark_elapsed(self.eng.handle, self.slot, ctypes.byref(ms)))
        return float(ms.value)

    def synchronize(self):
        N.check(self.eng.lib.ryd_synchronize(self.eng.handle))

    def fetch(self) -> TrajectoryResult:
        lib, h, s = self.eng.lib, self.eng.handle, self.slot
        rho = np.zeros((self.n, N.T["RHO_WIDTH"]))
        se = np.zeros((self.n, N.T["SE_WIDTH"]))
        summ = np.zeros((N.T_NSUMMARY, self.n))
        status = np.zeros(self.n, dtype=np.uint32)
        for arr, d in ((rho, self.d_rho), (se, self.d_se), (summ, self.d_summary), (status, self.d_status)):
            N.check(lib.ryd_memcpy_d2h(h, s, arr.ctypes.data, d, arr.nbytes))
        rec = None
        if self.d_rec is not None:
            rec = np.zeros((self.n, self.n_traj, N.T["REC_WIDTH"]))
            N.check(lib.ryd_memcpy_d2h(h, s, rec.ctypes.data, self.d_rec, rec.nbytes))
        return TrajectoryResult(self.n, self.n_traj, unpack_rho(rho), unpack_se(se), summ, status, rec)

    def free(self):
        for p in self._bufs:
            self.eng.lib.ryd_free(self.eng.handle, self.slot, p)
        self._bufs = []
