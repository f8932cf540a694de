"""ctypes binding of libryd_engine.so (include/ryd_engine.h).

The product path has no CPU fallback: if the in-tree HIP library is missing,
or no GPU is visible when a batch is run, these functions raise.
"""
from __future__ import annotations

import ctypes
import os
import threading
import warnings
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
# RYD_ENGINE_LIB selects an alternative build of the same library (tuning variants)
LIB_PATH = os.environ.get("RYD_ENGINE_LIB") or os.path.join(_HERE, "libryd_engine.so")

# keep in sync with include/ryd_engine.h
RYD_ABI_VERSION = 5
RYD_OK = 0
PROTO = {"lp_square": 0, "lp_shaped": 1, "bangbang": 2, "smooth_jp": 3}
EVOL = {"lindblad": 0, "ket": 1}
METHOD = {"chebyshev": 0, "dopri5": 1, "cheb_vector": 2, "cheb_squaring": 3}
SHAPE = {"square": 0, "gaussian": 1, "cosine": 2, "blackman": 3}
FLAG_SYMMETRIC_ATOMS = 1

P = dict(OMEGA=0, DELTA=1, V=2, DELTA1=3, G1_A=4, G0_A=5, GPHI_A=6, GSC_A=7, G1_B=8, G0_B=9,
         GPHI_B=10, GSC_B=11, TAU=12, XI_RE=13, XI_IM=14, AREA_CORR=15, A=16, OMEGA_MOD=17,
         PHI_OFF=18, OMEGA_TAU=19, NSEG=20, SWT0=21, PHI0=28, GMJ_A=36, GMJ_B=37)
NPARAM = 38
S = dict(POP0=0, OV_RE0=4, OV_IM0=8, AVG_POP=12, CTRL_PHASE=13, PENALTY=14, AVG_F=15,
         NMV_USEFUL=16, NMV_EXEC=17, TRACE11=18, NSQUARE=19)
NSUMMARY = 20
STATUS_NONFINITE, STATUS_STEP_CAP, STATUS_BAD_INPUT = 1, 2, 4
STATUS_FAIL_MASK = 7                      # kernel failures; the bits below are warnings
STATUS_WEAK_BLOCKADE, STATUS_DARK_STATE_SIGN, STATUS_OMEGA_RANGE = 8, 16, 32
STATUS_GAUGE_UNSTABLE = 64
STATUS_EXACT_FALLBACK = 128               # C5 exact mode: this point ran on the L = 16 ladder
# ryd_mixed_phase output rows
MP = dict(V0=0, CTRL=8, PENALTY=9, SPREAD=10)
MP_WIDTH = 11
STATE_WIDTH = {"lindblad": 25, "ket": 18}                 # dim 3
STATE_WIDTH_DIM = {3: STATE_WIDTH, 4: {"lindblad": 36, "ket": 32}}
# process-map coherence rows (ryd_run_coherences)
C = dict(K0=0, K1=8, K2=16, K3=18)
NCOH = 20

# three-atom quantum-jump trajectories (ryd_run_trajectories)
T = dict(DIM=27, RHO_WIDTH=1458, SE_WIDTH=729, EXACT=0, LADDER_MAX=40, REC_WIDTH=64, REC_NJUMPS=54,
         REC_JUMP0=55, REC_JUMPS=4, REC_ITERS=63)
TS = dict(MEAN_JUMPS=0, FRAC_JUMPED=1, MAX_JUMPS=2, TRACE=3, QUBIT_POP=4, ITER_USEFUL=5,
          ITER_EXEC=6, NLADDER=7, NSQUARE=8, RESERVED=9)
T_NSUMMARY = 10
# exact-mode kernel selection (ryd_traj_desc.flags)
T_FLAG = {"auto": 0, "rows": 1, "lanes": 2}

# ryd_last_timeline layout
TL_HEAD, TL_SLOT = 4, 8

EXPORTED = ("ryd_abi_version", "ryd_last_error", "ryd_param_count", "ryd_summary_width", "ryd_lp_unsquared",
            "ryd_state_width", "ryd_device_count", "ryd_create", "ryd_destroy", "ryd_run_batch",
            "ryd_run_batch_device", "ryd_run_coherences", "ryd_run_coherences_device",
            "ryd_run_trajectories", "ryd_run_trajectories_device",
            "ryd_mixed_phase", "ryd_lapack_pool", "ryd_last_timeline", "ryd_mark", "ryd_mark_elapsed",
            "ryd_malloc", "ryd_free", "ryd_memcpy_h2d", "ryd_memcpy_d2h", "ryd_synchronize", "ryd_evolve_generic",
            "ryd_derive", "ryd_derive_device")

# device derivation (ryd_derive): input fields, species-table columns, flags, diagnostic columns
DV = dict(SPECIES=0, N_RYD=1, P1=2, P2=3, W1=4, W2=5, DELTA_E=6, LW1=7, LW2=8, TW_POWER=9, TW_WAIST=10,
          TW_WL_NM=11, TEMPERATURE=12, B_FIELD=13, NA=14, SPACING=15, BG_LOSS=16, DOM=17, OMEGA_TAU=18,
          SJP_A=19, SJP_OMR=20, SJP_PHI_OFF=21, SJP_SDOM=22, BB_SWT0=23, BB_PHI0=30)
DV_NFIELD = 38
DV_NSPC = 24
DV_MAX_SPECIES = 4
DV_SPC = ("mass", "alpha_ground", "trap_wavelength", "n_ref", "C6_ref", "tau_0K_ref", "tau_ref",
          "alpha_rydberg_ref", "dipole_er_ref", "qd_S", "dipole_1e", "gamma_e", "f_ground_to_e", "E_ionization",
          "omega_D1", "K_quad_zeeman", "K_quad_noise", "stark_hz_per_mK", "g_F_lower", "F_lower", "exp_C6",
          "exp_tau0", "exp_tau_bbr", "exp_alpha")
DV_FLAG = dict(NOISE=1, TRAP_ON=2, DOPPLER=4, INTENSITY=8, COUNTERPROP=16, MOTIONAL=32)
DV_LEAK = dict(square=0, gaussian=1, cosine=2, blackman=3)          # anything else: 4 (sinc^2 + 1e-10)
DV_LEAK_OTHER = 4
# diagnostic columns -> the DerivedBatch column of the same quantity
DV_DIAG = ("Omega1", "Omega", "V", "R", "U0", "omega_r", "sigma_r", "dVV", "g_thermal", "g_scatter", "alpha_g",
           "alpha_r", "alpha_ratio", "g_antitrap_raw", "diff_shift", "enhancement", "k_eff", "v_thermal",
           "g_doppler", "g_intensity", "gamma_r_trap", "wavelength_nm", "tau_single", "tau_total", "Delta_gate",
           "delta_over_omega", "omega_tau", "delta_zeeman", "delta_stark", "V_over_Omega", "xi_re", "xi_im",
           "Delta_seg", "gamma_r", "gamma_phi_laser", "gamma_phi_thermal", "gamma_phi_zeeman",
           "gamma_loss_antitrap", "gamma_loss_background", "gamma_leakage", "gamma_scatter_intermediate",
           "mJ_leakage_rate", "area_correction")
DV_NDIAG = len(DV_DIAG)


class BatchDesc(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("dim", ctypes.c_int32),
                ("protocol", ctypes.c_int32), ("evolution", ctypes.c_int32),
                ("method", ctypes.c_int32), ("shape", ctypes.c_int32),
                ("n_steps", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("rtol", ctypes.c_double), ("atol", ctypes.c_double),
                ("max_steps", ctypes.c_int64)]


class TrajDesc(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("protocol", ctypes.c_int32),
                ("shape", ctypes.c_int32), ("n_steps", ctypes.c_int32),
                ("n_traj", ctypes.c_int32), ("ladder_levels", ctypes.c_int32),
                ("flags", ctypes.c_uint32), ("point_stride", ctypes.c_uint32),
                ("seed", ctypes.c_uint64), ("psi0", ctypes.c_double * 54)]


class DeriveDesc(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("protocol", ctypes.c_int32), ("shape", ctypes.c_int32),
                ("leak_shape", ctypes.c_int32), ("dim", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("n_species", ctypes.c_int32), ("bb_nseg", ctypes.c_int32), ("qubit", ctypes.c_double * 4),
                ("intensity_noise_frac", ctypes.c_double), ("polarization_purity", ctypes.c_double),
                ("species", (ctypes.c_double * DV_NSPC) * DV_MAX_SPECIES),
                ("value", ctypes.c_double * DV_NFIELD), ("col", ctypes.c_int32 * DV_NFIELD)]


class Stats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double),
                ("d2h_ms", ctypes.c_double), ("matvec_useful", ctypes.c_double),
                ("matvec_exec", ctypes.c_double), ("n_devices", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


_lock = threading.Lock()
_lib = None


class EngineError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load the in-tree HIP library (fails loudly if it was not built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise EngineError(f"{LIB_PATH} is missing: build it with `make` or "
                              "`python -c 'import __graft_entry__ as g; g.build()'`")
        lib = ctypes.CDLL(LIB_PATH)
        vp, i64, dp = ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_double)
        lib.ryd_abi_version.restype = ctypes.c_int
        lib.ryd_last_error.restype = ctypes.c_char_p
        lib.ryd_param_count.restype = ctypes.c_int
        lib.ryd_summary_width.restype = ctypes.c_int
        lib.ryd_lp_unsquared.restype = ctypes.c_int
        lib.ryd_state_width.argtypes = [ctypes.c_int, ctypes.c_int]
        lib.ryd_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        lib.ryd_create.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(vp)]
        lib.ryd_destroy.argtypes = [vp]
        lib.ryd_run_batch.argtypes = [vp, ctypes.POINTER(BatchDesc), dp, i64, i64, dp, i64, dp, i64,
                                      ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(Stats)]
        lib.ryd_run_batch_device.argtypes = [vp, ctypes.c_int, ctypes.POINTER(BatchDesc), vp, i64, i64,
                                             vp, i64, vp, i64, vp, vp, ctypes.POINTER(ctypes.c_float)]
        lib.ryd_run_coherences.argtypes = [vp, ctypes.POINTER(BatchDesc), dp, i64, i64, dp, i64,
                                           ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(Stats)]
        lib.ryd_run_coherences_device.argtypes = [vp, ctypes.c_int, ctypes.POINTER(BatchDesc), vp, i64,
                                                  i64, vp, i64, vp, vp, ctypes.POINTER(ctypes.c_float)]
        lib.ryd_run_trajectories.argtypes = [vp, ctypes.POINTER(TrajDesc), dp, i64, i64, dp, dp, dp, i64,
                                             dp, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(Stats)]
        lib.ryd_run_trajectories_device.argtypes = [vp, ctypes.c_int, ctypes.POINTER(TrajDesc), vp, i64, i64,
                                                    i64, vp, i64, vp, i64, vp, i64, vp, vp, vp,
                                                    ctypes.POINTER(ctypes.c_float)]
        lib.ryd_mixed_phase.argtypes = [vp, ctypes.c_int, dp, i64, i64, ctypes.c_int, ctypes.c_double,
                                        ctypes.c_double, ctypes.c_int, dp, i64, ctypes.POINTER(ctypes.c_uint32)]
        lib.ryd_last_timeline.argtypes = [vp, dp, i64]
        lib.ryd_mark.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        lib.ryd_mark_elapsed.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
        lib.ryd_lapack_pool.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_int)]
        lib.ryd_malloc.argtypes = [vp, ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(vp)]
        lib.ryd_free.argtypes = [vp, ctypes.c_int, vp]
        lib.ryd_memcpy_h2d.argtypes = [vp, ctypes.c_int, vp, vp, ctypes.c_size_t]
        lib.ryd_memcpy_d2h.argtypes = [vp, ctypes.c_int, vp, vp, ctypes.c_size_t]
        lib.ryd_synchronize.argtypes = [vp]
        lib.ryd_evolve_generic.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, i64, ctypes.c_int, dp, dp,
                                           dp, dp, dp, ctypes.POINTER(ctypes.c_uint32)]
        lib.ryd_derive.argtypes = [vp, ctypes.POINTER(DeriveDesc), dp, i64, i64, i64, dp, i64,
                                   ctypes.POINTER(ctypes.c_uint32), dp, i64]
        lib.ryd_derive_device.argtypes = [vp, ctypes.c_int, ctypes.POINTER(DeriveDesc), vp, i64, i64, vp, i64, vp,
                                          vp, i64, vp, ctypes.POINTER(ctypes.c_float)]
        if lib.ryd_abi_version() != RYD_ABI_VERSION:
            raise EngineError("libryd_engine.so ABI version mismatch; rebuild it")
        if lib.ryd_param_count() != NPARAM or lib.ryd_summary_width() != NSUMMARY:
            raise EngineError("libryd_engine.so layout mismatch; rebuild it")
        _lib = lib
        return lib


def check(rc: int) -> None:
    if rc != RYD_OK:
        msg = load().ryd_last_error().decode(errors="replace")
        raise EngineError(f"ryd_engine error {rc}: {msg}")


_zheevr = None


def scipy_zheevr() -> int:
    """Address of scipy's own LAPACK zheevr (scipy.linalg.cython_lapack), the routine
    scipy.linalg.eigh -- and through it QuTiP 5's Qobj.eigenstates -- calls."""
    global _zheevr
    if _zheevr is None:
        from scipy.linalg import cython_lapack
        cap = cython_lapack.__pyx_capi__["zheevr"]
        api = ctypes.pythonapi
        api.PyCapsule_GetName.restype = ctypes.c_char_p
        api.PyCapsule_GetName.argtypes = [ctypes.py_object]
        api.PyCapsule_GetPointer.restype = ctypes.c_void_p
        api.PyCapsule_GetPointer.argtypes = [ctypes.py_object, ctypes.c_char_p]
        _zheevr = api.PyCapsule_GetPointer(cap, api.PyCapsule_GetName(cap))
    return _zheevr


_pool_size: Optional[int] = None
# copies (each holds a glibc link namespace; RYD_LAPACK_POOL sets it, C cap 15).  Round 5: 11,
# what loads on the GPU box beside torch before glibc refuses another namespace; a request
# above what loads keeps the copies that did load (tests/test_mixed_phase_host.py checks
# that such a partial pool stays bit-identical)
LAPACK_POOL_DEFAULT = 11


def lapack_pool_copies(n_threads: int) -> int:
    """Copies the epilogue asks for: RYD_LAPACK_POOL (0 = off, N = at most N copies),
    default min(n_threads, LAPACK_POOL_DEFAULT)."""
    env = os.environ.get("RYD_LAPACK_POOL")
    cap = LAPACK_POOL_DEFAULT
    if env is not None and env.strip() != "":
        try:
            cap = int(env)
        except ValueError:
            warnings.warn(f"RYD_LAPACK_POOL={env!r} is not an integer copy cap (0 = off, N = at most N "
                          f"copies): using the default {LAPACK_POOL_DEFAULT}")
            cap = LAPACK_POOL_DEFAULT
        if cap == 1:
            # before round 3 the variable was an on/off switch and '1' meant 'on'; one copy
            # would serialise the epilogue like no pool at all, so '1' keeps the default on
            warnings.warn("RYD_LAPACK_POOL=1 is read as 'on' (the default cap); use 0 to turn the pool off")
            cap = LAPACK_POOL_DEFAULT
    return max(0, min(n_threads, cap))


def scipy_lapack_pool(copies: int) -> int:
    """Private copies of scipy's OpenBLAS for the threaded epilogue (ryd_lapack_pool):
    OpenBLAS serialises concurrent zheevr callers on a process-wide lock, each copy in
    its own link namespace has its own.  Copies are admitted only if bit-identical to
    scipy_zheevr() on test matrices.  Returns the pool size (0: none could be loaded --
    the epilogue then runs on scipy's zheevr itself, correct but serialised).

    Process-wide side effect: every copy occupies a glibc link namespace (about 16 per
    process) and static-TLS space for the life of the process.  The first call's outcome
    -- full, partial or failed -- is cached here and in the library: later calls never
    load again ("Host epilogue")."""
    global _pool_size
    if _pool_size is not None:
        return _pool_size
    import glob
    import scipy
    libs = sorted(glob.glob(os.path.join(os.path.dirname(os.path.dirname(scipy.__file__)), "scipy.libs",
                                         "libscipy_openblas*.so")))
    got = ctypes.c_int(0)
    if not libs or load().ryd_lapack_pool(scipy_zheevr(), libs[0].encode(), b"scipy_zheevr_",
                                          b"scipy_openblas_set_num_threads", copies, ctypes.byref(got)) != 0:
        _pool_size = 0
        return 0
    _pool_size = got.value
    return _pool_size
