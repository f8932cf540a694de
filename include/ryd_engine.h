/*
 * ryd_engine.h -- C-ABI of the MI355X batched Lindblad engine for the
 * two-atom Rydberg CZ gate (libryd_engine.so, loaded through ctypes).
 *
 * Drop-in boundary.  The reference has no FFI; its replaceable seams are plain
 * Python functions:
 *   evolve_state(H, psi0, tlist, c_ops, options) -> Qobj
 *       src/qpu_simulator/micro_physics/neutral_atoms/rydberg_gates/simulation.py:647-690
 *       (one state, one segment per call -> qutip.mesolve :689)
 *   evolve_two_pulse[_lp]  :693-776, evolve_smooth_sinusoidal_jp :1502-1760,
 *   evolve_bangbang_jp :1795-1943, evolve_shaped_pulse :2099-2231
 *       (the per-protocol loops over the 4 basis inputs and all segments)
 * ryd_run_batch() replaces ALL of these for a whole sweep: every parameter
 * point x 4 computational-basis inputs x every segment of the protocol, in one
 * launch.  The Python host layer (noisyquantumsimulator_amd.simulation) keeps
 * simulate_CZ_gate()'s signature (:2534-2567) on top of it.
 *
 * Data layout (all float64, structure-of-arrays so lanes read coalesced):
 *   params  [RYD_NPARAM][ld_params]     column f of point i at params[f*ld + i]
 *   state   [width][ld_state]           one row per (point, input) lane,
 *                                       lane = 4*i + input, input = 2*a1 + a2
 *                                       (labels "00","01","10","11")
 *   summary [RYD_NSUMMARY][ld_summary]  per point
 *   status  [n]                         RYD_STATUS_* bits per point
 * Lindblad state rows: the 25 real coordinates R[i][j] (i: atom 1, j: atom 2)
 * of rho = sum_ij R[i][j] e_i (x) e_j over the single-atom Hermitian basis
 * e = {|0><0|, |1><1|, |r><r|, |1><r|+|r><1|, i(|1><r|-|r><1|)}.  This is the
 * exact invariant sector of the 4 basis inputs (each atom's {1,r}-excitation
 * number is conserved by H and every c_op of RG/noise_models.py:1449-1620);
 * every other element of rho is structurally zero, as in QuTiP.  The host
 * expands it to the QuTiP column-stacked 9x9 rho (noisyquantumsimulator_amd.engine).
 * Ket state rows: 9 complex amplitudes, interleaved (re, im), basis 3*a1 + a2.
 * dim 4 (mJ sublevels): Lindblad rows are the 36 coordinates R[i][j] over
 * e = {|0><0|, |1><1|, |r+><r+|, |1><r+|+h.c., i(|1><r+|-h.c.), |r-><r-|} (the sigma+
 * drive never couples |r->, and no jump creates an |r-> coherence, so this is again
 * the exact invariant sector); ket rows are 16 complex amplitudes, basis 4*a1 + a2.
 *
 * Ownership/threading: the caller owns every buffer; the library never keeps a
 * pointer after return (device-buffer calls: until the stream work completes).
 * One handle per host thread.  Errors: negative return + ryd_last_error()
 * (thread-local).  Per-point failures never abort a batch: they set status bits
 * (the analogue of the reference's exception -> 1e6/NaN sentinels,
 * RG/optimize_cz_gate.py:1174-1177, examples/research_parameter_sweeps.py:133-135).
 */
#ifndef RYD_ENGINE_H
#define RYD_ENGINE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RYD_ABI_VERSION 5

/* ---- return codes ---- */
#define RYD_OK              0
#define RYD_ERR_INVALID    -1
#define RYD_ERR_HIP        -2
#define RYD_ERR_UNSUPPORTED -3
#define RYD_ERR_ALLOC      -4

/* ---- protocols (schedules generated on-device from per-point scalars) ---- */
#define RYD_PROTO_LP_SQUARE 0   /* 2 constant pulses: Omega, Omega*xi      (:693-776)   */
#define RYD_PROTO_LP_SHAPED 1   /* 2 x (n_steps-1) midpoint segments        (:2099-2231) */
#define RYD_PROTO_BANGBANG  2   /* <= 8 constant-phase segments, Delta = 0  (:1795-1943) */
#define RYD_PROTO_SMOOTH_JP 3   /* n_steps midpoint-phase segments          (:1502-1760) */

#define RYD_EVOL_LINDBLAD 0     /* rho (c_ops present)                                   */
#define RYD_EVOL_KET      1     /* Schrodinger (include_noise=False -> kets, :683-690)    */

#define RYD_METHOD_CHEBYSHEV      0  /* auto (Lindblad): propagator kernel for LP square,
                                         bang-bang and smooth JP, vector otherwise; kets:
                                         vector                                            */
#define RYD_METHOD_DOPRI5         1  /* adaptive Dormand-Prince 5(4) (reference-style stepper) */
#define RYD_METHOD_CHEB_VECTOR    2  /* Chebyshev on the 4 input states, one lane each      */
#define RYD_METHOD_CHEB_SQUARING  3  /* Chebyshev on 25 basis columns of exp(L dt/2^s),
                                         then s squarings in LDS (Lindblad only); segments
                                         that differ only in laser phase share one
                                         propagator (LP square, smooth JP)                  */

#define RYD_SHAPE_SQUARE   0
#define RYD_SHAPE_GAUSSIAN 1
#define RYD_SHAPE_COSINE   2
#define RYD_SHAPE_BLACKMAN 3

#define RYD_FLAG_SYMMETRIC_ATOMS 1u  /* atom-B rate columns equal atom-A: faster path */

/* ---- per-point parameter columns ---- */
#define RYD_P_OMEGA      0   /* |Omega| rad/s (two-photon Rabi)                          */
#define RYD_P_DELTA      1   /* static detuning of the segments: H -= Delta P_r (LP Delta,
                                smooth-JP two-photon delta; ignored by BANGBANG)         */
#define RYD_P_V          2   /* blockade V rad/s (H += V P_rr)                           */
#define RYD_P_DELTA1     3   /* qubit light shift on |1>: delta_zeeman + delta_stark     */
#define RYD_P_G1_A       4   /* atom A: |1><r| rate                                      */
#define RYD_P_G0_A       5   /* atom A: |0><r| rate (decay-to-0 + bbr + losses + leakage) */
#define RYD_P_GPHI_A     6   /* atom A: P_r dephasing                                    */
#define RYD_P_GSC_A      7   /* atom A: P_1 dephasing (intermediate scattering)          */
#define RYD_P_G1_B       8
#define RYD_P_G0_B       9
#define RYD_P_GPHI_B     10
#define RYD_P_GSC_B      11
#define RYD_P_TAU        12  /* LP: single pulse tau; smooth JP: total tau                */
#define RYD_P_XI_RE      13  /* LP second pulse factor e^{i xi}                           */
#define RYD_P_XI_IM      14
#define RYD_P_AREA_CORR  15  /* shaped LP peak scale                                      */
#define RYD_P_A          16  /* smooth JP amplitude A                                     */
#define RYD_P_OMEGA_MOD  17  /* smooth JP omega_mod (rad/s)                               */
#define RYD_P_PHI_OFF    18  /* smooth JP phase offset                                    */
#define RYD_P_OMEGA_TAU  19  /* bang-bang total pulse area                                */
#define RYD_P_NSEG       20  /* bang-bang number of segments (<= 8)                       */
#define RYD_P_SWT0       21  /* bang-bang dimensionless switching times [7]               */
#define RYD_P_PHI0       28  /* bang-bang segment phases [8]                              */
#define RYD_P_GMJ_A      36  /* dim 4: atom A mJ mixing |r-><r+| and |r+><r-| rate        */
#define RYD_P_GMJ_B      37
#define RYD_NPARAM       38

/* ---- per-point summary columns ---- */
#define RYD_S_POP0       0   /* <x|rho_x|x> (or |<x|psi_x>|^2), x = 00,01,10,11 (4 cols) */
#define RYD_S_OV_RE0     4   /* ket: Re <x|psi_x> (4 cols); Lindblad: NaN                 */
#define RYD_S_OV_IM0     8   /* ket: Im <x|psi_x> (4 cols)                                */
#define RYD_S_AVG_POP    12  /* mean population fidelity (no phase penalty)              */
#define RYD_S_CTRL_PHASE 13  /* ket: wrapped phi11-phi01-phi10+phi00                      */
#define RYD_S_PENALTY    14  /* ket: cos^2(err/2)                                         */
#define RYD_S_AVG_F      15  /* ket: reference avg fidelity (F11 penalised); Lindblad: =AVG_POP */
#define RYD_S_NMV_USEFUL 16  /* generator applications needed, whole point (flop accounting) */
#define RYD_S_NMV_EXEC   17  /* generator applications executed, whole point (wave-uniform)  */
#define RYD_S_TRACE11    18  /* Tr rho_11 (Lindblad sanity), ket: |psi_11|^2              */
#define RYD_S_NSQUARE    19  /* scaling-and-squaring depth s: the propagator is exp(L dt / 2^s)^(2^s),
                                * summed over the point's builds.  Every kernel performs s matrix
                                * squarings, except the identical-atom LP-square path, which performs
                                * s - min(s, ryd_lp_unsquared()) and applies the remaining
                                * 2^min(s, ryd_lp_unsquared()) factor to the states segment by segment */
#define RYD_NSUMMARY     20

/* ---- process-map coherences (ryd_run_coherences), rows of out_coh ----------
 * The qubit process map of the gate (the reference's
 * top-level noise_models/ Kraus/CPTP extraction, src/qpu_simulator/noise_models/
 * __init__.py:1-22, is a stub): the diagonal inputs |x><x| come from
 * ryd_run_batch (Lindblad state rows); the 6 upper off-diagonal qubit matrix
 * units |a><b| are evolved here, each in its excitation-number sector, and their
 * images projected on the qubit block are returned as (re, im) row pairs:
 *   RYD_C_K0 + 4s + 2o    input s in {|00><01|, |10><11|}, output coefficient
 *                         o in {|00><01|, |10><11|}
 *   RYD_C_K1 + 4s + 2o    input s in {|00><10|, |01><11|}, output o in {|00><10|, |01><11|}
 *   RYD_C_K2              |00><11| -> coefficient of |00><11|
 *   RYD_C_K3              |01><10| -> coefficient of |01><10|
 * (no other qubit-block element is reachable from these inputs; the remaining
 * 6 units are the adjoints).                                                   */
#define RYD_C_K0   0
#define RYD_C_K1   8
#define RYD_C_K2  16
#define RYD_C_K3  18
#define RYD_NCOH  20

/* ---- three-atom blockade, quantum-jump trajectories (ryd_run_trajectories) ----
 * BASELINE configs[4].  The reference has no 3-atom model; this
 * build defines it: three identical atoms on an equilateral triangle (pairwise
 * V P_r(x)P_r), the single-atom H of the two-atom path, the 4 channels per atom
 * (atom-A rate columns RYD_P_G1_A..GSC_A used for every atom), any protocol
 * schedule.  Waiting-time Monte-Carlo wave functions: n_traj trajectories per
 * point, Philox4x32-10 counter RNG keyed (seed; trajectory, jump cycle, global
 * point index).  Kets: 27 amplitudes, basis 9 a0 + 3 a1 + a2 (a: 0, 1, 2 = r).
 * Outputs (point-major rows, one per point):
 *   rho     [n][ld_rho >= RYD_T_RHO_WIDTH]  mean of |psi><psi| over trajectories,
 *           QuTiP column-stacked vec(rho) as (re, im): element (a, b) at 2 (a + 27 b)
 *   se      [n][ld_se >= RYD_T_SE_WIDTH]    standard error of element (a, b) at a + 27 b:
 *           sqrt((mean |X|^2 - |mean X|^2) / (n_traj - 1))
 *   summary [RYD_T_NSUMMARY][ld_summary]    RYD_TS_* per point
 *   records [n][n_traj][RYD_T_REC_WIDTH]    optional (NULL = off), per trajectory:
 *           final normalised ket, jump count, the first RYD_T_REC_JUMPS (time s,
 *           channel 4 atom + c; c = 0 |1><r|, 1 |0><r|, 2 P_r, 3 P_1), iterations */
#define RYD_T_DIM          27
#define RYD_T_RHO_WIDTH    1458
#define RYD_T_SE_WIDTH     729
#define RYD_T_EXACT        0     /* ladder_levels: exact jump times (eigen-decomposed H_eff) */
#define RYD_T_LADDER_MAX   40    /* jump times resolved to segment / 2^ladder_levels     */
#define RYD_T_REC_WIDTH    64
#define RYD_T_REC_NJUMPS   54
#define RYD_T_REC_JUMP0    55
#define RYD_T_REC_JUMPS    4
#define RYD_T_REC_ITERS    63
#define RYD_TS_MEAN_JUMPS  0
#define RYD_TS_FRAC_JUMPED 1
#define RYD_TS_MAX_JUMPS   2
#define RYD_TS_TRACE       3     /* trace of the mean rho                               */
#define RYD_TS_QUBIT_POP   4     /* population left in the 8 qubit states               */
#define RYD_TS_ITER_USEFUL 5     /* ladder steps, summed over trajectories (flops)      */
#define RYD_TS_ITER_EXEC   6     /* lane-steps the waves executed (divergence included) */
#define RYD_TS_NLADDER     7     /* ladders built (one per distinct |Omega|, Delta, dt) */
#define RYD_TS_NSQUARE     8     /* block squarings performed building them             */
#define RYD_TS_RESERVED    9     /* adapted-basis kernel: (I + X) applications; else 0 */
#define RYD_T_NSUMMARY     10

/* exact mode (ladder_levels = RYD_T_EXACT) kernel selection.  Both compute the same jump
 * times (Newton on the eigen-decomposed H_eff) from the same Philox streams; they differ in
 * the work mapping and so in the rounding of the sums (outputs agree to ~1e-15).  Every shard
 * of a multi-GPU run must use the same one as its single-launch reference. */
#define RYD_T_FLAG_ROWS  1u   /* one trajectory per 16-lane DPP row, pass 1 once per point
                                 (traj3p_kernel + traj3r_kernel)                              */
#define RYD_T_FLAG_LANES 2u   /* one trajectory per lane, points paired per wave, ranges
                                 split over waves for small launches (traj3e_kernel); the
                                 default                                                      */
typedef struct ryd_traj_desc {
  int32_t abi_version;     /* = RYD_ABI_VERSION */
  int32_t protocol;        /* RYD_PROTO_* */
  int32_t shape;           /* RYD_SHAPE_* (LP_SHAPED) */
  int32_t n_steps;         /* as ryd_batch_desc */
  int32_t n_traj;          /* trajectories per point: a multiple of 64 */
  int32_t ladder_levels;   /* RYD_T_EXACT: exact jump times (Newton on the eigen-
                              decomposed H_eff), for schedules with a
                              constant |Omega| and Delta (not a shaped LP envelope);
                              1 .. RYD_T_LADDER_MAX: the ladder walk, jump times
                              resolved to segment / 2^ladder_levels */
  uint32_t flags;          /* RYD_T_FLAG_*: which exact-mode kernel (0: the library's default) */
  uint32_t point_stride;   /* global index of point i = point_offset + point_stride * i (the
                              trajectories' random-stream key); 0 and 1: contiguous.  A strided
                              shard (rank r of N: offset r, stride N) reproduces rows r, r + N,
                              ... of the whole launch */
  uint64_t seed;
  double psi0[2 * RYD_T_DIM];  /* normalised initial ket, (re, im) interleaved */
} ryd_traj_desc;

/* ---- per-point status bits ----
 * Set by the kernels (failures: the analogue of the reference's exceptions -> 1e6 /
 * NaN sentinels): */
#define RYD_STATUS_NONFINITE   1u
#define RYD_STATUS_STEP_CAP    2u   /* DOPRI5 step cap (ZVODE nsteps analogue)          */
#define RYD_STATUS_BAD_INPUT   4u   /* Omega <= 0, tau <= 0, nseg out of range ...      */
#define RYD_STATUS_FAIL_MASK   7u
/* Warnings (the reference's UserWarnings, per point instead of per call; set by the
 * host layer's derivation, never by the kernels): */
#define RYD_STATUS_WEAK_BLOCKADE  8u   /* LP: V/Omega < 10 (RG/protocols.py:615-619); smooth JP:
                                          V/Omega < 5 (RG/simulation.py:1670-1676)          */
#define RYD_STATUS_DARK_STATE_SIGN 16u /* smooth JP: delta/Omega of the wrong sign for the
                                          intermediate detuning (RG/simulation.py:1631-1647) */
#define RYD_STATUS_OMEGA_RANGE   32u   /* Omega/2pi > 100 MHz or < 0.1 MHz (:2930-2946)     */
/* Set by ryd_mixed_phase: the reference's mixed-state phase penalty is not a function
 * of rho at the checked precision (LAPACK eigenvector gauge, see below). */
#define RYD_STATUS_GAUGE_UNSTABLE 64u
/* Set by ryd_run_trajectories in exact mode (RYD_T_EXACT): the point's |Omega| or Delta
 * changes between segments, or its H_eff eigen-decomposition is unconverged or
 * ill-conditioned (near an exceptional point); the point ran on the L = 16 ladder walk
 * instead (jump times resolved to segment / 2^16).  A warning, not a failure. */
#define RYD_STATUS_EXACT_FALLBACK 128u

typedef struct ryd_batch_desc {
    int32_t abi_version;     /* = RYD_ABI_VERSION */
    int32_t dim;             /* single-atom levels: 3, or 4 (|0>,|1>,|r+>,|r->; sigma+ drive,
                                RG/hamiltonians.py:490-516, :655-679, :741-753, :835-853;
                                methods CHEBYSHEV / CHEB_VECTOR only) */
    int32_t protocol;        /* RYD_PROTO_* */
    int32_t evolution;       /* RYD_EVOL_* */
    int32_t method;          /* RYD_METHOD_* */
    int32_t shape;           /* RYD_SHAPE_* (LP_SHAPED) */
    int32_t n_steps;         /* SMOOTH_JP segments (ref 300), LP_SHAPED n_time_steps (ref 500),
                                BANGBANG: max segments in the batch */
    uint32_t flags;          /* RYD_FLAG_* */
    double rtol;             /* DOPRI5 */
    double atol;             /* DOPRI5 */
    int64_t max_steps;       /* DOPRI5 step cap per segment */
} ryd_batch_desc;

typedef struct ryd_stats {
    double kernel_ms;        /* device time of the propagation kernel(s) */
    double h2d_ms;
    double d2h_ms;
    double matvec_useful;    /* sum over points of RYD_S_NMV_USEFUL */
    double matvec_exec;
    int32_t n_devices;
    int32_t reserved;
} ryd_stats;

typedef struct ryd_handle ryd_handle;

int         ryd_abi_version(void);
const char* ryd_last_error(void);
int         ryd_param_count(void);
int         ryd_summary_width(void);
int         ryd_state_width(int evolution, int dim);
/* squaring levels the identical-atom LP-square kernel leaves unsquared (see RYD_S_NSQUARE) */
int         ryd_lp_unsquared(void);
int         ryd_device_count(int* count);

int ryd_create(const int* device_ids, int n_devices, ryd_handle** out);
int ryd_destroy(ryd_handle* h);

/* Host buffers in/out; range-partitions the points over the handle's devices
 * (one stream each, no inter-device communication), blocks until done. */
int ryd_run_batch(ryd_handle* h, const ryd_batch_desc* desc,
                  const double* params, int64_t n, int64_t ld_params,
                  double* out_state, int64_t ld_state,
                  double* out_summary, int64_t ld_summary,
                  uint32_t* out_status, ryd_stats* stats);

/* Device buffers already resident on device slot `slot`; enqueues on `stream`
 * (hipStream_t, NULL = the handle's stream for that slot) and returns.
 * If `elapsed_ms` is non-NULL the call records HIP events around the launch on
 * that stream, waits, and reports the kernel's device time. */
int ryd_run_batch_device(ryd_handle* h, int slot, const ryd_batch_desc* desc,
                         const double* d_params, int64_t n, int64_t ld_params,
                         double* d_state, int64_t ld_state,
                         double* d_summary, int64_t ld_summary,
                         uint32_t* d_status, void* stream, float* elapsed_ms);

/* Process-map coherences (layout above).  Chebyshev state-vector method; any
 * protocol, either evolution value (rates may be zero).  Host-buffer form
 * range-partitions like ryd_run_batch; status bits as ryd_run_batch. */
int ryd_run_coherences(ryd_handle* h, const ryd_batch_desc* desc,
                       const double* params, int64_t n, int64_t ld_params,
                       double* out_coh, int64_t ld_coh,
                       uint32_t* out_status, ryd_stats* stats);
int ryd_run_coherences_device(ryd_handle* h, int slot, const ryd_batch_desc* desc,
                              const double* d_params, int64_t n, int64_t ld_params,
                              double* d_coh, int64_t ld_coh, uint32_t* d_status,
                              void* stream, float* elapsed_ms);

/* Three-atom quantum-jump trajectories (layout above).  Host-buffer form:
 * range-partitions the points over the handle's devices; rho and se are packed
 * (ld = RYD_T_RHO_WIDTH / RYD_T_SE_WIDTH); records may be NULL.  stats->
 * matvec_useful / matvec_exec carry the summed RYD_TS_ITER_USEFUL / _EXEC. */
int ryd_run_trajectories(ryd_handle* h, const ryd_traj_desc* desc,
                         const double* params, int64_t n, int64_t ld_params,
                         double* out_rho, double* out_se,
                         double* out_summary, int64_t ld_summary,
                         double* out_records, uint32_t* out_status, ryd_stats* stats);
/* Device form; point_offset = global index of point 0 (the RNG key), so range
 * shards run by separate processes draw the same streams as one big batch. */
int ryd_run_trajectories_device(ryd_handle* h, int slot, const ryd_traj_desc* desc,
                                const double* d_params, int64_t n, int64_t ld_params,
                                int64_t point_offset,
                                double* d_rho, int64_t ld_rho, double* d_se, int64_t ld_se,
                                double* d_summary, int64_t ld_summary, double* d_records,
                                uint32_t* d_status, void* stream, float* elapsed_ms);

/* ---- host epilogue: the reference's mixed-state controlled phase ----
 * RG/simulation.py:424-452 takes, for each output rho_x (x = 00, 01, 10, 11), the
 * eigenvector of the largest eigenvalue (rho.eigenstates(): QuTiP 5 -> scipy.linalg.
 * eigh -> LAPACK zheevr, JOBZ 'V', RANGE 'A', UPLO 'L', ABSTOL 0) and its phase at
 * |x>; cp = wrap(phi11 - phi01 - phi10 + phi00), penalty cos^2(err/2), err = min|cp -+
 * pi| (:444-452).  Output: the component <x|v_max> per input (the phase is its angle).  `zheevr` is the caller's LAPACK zheevr (Fortran ABI, 32-bit ints;
 * the Python layer passes scipy's, so the phases equal scipy.linalg.eigh's bit for
 * bit).  `state` = Lindblad sector rows as ryd_run_batch writes them ([25 | 36][ld]).
 * Gauge check (round 4 semantics): probe (x, c) replaces rho_x alone by copy c of it,
 * the real and imaginary parts of every lower-triangle entry scaled independently by
 * (1 +- rel_eps) (copy 1 all +, copy 2 all -, then splitmix64 sign patterns), the other
 * three rho unperturbed; rho_11 first, then rho_00, rho_01, rho_10, c = 1..n_perturb
 * each (one zheevr call per probe); out_flags[i] |= RYD_STATUS_GAUGE_UNSTABLE at the
 * first probe whose penalty moves by more than tol.  Rounds 1-3 perturbed all four rho
 * together; a flip that needs two phases to move together is not probed any more.  The
 * oracle's gauge_unstable (scheme "one_rho") is this procedure on scipy.linalg.eigh.  Host only, n_threads worker threads (0 = all cores). */
#define RYD_MP_V0       0   /* <x|v_max> as (re, im) row pairs, x = 00, 01, 10, 11; the
                               phase is its angle (taken by the caller: the reference
                               uses np.angle)                                       */
#define RYD_MP_CTRL     8   /* wrapped controlled phase (libm atan2; gauge check)    */
#define RYD_MP_PENALTY  9   /* cos^2(err / 2)                                       */
#define RYD_MP_SPREAD   10  /* max |penalty(perturbed) - penalty|                   */
#define RYD_MP_WIDTH    11
int ryd_mixed_phase(void* zheevr, int dim, const double* state, int64_t n, int64_t ld_state,
                    int n_perturb, double rel_eps, double tol, int n_threads,
                    double* out, int64_t ld_out, uint32_t* out_flags);

/* Private LAPACK instances for the threaded epilogue.  The pool is ref_zheevr itself
 * plus up to `copies` - 1 copies of the shared object `path` loaded into fresh link
 * namespaces (dlmopen), each set to one BLAS
 * thread (`threads_symbol`, may be NULL), and admits a copy only if its `zheevr_symbol`
 * reproduces `ref_zheevr` bit for bit on test matrices.  ryd_mixed_phase called with
 * ref_zheevr then runs one instance per worker thread (min(n_threads, pool size)
 * threads): OpenBLAS serialises concurrent callers of one instance on a process-wide
 * lock.  *n_loaded = pool size (loading stops quietly when namespaces or static TLS run
 * out); an error only if no copy could be loaded.  PROCESS-WIDE SIDE EFFECT: each copy
 * occupies a glibc link namespace and static-TLS space for the life of the process, so
 * copies are capped at 15 and loading is attempted once per process: later calls return
 * the first attempt's outcome (partial or failed) and never call dlmopen again. */
int ryd_lapack_pool(void* ref_zheevr, const char* path, const char* zheevr_symbol,
                    const char* threads_symbol, int copies, int* n_loaded);

/* The generic evolve_state seam (RG/simulation.py:647-690: mesolve(H, psi0, tlist, c_ops)
 * for any H and c_ops, SURVEY.md §8b's GENERIC_SCHEDULE with a generic jump-operator
 * list).  For each of n problems: n_seg piecewise-constant segments (H_s, dt_s), n_ops
 * jump operators L_k shared by the segments, evolve
 *     drho/dt = -i [H_s, rho] + sum_k (L_k rho L_k^dag - {L_k^dag L_k, rho} / 2)
 * (or, ket != 0 and n_ops == 0, dpsi/dt = -i H_s psi) from state0 and write the final
 * state.  Complex arrays are interleaved (re, im), matrices row-major:
 *   H [n][n_seg][dim][dim], dt [n][n_seg] (segments with dt <= 0 are skipped),
 *   ops [n][n_ops][dim][dim] (nullable when n_ops == 0),
 *   state0 / state_out [n][dim][dim] (density) or [n][dim] (ket).
 * dim <= 16, n_ops <= 32, at most 1024 nonzero operator entries per problem.  Exact
 * propagation per segment (Chebyshev series of exp(dt L), tail < 1e-17) on the handle's
 * first device; host buffers, blocking.  status[i]: RYD_STATUS_STEP_CAP (omega dt above
 * 2e6 rad, or more than 2e5 series terms, in one segment -- mesolve's nsteps cap; the state
 * is the last one reached), RYD_STATUS_NONFINITE. */
int ryd_evolve_generic(ryd_handle* h, int dim, int n_seg, int n_ops, int64_t n, int ket,
                       const double* H, const double* dt, const double* ops,
                       const double* state0, double* state_out, uint32_t* status);

/* ---- hot-path row a1 on the device: parameter derivation (ryd_derive) ----
 * The reference derives every point's physics on the host, one simulate_CZ_gate call at
 * a time: steps 0-8 of RG/simulation.py:2761-3355 (Rabi frequencies RG/laser_physics.py:
 * 111-427, blockade V = C6/R^6, the LP (Delta/Omega, Omega tau) lookup RG/protocols.py:
 * 562-651 and xi :747-819, trap-dependent noise RG/trap_physics.py:1614-1848, Zeeman /
 * Stark shifts :1851-2142, the noise rates :3230-3334 with RG/noise_models.py:483-963).
 * ryd_derive evaluates the same formulas elementwise on the GPU, from per-point input
 * fields straight into the engine's parameter block ([RYD_NPARAM][ld_params], the layout
 * ryd_run_batch reads), so a 1M-point sweep (C4: species x T x P_tweezer) never builds
 * its parameters on the host.  Each input field is either one value for every point
 * (desc->value[f], desc->col[f] < 0) or row desc->col[f] of the caller's input block
 * ([n_cols][ld_in] float64).  NaN means "not given" where the reference has a None
 * default (linewidths, tweezer wavelength, background loss, LP delta/Omega and
 * Omega tau, the signed smooth-JP delta/Omega); smooth-JP A / omega_mod_ratio / phi_offset
 * of 0 take the defaults (the reference's `x or default`).  Species constants are the
 * caller's table (noisyquantumsimulator_amd.species, RG/atom_database.py:104).
 * Outputs: params (every column the protocol reads; the others 0), warn[i] = the
 * RYD_STATUS_WEAK_BLOCKADE / DARK_STATE_SIGN / OMEGA_RANGE warning bits, and optionally
 * the derived diagnostic columns diag [RYD_DV_NDIAG][ld_diag] (NULL = off). */
#define RYD_DV_SPECIES      0   /* index into desc->species                              */
#define RYD_DV_N_RYD        1
#define RYD_DV_P1           2   /* laser 1 power W, waist m                              */
#define RYD_DV_P2           3
#define RYD_DV_W1           4
#define RYD_DV_W2           5
#define RYD_DV_DELTA_E      6   /* intermediate detuning rad/s                           */
#define RYD_DV_LW1          7   /* laser linewidths Hz (NaN: None)                       */
#define RYD_DV_LW2          8
#define RYD_DV_TW_POWER     9
#define RYD_DV_TW_WAIST     10
#define RYD_DV_TW_WL_NM     11  /* NaN: the species' default trap wavelength             */
#define RYD_DV_TEMPERATURE  12
#define RYD_DV_B_FIELD      13
#define RYD_DV_NA           14
#define RYD_DV_SPACING      15
#define RYD_DV_BG_LOSS      16  /* NaN: 1e3 /s                                           */
#define RYD_DV_DOM          17  /* LP / smooth JP delta/Omega (NaN: lookup / default)    */
#define RYD_DV_OMEGA_TAU    18  /* NaN: lookup / protocol default                        */
#define RYD_DV_SJP_A        19  /* smooth JP A, omega_mod/Omega, phi_offset (0: default) */
#define RYD_DV_SJP_OMR      20
#define RYD_DV_SJP_PHI_OFF  21
#define RYD_DV_SJP_SDOM     22  /* signed smooth-JP delta/Omega override (NaN: derived)  */
#define RYD_DV_BB_SWT0      23  /* bang-bang switching times [7] and phases [8]          */
#define RYD_DV_BB_PHI0      30
#define RYD_DV_NFIELD       38
/* species table row: mass, alpha_ground, trap_wavelength, n_ref, C6_ref, tau_0K_ref,
 * tau_ref, alpha_rydberg_ref, dipole_er_ref, qd_S, dipole_1e, gamma_e, f_ground_to_e,
 * E_ionization, omega_D1, K_quad_zeeman, K_quad_noise, stark_hz_per_mK, g_F_lower,
 * F_lower, exp_C6, exp_tau0, exp_tau_bbr, exp_alpha */
#define RYD_DV_NSPC         24
#define RYD_DV_MAX_SPECIES  4
/* flags */
#define RYD_DV_NOISE        1u   /* include_noise                                          */
#define RYD_DV_TRAP_ON      2u   /* trap_laser_on (Stark shift)                            */
#define RYD_DV_DOPPLER      4u   /* NoiseSourceConfig.include_doppler_dephasing            */
#define RYD_DV_INTENSITY    8u   /* include_intensity_noise                                */
#define RYD_DV_COUNTERPROP  16u  /* TwoPhotonExcitationConfig.counter_propagating          */
#define RYD_DV_MOTIONAL     32u  /* include_motional_dephasing                             */
/* leakage spectral factor (RG/noise_models.py:732-853): the pulse shape's name */
#define RYD_DV_LEAK_SQUARE   0
#define RYD_DV_LEAK_GAUSSIAN 1
#define RYD_DV_LEAK_COSINE   2
#define RYD_DV_LEAK_BLACKMAN 3
#define RYD_DV_LEAK_OTHER    4   /* smooth_sinusoidal, bangbang: sinc^2 with +1e-10       */
/* diagnostic columns (the DerivedBatch fields of the same name) */
#define RYD_DV_D_OMEGA1        0
#define RYD_DV_D_OMEGA         1
#define RYD_DV_D_V             2
#define RYD_DV_D_R             3
#define RYD_DV_D_U0            4
#define RYD_DV_D_OMEGA_R       5
#define RYD_DV_D_SIGMA_R       6
#define RYD_DV_D_DVV           7
#define RYD_DV_D_G_THERMAL     8
#define RYD_DV_D_G_SCATTER     9
#define RYD_DV_D_ALPHA_G       10
#define RYD_DV_D_ALPHA_R       11
#define RYD_DV_D_ALPHA_RATIO   12
#define RYD_DV_D_G_ANTITRAP    13
#define RYD_DV_D_DIFF_SHIFT    14
#define RYD_DV_D_ENHANCEMENT   15
#define RYD_DV_D_K_EFF         16
#define RYD_DV_D_V_THERMAL     17
#define RYD_DV_D_G_DOPPLER     18
#define RYD_DV_D_G_INTENSITY   19
#define RYD_DV_D_GAMMA_R_TRAP  20
#define RYD_DV_D_WAVELENGTH_NM 21
#define RYD_DV_D_TAU_SINGLE    22
#define RYD_DV_D_TAU_TOTAL     23
#define RYD_DV_D_DELTA_GATE    24
#define RYD_DV_D_DOM           25
#define RYD_DV_D_OMEGA_TAU     26
#define RYD_DV_D_DELTA_ZEEMAN  27
#define RYD_DV_D_DELTA_STARK   28
#define RYD_DV_D_V_OVER_OMEGA  29
#define RYD_DV_D_XI_RE         30
#define RYD_DV_D_XI_IM         31
#define RYD_DV_D_DELTA_SEG     32
#define RYD_DV_D_GAMMA_R       33   /* the noise rates (0 without include_noise)          */
#define RYD_DV_D_GAMMA_PHI_LASER   34
#define RYD_DV_D_GAMMA_PHI_THERMAL 35
#define RYD_DV_D_GAMMA_PHI_ZEEMAN  36
#define RYD_DV_D_GAMMA_LOSS_ANTITRAP 37
#define RYD_DV_D_GAMMA_LOSS_BG     38
#define RYD_DV_D_GAMMA_LEAKAGE     39
#define RYD_DV_D_GAMMA_SCATTER     40
#define RYD_DV_D_MJ_RATE           41
#define RYD_DV_D_AREA_CORR         42
#define RYD_DV_NDIAG           43

typedef struct ryd_derive_desc {
  int32_t abi_version;       /* = RYD_ABI_VERSION */
  int32_t protocol;          /* RYD_PROTO_* */
  int32_t shape;             /* RYD_SHAPE_* (LP_SHAPED: area correction) */
  int32_t leak_shape;        /* RYD_DV_LEAK_* */
  int32_t dim;               /* 3 | 4 (dim 4: the mJ-mixing rate columns) */
  uint32_t flags;            /* RYD_DV_* flags */
  int32_t n_species;         /* rows of species[] in use */
  int32_t bb_nseg;           /* bang-bang segments (= phases), 0 otherwise */
  double qubit[4];           /* F0, mF0, F1, mF1 */
  double intensity_noise_frac;
  double polarization_purity;  /* min of the two lasers' (dim 4) */
  double species[RYD_DV_MAX_SPECIES][RYD_DV_NSPC];
  double value[RYD_DV_NFIELD];
  int32_t col[RYD_DV_NFIELD];
} ryd_derive_desc;

/* Device form: d_in [n_cols][ld_in] on slot `slot` (may be NULL if every col < 0);
 * d_params [RYD_NPARAM][ld_params]; d_warn [n]; d_diag nullable.  Enqueues on `stream`
 * (NULL: the slot's stream); elapsed_ms as ryd_run_batch_device. */
int ryd_derive_device(ryd_handle* h, int slot, const ryd_derive_desc* desc,
                      const double* d_in, int64_t ld_in, int64_t n,
                      double* d_params, int64_t ld_params, uint32_t* d_warn,
                      double* d_diag, int64_t ld_diag, void* stream, float* elapsed_ms);
/* Host form (blocking, the handle's first device): in [n_cols][ld_in] host (NULL if every
 * col < 0), params [RYD_NPARAM][ld_params], warn [n], diag nullable. */
int ryd_derive(ryd_handle* h, const ryd_derive_desc* desc, const double* in, int64_t n_cols,
               int64_t ld_in, int64_t n, double* params, int64_t ld_params, uint32_t* warn,
               double* diag, int64_t ld_diag);

/* Timeline of the handle's last host-buffer call (ryd_run_batch / _coherences /
 * _trajectories).  Those calls keep a device workspace and a pinned host staging buffer
 * per slot across calls, enqueue every slot (pack -> H2D -> kernel -> D2H into staging)
 * before the first wait, then unpack staging into the caller's buffers with host
 * threads.  out[0] = n_slots, out[1] = host pack ms, out[2] = host unpack ms,
 * out[3] = call wall ms; then per slot RYD_TL_SLOT doubles: device id, H2D start,
 * kernel start, kernel end, D2H end (ms, HIP events, relative to the start of the first
 * slot on the same device), points, then host ms since the call began at which the
 * slot's kernel was enqueued and at which the host began waiting for the slot (every
 * slot is enqueued before the first wait).  cap >= 4 + RYD_TL_SLOT * n_slots. */
#define RYD_TL_HEAD 4
#define RYD_TL_SLOT 8
int ryd_last_timeline(ryd_handle* h, double* out, int64_t cap);

/* Region timing on a slot's stream: ryd_mark(h, slot, 0) ... launches ...
 * ryd_mark(h, slot, 1); ryd_mark_elapsed waits for mark 1 and returns the device time
 * between the two (HIP events on the stream the *_device calls use by default). */
int ryd_mark(ryd_handle* h, int slot, int mark);
int ryd_mark_elapsed(ryd_handle* h, int slot, float* ms);

/* Minimal device-memory plumbing so callers need no other GPU runtime. */
int ryd_malloc(ryd_handle* h, int slot, size_t bytes, void** d_ptr);
int ryd_free(ryd_handle* h, int slot, void* d_ptr);
int ryd_memcpy_h2d(ryd_handle* h, int slot, void* d_dst, const void* src, size_t bytes);
int ryd_memcpy_d2h(ryd_handle* h, int slot, void* dst, const void* d_src, size_t bytes);
int ryd_synchronize(ryd_handle* h);

#ifdef __cplusplus
}
#endif
#endif /* RYD_ENGINE_H */
