"""Batched sweep drivers (replacing the serial loops of
examples/research_parameter_sweeps.py:81-195 and the per-point optimizer calls).

Also defines the synthetic benchmark workloads of SURVEY.md §8d.
"""
from __future__ import annotations

import warnings
from typing import Dict, Optional

import numpy as np

from . import configurations as CF
from . import physics as PH

# cz_gate_optimization_demo.ipynb ApparatusConstraints "medium" tier
MEDIUM = dict(laser_1_power=50e-6, laser_1_waist=50e-6, laser_2_power=0.3, laser_2_waist=50e-6,
              temperature=2e-6, spacing_factor=2.8, n_rydberg=70, species="Rb87",
              tweezer_power=0.020, tweezer_waist=0.8e-6, B_field=1e-4, NA=0.5)


def medium_excitation(purity: float = 0.99) -> CF.TwoPhotonExcitationConfig:
    return CF.TwoPhotonExcitationConfig(
        laser_1=CF.LaserParameters(power=MEDIUM["laser_1_power"], waist=MEDIUM["laser_1_waist"],
                                   polarization="pi", polarization_purity=purity, linewidth_hz=100.0),
        laser_2=CF.LaserParameters(power=MEDIUM["laser_2_power"], waist=MEDIUM["laser_2_waist"],
                                   polarization="sigma+", polarization_purity=purity, linewidth_hz=100.0),
        Delta_e=2 * np.pi * 1e9)


def _apparatus_kwargs(**over):
    kw = dict(species=MEDIUM["species"], n_rydberg=MEDIUM["n_rydberg"],
              tweezer_power=MEDIUM["tweezer_power"], tweezer_waist=MEDIUM["tweezer_waist"],
              temperature=MEDIUM["temperature"], spacing_factor=MEDIUM["spacing_factor"],
              B_field=MEDIUM["B_field"], NA=MEDIUM["NA"])
    kw.update(over)
    return kw


def omega_delta_grid(n_omega: int = 100, n_delta: int = 100, omega_mhz=(1.0, 10.0),
                     delta_over_omega=(0.30, 0.45), omega_tau: float = 4.29268,
                     include_noise: bool = True, delta_slice: Optional[slice] = None,
                     pulse_shape: str = "square", hilbert_space_dim: int = 3) -> PH.DerivedBatch:
    """C2: (Omega, Delta) sweep of the LP square CZ gate on the medium apparatus.

    Omega/2pi = linspace(1, 10) MHz is produced the physical way, by scaling the
    480 nm leg power (Omega ∝ sqrt(P2)); Delta/Omega = linspace(0.30, 0.45);
    Omega*tau = 4.29268; V = C6/R^6 = 2pi x 1233.83 MHz; every noise rate from the
    reference formulas per point.  ``pulse_shape`` / ``hilbert_space_dim``
    give the same grid for the shaped-LP and dim-4 kernels (bench.py secondary lines)."""
    si, n, kw = omega_delta_call(n_omega, n_delta, omega_mhz, delta_over_omega, omega_tau, include_noise,
                                 delta_slice, pulse_shape, hilbert_space_dim)
    return PH.derive_batch(si, n=n, **kw)


def omega_delta_call(n_omega: int = 100, n_delta: int = 100, omega_mhz=(1.0, 10.0),
                     delta_over_omega=(0.30, 0.45), omega_tau: float = 4.29268,
                     include_noise: bool = True, delta_slice: Optional[slice] = None,
                     pulse_shape: str = "square", hilbert_space_dim: int = 3):
    """The C2 grid as (simulation_inputs, n, keyword arguments) of derive_batch /
    simulate_CZ_gate_batch (the end-to-end form of omega_delta_grid)."""
    warnings.simplefilter("ignore")
    exc = medium_excitation()
    ref = PH.derive_batch(CF.LPSimulationInputs(excitation=exc), **_apparatus_kwargs(),
                          include_noise=False)
    om0 = ref["Omega"][0]
    om = 2 * np.pi * 1e6 * np.linspace(*omega_mhz, n_omega)
    dom = np.linspace(*delta_over_omega, n_delta)
    if delta_slice is not None:
        dom = dom[delta_slice]
    OM, DOM = np.meshgrid(om, dom, indexing="ij")
    p2 = MEDIUM["laser_2_power"] * (OM.ravel() / om0) ** 2
    si = CF.LPSimulationInputs(excitation=exc, omega_tau=omega_tau, pulse_shape=pulse_shape)
    return si, p2.size, dict(**_apparatus_kwargs(), include_noise=include_noise,
                             hilbert_space_dim=hilbert_space_dim,
                             overrides=dict(laser_2_power=p2, delta_over_omega=DOM.ravel()))


def pareto_tgate_grid(n_omega: int = 1000, n_tau: int = 100, include_noise: bool = True,
                      omega_slice: Optional[slice] = None) -> PH.DerivedBatch:
    """C3: smooth-JP fidelity vs t_gate: Omega/2pi in linspace(1,10) MHz x Omega*tau in
    linspace(5, 25), medium apparatus (reference noise model)."""
    warnings.simplefilter("ignore")
    exc = medium_excitation()
    ref = PH.derive_batch(CF.SmoothJPSimulationInputs(excitation=exc), **_apparatus_kwargs(),
                          include_noise=False)
    om0 = ref["Omega"][0]
    om = 2 * np.pi * 1e6 * np.linspace(1, 10, n_omega)
    if omega_slice is not None:
        om = om[omega_slice]
    ot = np.linspace(5, 25, n_tau)
    OM, OT = np.meshgrid(om, ot, indexing="ij")
    p2 = MEDIUM["laser_2_power"] * (OM.ravel() / om0) ** 2
    return PH.derive_batch(CF.SmoothJPSimulationInputs(excitation=exc), n=p2.size,
                           **_apparatus_kwargs(), include_noise=include_noise,
                           overrides=dict(laser_2_power=p2, omega_tau=OT.ravel()))


# C3's noise model as BASELINE configs[2] / SURVEY.md §8d state it: 4 collapse ops,
# sqrt(gamma_r)|1><r| and sqrt(gamma_phi) P_r on each atom
C3_GAMMA_R = 1.0 / 140e-6               # 7142.857 s^-1 (Rb87 n = 70 Rydberg lifetime)
C3_GAMMA_PHI = 2 * np.pi * 1e4


def c3_four_op_params(batch: PH.DerivedBatch) -> np.ndarray:
    """Packed parameters of a C3 batch with the 4-collapse-op model (Rydberg decay to
    |1> + Rydberg dephasing on each atom) in place of the full reference noise."""
    from . import engine as E
    p = E.pack_params(batch)
    P = E.N.P
    for ab in ("A", "B"):
        p[P["G1_" + ab]] = C3_GAMMA_R
        p[P["G0_" + ab]] = 0.0
        p[P["GPHI_" + ab]] = C3_GAMMA_PHI
        p[P["GSC_" + ab]] = 0.0
    return p


C4_SHAPE = (2, 1000, 500)          # species x T x P_tweezer
C4_POINTS = 2 * 1000 * 500


def species_temperature_power_grid(n_T: int = 1000, n_P: int = 500, include_noise: bool = True,
                                   point_slice: Optional[slice] = None,
                                   point_index: Optional[np.ndarray] = None) -> PH.DerivedBatch:
    """C4: species {Rb87, Cs133} x T in logspace(1, 100) uK x P_tweezer in logspace(1, 100) mW,
    LP square, medium apparatus otherwise.  Point order is
    species-major, then T, then P.  ``point_slice`` (a contiguous range shard, the
    multi-GPU partition) or ``point_index`` selects points before derivation."""
    warnings.simplefilter("ignore")
    sp = np.array(["Rb87", "Cs133"])
    T = np.logspace(-6, -4, n_T)
    P = np.logspace(-3, -1, n_P)
    S_, T_, P_ = np.meshgrid(np.arange(2), T, P, indexing="ij")
    S_, T_, P_ = S_.ravel(), T_.ravel(), P_.ravel()
    if point_slice is not None:
        S_, T_, P_ = S_[point_slice], T_[point_slice], P_[point_slice]
    if point_index is not None:
        S_, T_, P_ = S_[point_index], T_[point_index], P_[point_index]
    return PH.derive_batch(CF.LPSimulationInputs(excitation=medium_excitation()), n=T_.size,
                           **_apparatus_kwargs(species=sp[S_], temperature=T_, tweezer_power=P_),
                           include_noise=include_noise)


def c4_columns(n_T: int = 1000, n_P: int = 500, point_slice: Optional[slice] = None):
    """The C4 grid's varying columns (species-table index: 0 Rb87, 1 Cs133; T; P_tweezer),
    species-major."""
    T = np.logspace(-6, -4, n_T)
    P = np.logspace(-3, -1, n_P)
    S_, T_, P_ = np.meshgrid(np.arange(2), T, P, indexing="ij")
    S_, T_, P_ = S_.ravel(), T_.ravel(), P_.ravel()
    if point_slice is not None:
        S_, T_, P_ = S_[point_slice], T_[point_slice], P_[point_slice]
    return S_, T_, P_


def species_temperature_power_inputs(n_T: int = 1000, n_P: int = 500, include_noise: bool = True,
                                     point_slice: Optional[slice] = None) -> PH.DeriveInputs:
    """C4 as device-derivation inputs (ryd_derive): the same points as
    species_temperature_power_grid, but only the species / T / P_tweezer columns travel;
    every other field is a descriptor value, and the parameters are derived in HBM."""
    warnings.simplefilter("ignore")
    sp, T_, P_ = c4_columns(n_T, n_P, point_slice)
    return PH.derive_inputs(CF.LPSimulationInputs(excitation=medium_excitation()), n=T_.size,
                            **_apparatus_kwargs(species=sp, temperature=T_, tweezer_power=P_),
                            include_noise=include_noise)


def c4_rank_inputs(rank: int, world_size: int, include_noise: bool = True) -> PH.DeriveInputs:
    """Rank r's contiguous range of the 1M-point C4 grid as device-derivation inputs."""
    return species_temperature_power_inputs(include_noise=include_noise,
                                            point_slice=range_shard(C4_POINTS, rank, world_size))


# C1: one dim-3 LP-square point, Omega = 2 pi 5 MHz, V/Omega = 100, the LP
# defaults Delta/Omega = 0.377371 and Omega tau = 4.29268, xi from compute_phase_shift_xi,
# one collapse operator sqrt(gamma) |1><r| (x) I with gamma = 1/140 us (Rb87 n = 70)
C1_OMEGA = 2 * np.pi * 5e6
C1_V_OVER_OMEGA = 100.0
C1_GAMMA = 1.0 / 140e-6


def c1_point() -> Dict[str, float]:
    """The C1 point's physics inputs (the columns the kernel reads)."""
    from . import protocols as PR
    Om = C1_OMEGA
    Dl = PR.LP_DELTA_OVER_OMEGA_DEFAULT * Om
    tau = PR.LP_OMEGA_TAU_DEFAULT / Om
    xi = complex(PR.compute_phase_shift_xi(np.array([Dl]), np.array([Om]), np.array([tau]))[0])
    return dict(Omega=Om, V=C1_V_OVER_OMEGA * Om, Delta=Dl, tau=tau, xi=xi, gamma=C1_GAMMA)


def c1_params() -> np.ndarray:
    """C1 packed for the engine: atom A's |1><r| channel only (the c_op acts on atom A)."""
    from . import engine as E
    c = c1_point()
    P = E.N.P
    p = np.zeros((E.N.NPARAM, 1))
    p[P["OMEGA"]], p[P["DELTA"]], p[P["V"]], p[P["TAU"]] = c["Omega"], c["Delta"], c["V"], c["tau"]
    p[P["XI_RE"]], p[P["XI_IM"]] = c["xi"].real, c["xi"].imag
    p[P["AREA_CORR"]] = 1.0
    p[P["G1_A"]] = c["gamma"]
    return p


C5_SHAPE = (64, 64)                # Omega x V/Omega
C5_POINTS = 64 * 64


def blockade_grid_3atom(n_omega: int = 64, n_vo: int = 64, include_noise: bool = True,
                        point_slice: Optional[slice] = None, order: str = "omega") -> PH.DerivedBatch:
    """C5: Omega/2pi in linspace(1, 10) MHz x V/Omega in logspace(10, 1000),
    LP square, medium apparatus.  Omega is set the physical way (480 nm leg power,
    Omega ∝ sqrt(P2)) and V/Omega through the atom spacing (V = C6/R^6, via
    spacing_factor), so the LP (Delta/Omega, Omega tau) lookup, xi and every noise rate
    follow from the reference formulas per point.  The point ORDER decides how a launch's
    tail packs and how balanced the range shards are (the results do not depend on it):
      * ``"omega"`` (the default): Omega-major.  The exact-jump kernel's waves pair point b
        with its mirror, so the first-dispatched waves hold the Omega extremes -- the
        longest walks -- and the short ones fill the tail (C5, N = 1: 0.51 ms); but rank 0's
        eighth at N = 8 holds the 8 lowest Omega values (its shard 0.32 ms);
      * ``"blocked"``: 8 blocks of 8 V/Omega rows (512 points each), Omega-major inside a
        block: every range shard of N = 1, 2, 4, 8 ranks is a union of whole blocks spanning
        the whole Omega axis (shard 0.28 ms), but long walks are dispatched last at N = 1
        (0.72 ms);
      * ``"balanced"``: V/Omega-major with Omega fastest (0.70 ms at N = 1).
    (profiles/r04/c5_order/: per-wave start/end clocks of the three orders.)  The
    three-atom engine uses these two-atom columns for each atom and each pair."""
    warnings.simplefilter("ignore")
    exc = medium_excitation()
    ref = PH.derive_batch(CF.LPSimulationInputs(excitation=exc), **_apparatus_kwargs(), include_noise=False)
    om0, V0 = ref["Omega"][0], ref["V"][0]
    om = 2 * np.pi * 1e6 * np.linspace(1, 10, n_omega)
    vo = np.logspace(1, 3, n_vo)
    if order not in ("blocked", "balanced", "omega"):
        raise ValueError("order must be 'omega', 'blocked' or 'balanced'")
    if order == "blocked" and n_vo % 8 != 0:
        raise ValueError("order='blocked' needs n_vo divisible by 8 (8 blocks of V/Omega rows)")
    if order == "blocked":
        # [block][Omega][V/Omega within the block]
        VB = vo.reshape(8, n_vo // 8)
        OM = np.broadcast_to(om[None, :, None], (8, n_omega, n_vo // 8))
        VO = np.broadcast_to(VB[:, None, :], (8, n_omega, n_vo // 8))
    else:                                                        # [Omega][V/Omega] | [V/Omega][Omega]
        OM, VO = np.meshgrid(om, vo, indexing="ij" if order == "omega" else "xy")
    OM, VO = OM.ravel(), VO.ravel()
    if point_slice is not None:
        OM, VO = OM[point_slice], VO[point_slice]
    p2 = MEDIUM["laser_2_power"] * (OM / om0) ** 2
    sf = MEDIUM["spacing_factor"] * (V0 / (VO * OM)) ** (1.0 / 6.0)
    return PH.derive_batch(CF.LPSimulationInputs(excitation=exc), n=OM.size,
                           **_apparatus_kwargs(spacing_factor=sf), include_noise=include_noise,
                           overrides=dict(laser_2_power=p2))


def c5_rank_shard(rank: int, world_size: int, include_noise: bool = True, order: str = "omega"):
    """Strong-scaling shard of the fixed 4096-point C5 grid: (batch, global offset of
    its first point) -- the offset keys the trajectories' random streams."""
    sl = range_shard(C5_POINTS, rank, world_size)
    return blockade_grid_3atom(include_noise=include_noise, point_slice=sl, order=order), sl.start


def c5_strided_shard(rank: int, world_size: int, include_noise: bool = True):
    """Strided shard of the Omega-major C5 grid: points rank, rank + N, rank + 2N, ... --
    (batch, offset, stride) for TrajectoryDeviceBatch(point_offset=offset, point_stride=
    stride).  Every rank then spans the whole Omega axis (the ranks' loads even out) while
    each shard keeps the Omega-major order its launch packs best, and the single launch of
    the whole grid stays the Omega-major one."""
    if not 0 <= rank < world_size:
        raise ValueError("rank out of range")
    return (blockade_grid_3atom(include_noise=include_noise, point_slice=slice(rank, C5_POINTS, world_size)),
            rank, world_size)


def range_shard(n: int, rank: int, world_size: int) -> slice:
    """Contiguous range partition: point i -> rank floor(world_size * i / n)."""
    if not 0 <= rank < world_size:
        raise ValueError("rank out of range")
    return slice(n * rank // world_size, n * (rank + 1) // world_size)


def c4_rank_shard(rank: int, world_size: int, include_noise: bool = True) -> PH.DerivedBatch:
    """Strong-scaling shard of the fixed 1M-point C4 grid: rank r owns the contiguous
    range [r N / W, (r+1) N / W) -- no data exchange between ranks."""
    return species_temperature_power_grid(include_noise=include_noise,
                                          point_slice=range_shard(C4_POINTS, rank, world_size))


def c2_rank_shard(rank: int, world_size: int, points_per_rank_delta: int = 100,
                  n_omega: int = 100, include_noise: bool = True) -> PH.DerivedBatch:
    """Weak-scaling shard for multi-GPU runs: the global sweep has
    world_size x 10k points (Delta/Omega grid refined world_size times) and rank r
    owns the contiguous Delta/Omega range [r*100, (r+1)*100) -- no data exchange."""
    if not 0 <= rank < world_size:
        raise ValueError("rank out of range")
    return omega_delta_grid(n_omega, points_per_rank_delta * world_size, include_noise=include_noise,
                            delta_slice=slice(rank * points_per_rank_delta,
                                              (rank + 1) * points_per_rank_delta))


def c3_rank_shard(rank: int, world_size: int, n_omega_per_rank: int = 1000, n_tau: int = 100,
                  include_noise: bool = True) -> PH.DerivedBatch:
    """Weak-scaling shard of the C3 smooth-JP Pareto sweep: world_size x 100k points,
    the Omega axis refined world_size times, rank r owning a contiguous Omega range."""
    if not 0 <= rank < world_size:
        raise ValueError("rank out of range")
    return pareto_tgate_grid(n_omega_per_rank * world_size, n_tau, include_noise=include_noise,
                             omega_slice=slice(rank * n_omega_per_rank, (rank + 1) * n_omega_per_rank))
