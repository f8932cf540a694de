"""Generate the committed golden fixtures (run in the build container only).

    python tests/golden/make_golden.py      # needs /root/reference (read-only)

What it does
1. Imports the reference's eight QuTiP-free modules file-by-file (constants,
   atom_database, laser_physics, noise_models, trap_physics, protocols,
   pulse_shaping, configurations).  QuTiP is absent here (an ordinary missing
   module), so RG/simulation.py itself cannot be imported; the
   call ORDER of simulate_CZ_gate steps 0-8 (RG/simulation.py:2761-3355) is
   restated below, but every formula is the reference's own function.
2. Records the reference-derived physics (Omega, V, tau, xi, shifts, rates) for a
   set of configurations and a random apparatus grid -> physics_golden.json.
3. Evolves the App-B / parity configurations with the expm oracle
   (oracle/lindblad_oracle.py) and records final states + fidelities, together
   with the reference notebooks' PUBLISHED numbers -> evolution_golden.json.
   Noisy states get QuTiP's exact structural zeros (snap_structural_zeros), their
   reference avg_fidelity uses scipy.linalg.eigh (QuTiP 5's eigensolver), and each
   records whether that penalty is a function of rho at 1e-12 (gauge_unstable).

Nothing here is shipped; the GPU box only sees the JSON fixtures.
"""
from __future__ import annotations

import os

for _v in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
    os.environ.setdefault(_v, "1")

import importlib.util
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
REF = "/root/reference/src/qpu_simulator/micro_physics/neutral_atoms/rydberg_gates/"


def load_reference():
    pkg = types.ModuleType("rg")
    pkg.__path__ = [REF]
    sys.modules["rg"] = pkg
    mods = {}
    for name in ["constants", "atom_database", "laser_physics", "noise_models", "trap_physics",
                 "protocols", "pulse_shaping", "configurations"]:
        spec = importlib.util.spec_from_file_location("rg." + name, REF + name + ".py")
        m = importlib.util.module_from_spec(spec)
        sys.modules["rg." + name] = m
        spec.loader.exec_module(m)
        mods[name] = m
    return types.SimpleNamespace(**mods)


APPARATUS = {
    # cz_gate_optimization_demo.ipynb cell 4 (ApparatusConstraints tiers)
    "high": dict(l1p=100e-6, l1w=40e-6, l2p=0.5, l2w=25e-6, T=1e-6, sf=2.8, n=80,
                 Ptw=0.030, wtw=0.8e-6),
    "medium": dict(l1p=50e-6, l1w=50e-6, l2p=0.3, l2w=50e-6, T=2e-6, sf=2.8, n=70,
                   Ptw=0.020, wtw=0.8e-6),
    "low": dict(l1p=20e-6, l1w=60e-6, l2p=0.1, l2w=60e-6, T=5e-6, sf=3.0, n=60,
                Ptw=0.015, wtw=1.0e-6),
}


def ref_derive(R, cfg):
    """simulate_CZ_gate steps 0-8 with the reference's functions (call order of
    RG/simulation.py:2761-3355)."""
    c = R.configurations
    proto = cfg["protocol"]
    lw1, lw2 = cfg.get("lw1", 100.0), cfg.get("lw2", 100.0)
    pur = cfg.get("purity", 1.0)
    L1 = c.LaserParameters(power=cfg["l1p"], waist=cfg["l1w"], polarization="pi",
                           polarization_purity=pur, linewidth_hz=lw1)
    L2 = c.LaserParameters(power=cfg["l2p"], waist=cfg["l2w"], polarization="sigma+",
                           polarization_purity=pur, linewidth_hz=lw2)
    Delta_e = cfg.get("Delta_e", 2 * np.pi * 1e9)
    exc = c.TwoPhotonExcitationConfig(laser_1=L1, laser_2=L2, Delta_e=Delta_e,
                                      counter_propagating=cfg.get("counter", True))
    nz = cfg.get("noise_cfg", {})
    noise = c.NoiseSourceConfig(**nz)
    species, n_ryd = cfg.get("species", "Rb87"), cfg["n"]
    q0, q1 = tuple(cfg.get("qubit_0", (1, 0))), tuple(cfg.get("qubit_1", (2, 0)))
    config = c.AtomicConfiguration(species=species, qubit_0=q0, qubit_1=q1, n_rydberg=n_ryd,
                                   L_rydberg="S")
    atom = R.atom_database.get_atom_properties(species)
    lw = np.sqrt(lw1 ** 2 + lw2 ** 2)
    if cfg.get("wl_nm") is not None:
        trap_wl = cfg["wl_nm"] * 1e-9
    else:
        trap_wl = atom["trap_wavelength"]
    wl_nm = trap_wl * 1e9
    NA = cfg.get("NA", 0.5)
    Rsp = R.trap_physics.tweezer_spacing(trap_wl, NA, cfg["sf"])
    E01 = R.laser_physics.laser_E0(cfg["l1p"], cfg["l1w"])
    E02 = R.laser_physics.laser_E0(cfg["l2p"], cfg["l2w"])
    inter = R.atom_database.get_default_intermediate_state(species)
    d1e = atom["intermediate_states"][inter]["dipole_from_ground"]
    d_er = atom["dipole_intermediate_to_rydberg_ref"] * (n_ryd / atom["n_ref"]) ** (-1.5)
    Om1 = R.laser_physics.single_photon_rabi(d1e, E01)
    Om2 = R.laser_physics.single_photon_rabi(d_er, E02)
    Om = R.laser_physics.two_photon_rabi(Om1, Om2, Delta_e)
    C6 = R.atom_database.get_C6(n_ryd, species)
    V = R.laser_physics.rydberg_blockade(C6, Rsp)
    vo = V / Om
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        pp = R.protocols.get_protocol_params(proto, V_over_Omega=vo)
    out = {}
    if proto == "levine_pichler":
        dom = cfg.get("delta_over_omega") if cfg.get("delta_over_omega") is not None else pp["delta_over_omega"]
        ot = cfg.get("omega_tau") if cfg.get("omega_tau") is not None else pp["omega_tau"]
        tau_s = ot / Om
        tau_t = 2 * tau_s
        Dg = dom * Om
        pulse_shape = cfg.get("pulse_shape", "square")
    elif proto == "jandura_pupillo":
        ot = cfg.get("omega_tau") if cfg.get("omega_tau") is not None else pp.get("omega_tau", 22.08)
        tau_s = ot / Om
        tau_t = tau_s
        Dg = 0.0
        dom = 0.0
        pulse_shape = "bangbang"
        out["switching_times"] = list(cfg.get("switching_times") or pp.get("switching_times"))
        out["phases"] = list(cfg.get("phases") or pp.get("phases"))
    else:
        ot = cfg.get("omega_tau") if cfg.get("omega_tau") is not None else pp.get("omega_tau", 10.09)
        tau_s = ot / Om
        tau_t = tau_s
        Dg = 0.0
        dom = cfg.get("delta_over_omega") if cfg.get("delta_over_omega") is not None else pp.get("delta_over_omega", 0.0205)
        pulse_shape = "smooth_sinusoidal"
    tn = R.trap_physics.compute_trap_dependent_noise(
        species=species, tweezer_power=cfg["Ptw"], tweezer_waist=cfg["wtw"],
        temperature=cfg["T"], spacing=Rsp, gate_time=tau_t, n_rydberg=n_ryd,
        gamma_phi_laser=np.pi * lw, Omega_1=Om1, Delta_e=Delta_e,
        intermediate_state=config.intermediate_state, Omega_eff=Om,
        tweezer_wavelength_nm=wl_nm, include_doppler=noise.include_doppler_dephasing,
        include_intensity_noise=noise.include_intensity_noise,
        intensity_noise_frac=noise.intensity_noise_frac,
        rydberg_wavelength_1_nm=config.excitation_wavelength_1_nm,
        rydberg_wavelength_2_nm=config.excitation_wavelength_2_nm,
        counter_propagating=exc.counter_propagating)
    B = cfg.get("B", 1e-4)
    dz = R.trap_physics.calculate_zeeman_shift(B_field=B, qubit_0=q0, qubit_1=q1, species=species)
    trap_on = cfg.get("trap_on", True)
    if trap_on:
        tdm = tn.get("trap_depth_uK", 0) / 1000
        ds = R.trap_physics.calculate_qubit_stark_shift(
            tweezer_power=cfg["Ptw"], tweezer_waist=cfg["wtw"], species=species,
            trap_depth_mK=tdm if tdm > 0 else None)
    else:
        ds = 0.0
    xi = complex(R.protocols.compute_phase_shift_xi(Dg, Om, tau_s)) if proto == "levine_pichler" else 1.0 + 0j
    rates = {k: 0.0 for k in ("gamma_r", "gamma_bbr", "gamma_phi_laser", "gamma_phi_thermal",
                              "gamma_phi_zeeman", "gamma_loss_antitrap", "gamma_loss_background",
                              "gamma_scatter_intermediate", "gamma_leakage", "mJ_leakage_rate")}
    if cfg.get("include_noise", True):
        gmot = tn["gamma_phi_thermal"] if noise.include_motional_dephasing else 0.0
        B_rms = max(0.01 * B * 1e4, 1e-3)
        qt = "clock" if config.is_clock_transition else "stretched"
        Kq = 575.0 if species == "Rb87" else 427.0
        tf = min(1.0, (tau_t / 1e-6) ** 2)
        Dleak = R.pulse_shaping.compute_leakage_detuning(species, n_ryd)
        rates.update(
            gamma_r=tn["gamma_r"], gamma_bbr=tn.get("gamma_bbr", 0),
            gamma_phi_laser=np.pi * lw,
            gamma_phi_thermal=gmot + tn.get("gamma_phi_doppler", 0.0) + tn.get("gamma_phi_intensity", 0.0),
            gamma_phi_zeeman=R.noise_models.zeeman_dephasing_rate(B_rms, qt, Kq),
            gamma_loss_antitrap=tn["gamma_loss_antitrap"] * 0.3 * tf,
            gamma_loss_background=cfg.get("bg") if cfg.get("bg") is not None else tn["gamma_loss_background"],
            gamma_scatter_intermediate=tn["gamma_scatter_intermediate"],
            gamma_leakage=R.noise_models.leakage_rate_to_adjacent_states(
                Omega=Om, Delta_leak=Dleak, pulse_shape=pulse_shape, tau=tau_s,
                gamma_rydberg=tn["gamma_r"]),
        )
        if cfg.get("dim", 3) == 4:
            dZ = R.noise_models.rydberg_zeeman_splitting(B, L=0, J=0.5)
            rates["mJ_leakage_rate"] = R.noise_models.mJ_mixing_rate(Om, min(pur, pur), dZ)
    out.update(Omega=Om, Omega1=Om1, V=V, R=Rsp, V_over_Omega=vo, tau_single=tau_s, tau_total=tau_t,
               Delta_gate=Dg, delta_over_omega=dom, omega_tau=ot, delta_zeeman=dz,
               delta_stark=ds, xi_re=xi.real, xi_im=xi.imag,
               U0_mK=tn["trap_depth_uK"] / 1000, omega_r_kHz=tn["trap_freq_radial_kHz"],
               sigma_r_nm=tn["position_uncertainty_nm"], alpha_ratio=tn["alpha_ratio"],
               magic_enhancement=tn["magic_enhancement"], differential_shift_Hz=tn["differential_shift_Hz"],
               gamma_phi_doppler=tn["gamma_phi_doppler"], gamma_phi_intensity=tn["gamma_phi_intensity"],
               gamma_phi_thermal_motional=tn["gamma_phi_thermal"], **rates)
    if proto == "smooth_jp":
        sp = R.protocols.get_protocol_params("smooth_jp", V_over_Omega=vo)
        A = cfg.get("A") or sp.get("A", 0.311 * np.pi)
        omr = cfg.get("omega_mod_ratio") or sp.get("omega_mod_ratio", 1.242)
        phoff = cfg.get("phi_offset") or sp.get("phi_offset", 4.696)
        raw = cfg.get("delta_over_omega")
        mag = abs(raw if raw is not None else sp.get("delta_over_omega", 0.0205))
        sot = cfg.get("omega_tau") if cfg.get("omega_tau") is not None else sp.get("omega_tau", 10.09)
        out.update(A=A, omega_mod=omr * Om, phi_offset=phoff,
                   smooth_delta_over_omega=(-mag if Delta_e > 0 else mag),
                   tau_total=sot / Om)
    if cfg.get("pulse_shape", "square") not in ("square",) and proto == "levine_pichler":
        out["area_correction"] = R.pulse_shaping.area_correction_factor(cfg["pulse_shape"], tau_s)
    return out


def nf_noise():
    return dict(include_spontaneous_emission=False, include_intermediate_scattering=False,
                include_motional_dephasing=False, include_doppler_dephasing=False,
                include_intensity_noise=False, intensity_noise_frac=0.0,
                include_laser_dephasing=False, include_magnetic_dephasing=False)


def configs():
    C = []
    med = APPARATUS["medium"]
    for tier in ("high", "medium", "low"):
        a = APPARATUS[tier]
        C.append(dict(name=f"lp_{tier}_nf", protocol="levine_pichler", include_noise=False,
                      noise_cfg=nf_noise(), **a))
        C.append(dict(name=f"smooth_{tier}_nf", protocol="smooth_jp", include_noise=False,
                      noise_cfg=nf_noise(), **a))
    full = dict(purity=0.99)
    C.append(dict(name="lp_medium_noisy", protocol="levine_pichler", include_noise=True, **full, **med))
    C.append(dict(name="smooth_medium_noisy", protocol="smooth_jp", include_noise=True, **full, **med))
    C.append(dict(name="bangbang_medium_noisy", protocol="jandura_pupillo", include_noise=True, **full, **med))
    C.append(dict(name="bangbang_medium_nf", protocol="jandura_pupillo", include_noise=False,
                  noise_cfg=nf_noise(), **med))
    C.append(dict(name="lp_cosine_noisy", protocol="levine_pichler", include_noise=True,
                  pulse_shape="cosine", **full, **med))
    C.append(dict(name="lp_gaussian_nf", protocol="levine_pichler", include_noise=False,
                  pulse_shape="gaussian", noise_cfg=nf_noise(), **med))
    C.append(dict(name="lp_cs133_noisy", protocol="levine_pichler", include_noise=True, species="Cs133",
                  **full, **{**med, "n": 60}))
    C.append(dict(name="lp_nonclock_trapoff_noisy", protocol="levine_pichler", include_noise=True,
                  qubit_1=(2, 1), trap_on=False, **full, **med))
    C.append(dict(name="lp_850nm_hot_noisy", protocol="levine_pichler", include_noise=True, wl_nm=850.0,
                  **full, **{**med, "T": 20e-6}))
    C.append(dict(name="smooth_override_noisy", protocol="smooth_jp", include_noise=True, A=0.0,
                  omega_mod_ratio=1.3, phi_offset=0.0, delta_over_omega=0.03, omega_tau=9.5,
                  **full, **med))
    C.append(dict(name="lp_override_noisy", protocol="levine_pichler", include_noise=True,
                  delta_over_omega=0.36, omega_tau=4.4, lw1=1000.0, lw2=1000.0, **full, **med))
    return C


def point_spec(R, cfg, d, with_cops=True):
    from oracle import lindblad_oracle as O
    proto = cfg["protocol"]
    kw = dict(Omega=d["Omega"], V=d["V"], delta_zeeman=d["delta_zeeman"],
              delta_stark=d["delta_stark"], trap_laser_on=cfg.get("trap_on", True), dim=cfg.get("dim", 3))
    cops = O.collapse_operators(d, dim=cfg.get("dim", 3)) if cfg.get("include_noise", True) else []
    if proto == "levine_pichler":
        shape = cfg.get("pulse_shape", "square")
        if shape == "square":
            return O.PointSpec(protocol="lp_square", Delta=d["Delta_gate"], tau=d["tau_single"],
                               xi=complex(d["xi_re"], d["xi_im"]), c_ops=cops, **kw)
        return O.PointSpec(protocol="lp_shaped", Delta=d["Delta_gate"], tau=d["tau_single"],
                           xi=complex(d["xi_re"], d["xi_im"]), pulse_shape=shape,
                           area_correction=d["area_correction"], c_ops=cops, **kw)
    if proto == "jandura_pupillo":
        return O.PointSpec(protocol="bangbang", omega_tau=d["omega_tau"],
                           switching_times=d["switching_times"], phases=d["phases"], c_ops=cops, **kw)
    return O.PointSpec(protocol="smooth_jp", Delta=d["smooth_delta_over_omega"] * d["Omega"],
                       tau=d["tau_total"], A=d["A"], omega_mod=d["omega_mod"],
                       phi_offset=d["phi_offset"], n_steps=300, c_ops=cops, **kw)


PUBLISHED = {
    # cz_gate_optimization_demo.ipynb:268-272 (LP, medium) and :314-317 (smooth JP, medium)
    "lp_medium_nf": dict(avg=(0.994423, 6), F11=(0.977897, 6), cz_phase_fidelity=(0.978587, 6),
                         phase_error_deg=(16.83, 2), controlled_phase_deg=(163.17, 2),
                         gate_time_us=(0.379, 3), V_over_Omega=(342.5, 1), Omega_MHz=(3.602, 3)),
    "smooth_medium_nf": dict(avg=(0.992310, 6), F11=(0.969240, 6), cz_phase_fidelity=(0.969287, 6),
                             phase_error_deg=(20.19, 2), controlled_phase_deg=(159.81, 2),
                             gate_time_us=(0.446, 3)),
    # cz_gate_optimization_demo.ipynb:374-376 (tier comparison)
    "lp_high_nf": dict(avg=(0.9991, 4)), "lp_low_nf": dict(avg=(0.9887, 4)),
    "smooth_high_nf": dict(avg=(0.9982, 4)), "smooth_low_nf": dict(avg=(0.9845, 4)),
}


def random_grid(R, n=40, seed=20260215):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        proto = ["levine_pichler", "smooth_jp", "jandura_pupillo"][i % 3]
        cfg = dict(name=f"grid{i}", protocol=proto, include_noise=True,
                   species=["Rb87", "Cs133"][int(rng.integers(2))],
                   n=int(rng.integers(50, 100)), l1p=float(10 ** rng.uniform(-5.3, -3.7)),
                   l1w=float(rng.uniform(20e-6, 80e-6)), l2p=float(10 ** rng.uniform(-1.5, 0.3)),
                   l2w=float(rng.uniform(20e-6, 80e-6)), T=float(10 ** rng.uniform(-6.5, -4.5)),
                   sf=float(rng.uniform(2.0, 5.0)), Ptw=float(10 ** rng.uniform(-3, -1)),
                   wtw=float(rng.uniform(0.6e-6, 1.5e-6)), B=float(10 ** rng.uniform(-5, -3)),
                   NA=float(rng.uniform(0.4, 0.7)), Delta_e=float(2 * np.pi * 10 ** rng.uniform(8.5, 10)),
                   purity=float(rng.uniform(0.95, 1.0)), lw1=float(rng.uniform(10, 2000)),
                   lw2=float(rng.uniform(10, 2000)), dim=[3, 4][int(rng.integers(2))],
                   counter=bool(rng.integers(2)),
                   noise_cfg=dict(include_motional_dephasing=bool(rng.integers(2)),
                                  include_doppler_dephasing=bool(rng.integers(2)),
                                  include_intensity_noise=bool(rng.integers(2)),
                                  intensity_noise_frac=float(rng.uniform(0, 0.05))))
        if i % 5 == 0:
            cfg["wl_nm"] = float(rng.uniform(780, 1100))
        if i % 7 == 0:
            cfg["qubit_1"] = (2, 1)
        if i % 4 == 0:
            cfg["trap_on"] = False
        out.append(cfg)
    return out


def _jsonable(x):
    if isinstance(x, dict):
        return {k: _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    if isinstance(x, (np.floating, float)):
        return float(x)
    if isinstance(x, (np.integer, int)):
        return int(x)
    if isinstance(x, np.bool_):
        return bool(x)
    return x


def main():
    import warnings
    warnings.simplefilter("ignore")
    R = load_reference()
    sys.path.insert(0, REPO)
    from oracle import lindblad_oracle as O
    phys = []
    for cfg in configs() + random_grid(R):
        d = ref_derive(R, cfg)
        phys.append(dict(config=cfg, derived=d))
    with open(os.path.join(HERE, "physics_golden.json"), "w") as f:
        json.dump(_jsonable(phys), f, indent=1)
    evo = []
    for cfg in configs():
        d = ref_derive(R, cfg)
        p = point_spec(R, cfg, d)
        res = O.run_point(p, method="expm")
        unstable, spread = False, 0.0
        if cfg.get("include_noise", True):
            # QuTiP keeps the structural zeros exact; the reference's eigensolver is
            # scipy.linalg.eigh (QuTiP 5 Qobj.eigenstates)
            res = {k: O.snap_structural_zeros(v, cfg.get("dim", 3)) for k, v in res.items()}
            unstable, spread = O.gauge_unstable(res, cfg.get("dim", 3), scheme="all_at_once")
        import scipy.linalg as sla
        fid, avg, info = O.cz_fidelity(res, eigh=lambda m: sla.eigh(m))
        states = {k: (np.stack([v.real, v.imag]).tolist()) for k, v in res.items()}
        evo.append(dict(name=cfg["name"], config=cfg, derived=d, states=states, fidelities=fid,
                        avg_fidelity=avg, phase_info={k: v for k, v in info.items()},
                        gauge_unstable=bool(unstable), gauge_spread=float(spread),
                        published=PUBLISHED.get(cfg["name"], {})))
        print(f"{cfg['name']:28s} avg={avg:.8f} F11={fid['11']:.8f} "
              f"pen={info['cz_phase_fidelity']:.6f} perr={info['phase_error_from_pi_deg']:.2f} "
              f"gauge_unstable={unstable} spread={spread:.3g}")
    # App B row 5 (examples/neutral_atoms_rydberg_cz_gate.ipynb:10294-10299): notebook-local
    # two-pulse LP, kets, no light shifts, Omega = 2 pi 1 MHz, V/Omega = 100
    Om = 2 * np.pi * 1e6
    tau = 4.29268 / Om
    Dl = 0.377371 * Om
    xi = complex(R.protocols.compute_phase_shift_xi(Dl, Om, tau))
    p = O.PointSpec(protocol="lp_square", Omega=Om, V=100 * Om, Delta=Dl, tau=tau, xi=xi)
    res = O.run_point(p, method="expm")
    pops = {k: float(abs(v[O.initial_kets()[k].argmax()]) ** 2) for k, v in res.items()}
    evo.append(dict(name="lp_row5_physics", config=dict(protocol="levine_pichler", physics_only=True),
                    derived=dict(Omega=Om, V=100 * Om, Delta_gate=Dl, tau_single=tau, xi_re=xi.real,
                                 xi_im=xi.imag, delta_zeeman=0.0, delta_stark=0.0),
                    states={k: np.stack([v.real, v.imag]).tolist() for k, v in res.items()},
                    populations=pops,
                    published=dict(F00=(1.0, 8), F01=(1.0, 8), F10=(1.0, 8), F11=(0.99999617, 8),
                                   avg_no_penalty=(0.99999904, 8), phi_01_deg=(136.41, 2),
                                   phase_error_deg=(1.1529, 4))))
    print("row5 pops", pops, np.mean(list(pops.values())))
    with open(os.path.join(HERE, "evolution_golden.json"), "w") as f:
        json.dump(_jsonable(evo), f)


if __name__ == "__main__":
    main()
