"""Calibration-data writer for the Rydberg CZ gate.

The reference describes, but does not ship, per-platform calibration files fed
by micro-physics runs (calibration_data/README.md:1-27): JSON under
``neutral_atoms/rydberg_cz/n<N>_*.json`` holding the parameter values used, the
resulting error rates, gate durations and metadata.  ``calibrate_cz`` produces
them from ONE batched engine pass (plus the process-map pass when requested):

    root/neutral_atoms/rydberg_cz/n70_Rb87_levine_pichler.json

one file per (species, n_rydberg, protocol), one record per sweep point:
``parameters`` (apparatus + protocol), ``error_rates`` (average infidelity,
per-basis-state infidelities, controlled-phase error, and -- with the process
map -- process / average gate fidelity to CZ up to local Z phases, leakage and
the twirled two-qubit Pauli error probabilities), ``durations`` and ``status``.
The layout is this package's own (schema ``SCHEMA``); the reference fixes only
the directory convention and the four content groups.
"""
from __future__ import annotations

import datetime
import json
import os
from typing import Any, Dict, List, Optional

import numpy as np

SCHEMA = "noisyquantumsimulator_amd.calibration.rydberg_cz/1"
APPARATUS_KEYS = ("tweezer_power", "tweezer_waist", "temperature", "B_field", "NA", "spacing_factor")


def _f(x) -> Any:
    x = np.asarray(x)
    return float(x) if np.isfinite(x) else None


def records(br, apparatus: Dict[str, np.ndarray], maps=None) -> List[Dict[str, Any]]:
    """One calibration record per point of a simulation.BatchResult (optionally with
    noise_models.ProcessMaps of the same points)."""
    from .noise_models import PAULI_LABELS
    b = br.batch
    c = b.cols
    cp = br.controlled_phase
    err = np.degrees(np.minimum(np.abs(cp - np.pi), np.abs(cp + np.pi)))
    out = []
    for i in range(b.n):
        params = {k: _f(np.broadcast_to(apparatus[k], (b.n,))[i]) for k in APPARATUS_KEYS if k in apparatus}
        params.update(Omega_rad_s=_f(c["Omega"][i]), V_rad_s=_f(c["V"][i]), V_over_Omega=_f(c["V_over_Omega"][i]),
                      R_m=_f(c["R"][i]), Delta_rad_s=_f(c["Delta_gate"][i]),
                      delta_over_omega=_f(c["delta_over_omega"][i]), omega_tau=_f(c["omega_tau"][i]),
                      delta_zeeman_rad_s=_f(c["delta_zeeman"][i]), delta_stark_rad_s=_f(c["delta_stark"][i]))
        if b.protocol == "smooth_jp":
            params.update(A=_f(c["A"][i]), omega_mod_rad_s=_f(c["omega_mod"][i]), phi_offset=_f(c["phi_offset"][i]))
        if b.protocol == "jandura_pupillo":
            params.update(switching_times=[float(t) for t in b.bangbang_times[i]],
                          phases=[float(p) for p in b.bangbang_phases[i]])
        rates = {k: _f(c[k][i]) for k in ("gamma_r", "gamma_phi_laser", "gamma_phi_thermal", "gamma_phi_zeeman",
                                          "gamma_loss_antitrap", "gamma_loss_background",
                                          "gamma_scatter_intermediate", "gamma_leakage")}
        er = {"avg_infidelity": _f(1 - br.avg_fidelity[i]),
              "basis_infidelity": {lab: _f(1 - br.fidelities[i, k]) for k, lab in enumerate(("00", "01", "10", "11"))},
              "controlled_phase_deg": _f(np.degrees(cp[i])), "phase_error_deg": _f(err[i]),
              "noise_rates_per_s": rates}
        if maps is not None:
            er.update(process_infidelity=_f(1 - maps.process_fidelity[i]),
                      avg_gate_infidelity=_f(1 - maps.avg_gate_fidelity[i]), leakage=_f(maps.leakage[i]),
                      local_z_phases_rad=[_f(maps.alpha[i]), _f(maps.beta[i])],
                      pauli_error_probs={lab: _f(maps.pauli_probs[i, k])
                                         for k, lab in enumerate(PAULI_LABELS) if lab != "II"})
        out.append({"parameters": params, "error_rates": er,
                    "durations": {"gate_time_us": _f(c["tau_total"][i] * 1e6),
                                  "tau_single_us": _f(c["tau_single"][i] * 1e6)},
                    "status": int(br.status[i])})
    return out


def calibration_path(root: str, species: str, n_rydberg: int, protocol: str) -> str:
    return os.path.join(root, "neutral_atoms", "rydberg_cz", f"n{int(n_rydberg)}_{species}_{protocol}.json")


def write_calibration(path: str, recs: List[Dict[str, Any]], species: str, n_rydberg: int, protocol: str,
                      metadata: Optional[Dict[str, Any]] = None) -> str:
    meta = {"created_utc": datetime.datetime.now(datetime.timezone.utc).isoformat(timespec="seconds"),
            "n_points": len(recs)}
    meta.update(metadata or {})
    doc = {"schema": SCHEMA, "platform": "neutral_atoms", "gate": "rydberg_cz", "species": species,
           "n_rydberg": int(n_rydberg), "protocol": protocol, "metadata": meta, "points": recs}
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(doc, f, indent=1)
    os.replace(tmp, path)
    return path


def load_calibration(path: str) -> Dict[str, Any]:
    with open(path) as f:
        doc = json.load(f)
    if doc.get("schema") != SCHEMA:
        raise ValueError(f"{path}: not a {SCHEMA} file")
    return doc


def calibrate_cz(simulation_inputs, root: str, *, species="Rb87", n_rydberg=70, include_noise: bool = True,
                 with_process_map: bool = True, devices=None, **apparatus) -> List[str]:
    """Run a (batched) CZ sweep and write its calibration files; returns the paths.
    ``species`` / ``n_rydberg`` / apparatus arguments may be arrays (one file per
    (species, n) group)."""
    from . import engine as E
    from . import noise_models as NM
    from .simulation import simulate_CZ_gate_batch
    br = simulate_CZ_gate_batch(simulation_inputs, species=species, n_rydberg=n_rydberg,
                                include_noise=include_noise, devices=devices, **apparatus)
    n = br.n
    maps = None
    if with_process_map:
        b = br.batch
        key = E.protocol_key(b)
        shape = b.pulse_shape.lower() if key == "lp_shaped" else "square"
        maps = NM.gate_process_maps(E.pack_params(b), key, shape=shape,
                                    engine=E.Engine(list(devices)) if devices else None)
    full_app = {k: np.broadcast_to(np.asarray(apparatus.get(k, d), dtype=float), (n,))
                for k, d in zip(APPARATUS_KEYS, (30e-3, 1.0e-6, 2e-6, 1e-4, 0.5, 2.8))}
    recs = records(br, full_app, maps)
    sp = np.broadcast_to(np.asarray(species), (n,))
    nr = np.broadcast_to(np.asarray(n_rydberg), (n,)).astype(int)
    from . import _native as N
    meta = {"engine": "libryd_engine (HIP, gfx950)", "abi_version": N.RYD_ABI_VERSION,
            "include_noise": include_noise, "process_map": bool(with_process_map),
            "source": "noisyquantumsimulator_amd.calibration.calibrate_cz"}
    paths = []
    for s in np.unique(sp):
        for nn in np.unique(nr[sp == s]):
            idx = np.nonzero((sp == s) & (nr == nn))[0]
            path = calibration_path(root, str(s), int(nn), br.batch.protocol)
            paths.append(write_calibration(path, [recs[i] for i in idx], str(s), int(nn), br.batch.protocol,
                                           dict(meta, point_index=[int(i) for i in idx])))
    return paths


__all__ = ["SCHEMA", "records", "calibration_path", "write_calibration", "load_calibration", "calibrate_cz"]
