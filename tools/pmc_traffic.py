"""Fold two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) into profiles/pmc_traffic.json.

    python tools/pmc_traffic.py --fetch DIR --write DIR --workload c2 --method chebyshev \
        --n 10000 --kernel lindblad_prop_kernel [--out profiles/pmc_traffic.json]

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide reads, so
it is doubled; WRITE_SIZE is taken as is.  The per-launch figure is the mean over the
profiled dispatches of the named kernel.  bench.py reads the file for roofline.traffic.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os


def per_dispatch(directory: str, counter: str, kernel: str) -> list:
    files = glob.glob(os.path.join(directory, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {directory}")
    acc = collections.defaultdict(float)
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
                    acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
    if not acc:
        raise SystemExit(f"{counter} for {kernel} not found in {directory}")
    return list(acc.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--workload", required=True)
    ap.add_argument("--method", required=True)
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    fk = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    wk = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    fetch = 2.0 * 1024 * sum(fk) / len(fk)
    write = 1024 * sum(wk) / len(wk)
    row = {"workload": a.workload, "method": a.method, "n": a.n, "kernel": a.kernel,
           "fetch_size_kib_raw": sum(fk) / len(fk), "write_size_kib": sum(wk) / len(wk),
           "fetch_bytes": fetch, "write_bytes": write, "bytes_per_launch": fetch + write,
           "dispatches": [len(fk), len(wk)],
           "correction": "FETCH_SIZE x2 (gfx950), KiB -> B; MI355X_MICROARCH.md HBM section"}
    rows = []
    if os.path.exists(a.out):
        with open(a.out) as f:
            rows = [r for r in json.load(f)
                    if (r["workload"], r["method"], r["n"], r["kernel"]) != (a.workload, a.method, a.n, a.kernel)]
    rows.append(row)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)
    print(json.dumps(row))


if __name__ == "__main__":
    main()
