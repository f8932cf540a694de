"""Summarise a rocprofv3 --pmc directory: per-dispatch mean of every counter for the
kernels whose name contains --kernel, plus the SQ issue/stall fractions.

    python tools/pmc_summary.py DIR --kernel lindblad_sym16_kernel
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os


def collect(directory: str, kernel: str):
    files = glob.glob(os.path.join(directory, "**", "*counter_collection.csv"), recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                if kernel in r["Kernel_Name"]:
                    acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {c: sum(d.values()) / len(d) for c, d in acc.items() if d}, \
        max((len(d) for d in acc.values()), default=0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("directory")
    ap.add_argument("--kernel", required=True)
    a = ap.parse_args()
    m, nd = collect(a.directory, a.kernel)
    out = {"kernel": a.kernel, "dispatches": nd, "per_dispatch_mean": m}
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in m:
                out[k.lower().replace("sq_", "") + "_frac"] = m[k] / wc
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
