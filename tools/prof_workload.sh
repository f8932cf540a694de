#!/bin/bash
# Profile one bench.py workload on the GPU box: rocprofv3 kernel statistics of the bench
# line itself, then three PMC passes of their own (FETCH_SIZE, WRITE_SIZE, the SQ issue /
# wait counters -- at most 8 SQ counters in one pass), each under its own time limit.
#   tools/prof_workload.sh OUTDIR WORKLOAD [extra bench.py args]
# Writes OUTDIR/bench.json, OUTDIR/trace (kernel trace + stats), OUTDIR/{fetch,write,sq}.
# Fold the passes with tools/pmc_traffic.py and tools/pmc_summary.py afterwards.
set -euo pipefail
out=$(realpath -m "$1")
wl=$2
shift 2
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$out"
cd /tmp
export TMPDIR=/tmp
bench=("$root/bench.py" --workload "$wl" --no-cpu-baseline "$@")
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 "${bench[@]}" --steps 20 --warmup 3 > "$out/bench.json" 2> "$out/trace.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
  python3 "${bench[@]}" --steps 5 --warmup 1 > /dev/null 2> "$out/fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
  python3 "${bench[@]}" --steps 5 --warmup 1 > /dev/null 2> "$out/write.err"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
  SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS --output-format csv -d "$out/sq" -o run -- \
  python3 "${bench[@]}" --steps 5 --warmup 1 > /dev/null 2> "$out/sq.err"
echo "profiled $wl into $out"
