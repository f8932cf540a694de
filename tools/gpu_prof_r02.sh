# Round-2 profile set for the sym16 kernel: rocprofv3 kernel stats, one SQ issue/stall
# pass (incl. LDS waits) and the FETCH_SIZE / WRITE_SIZE HBM passes, for C2, C3, C4.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_prof_r02.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-prof_r02}
mkdir -p $O
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS"
for W in ${2:-c2 c3 c4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$W -o run -- python bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline > $O/stats_$W.json 2> $O/stats_$W.err || { echo "stats $W failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/sq_$W -o run -- python bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline > $O/sq_$W.log 2>&1 || { echo "sq $W failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$W -o run -- python bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch_$W.log 2>&1 || { echo "fetch $W failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$W -o run -- python bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline > $O/write_$W.log 2>&1 || { echo "write $W failed"; exit 1; }
  echo "$W ok"
done
echo done
