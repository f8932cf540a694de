# rocprofv3 kernel stats + PMC (SQ issue/stall, HBM traffic) for the sym16 kernel on C2/C3/C4.
# Usage: gpurun --timeout 900 -- bash tools/gpu_prof_s16.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-prof_s16}
mkdir -p $O
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
for W in c2 c3 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$W -o run -- python bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline > $O/stats_$W.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/sq_$W -o run -- python bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline > $O/sq_$W.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$W -o run -- python bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch_$W.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$W -o run -- python bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline > $O/write_$W.log 2>&1 || exit 1
done
echo done
