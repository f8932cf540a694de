# Round-3 final profile set: the driver's bench command, rocprofv3 kernel statistics of
# C2-C5, one SQ issue/stall pass each for C2 and C5, and the HBM FETCH/WRITE passes of C5.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_prof_r03.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$PWD
O=gpurun_out/${1:-prof_r03}
mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || { echo "driver bench failed"; exit 1; }
echo "driver bench ok"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS"
for W in c2 c3 c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$W -o run -- python bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline > $O/stats_$W.json 2> $O/stats_$W.err || { echo "stats $W failed"; exit 1; }
  echo "stats $W ok"
done
for W in c2 c5; do
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/sq_$W -o run -- python bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline > $O/sq_$W.log 2>&1 || { echo "sq $W failed"; exit 1; }
  echo "sq $W ok"
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c5 -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch_c5.log 2>&1 || { echo "fetch c5 failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c5 -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/write_c5.log 2>&1 || { echo "write c5 failed"; exit 1; }
echo done
