#!/bin/bash
# Exact-jump-time C5 kernel as the default: whole GPU suite, smoke, the C5 line (with the
# CPU baseline), rocprofv3 kernel stats, one SQ pass and the HBM FETCH/WRITE passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$PWD PYTHONUNBUFFERED=1
O=gpurun_out/${1:-c5exact}
mkdir -p $O
[ "$2" = skiptests ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_c5 -o run -- python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/stats_c5.json 2> $O/stats_c5.err || { echo "stats failed"; exit 1; }
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS"
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/sq_c5 -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/sq_c5.log 2>&1 || { echo "sq failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c5 -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch_c5.log 2>&1 || { echo "fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c5 -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/write_c5.log 2>&1 || { echo "write failed"; exit 1; }
RYD_ENGINE_LIB=$PWD/build/libryd_tprof.so timeout -k 10 200 python -u tools/traj_prof.py > $O/phase.log 2>&1 || exit 1
cat $O/phase.log
for f in $O/bench_c5.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', d['value'], r['kernel_ms'], r['frac'], r['exec_over_useful'], d.get('cpu_baseline', {}).get('value'))"; done
