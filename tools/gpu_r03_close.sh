#!/bin/bash
# Round-3 closing check on the final tree: the whole GPU suite, smoke, the driver's bench
# command, and the C5 line with its rocprofv3 kernel statistics.
# Usage: gpurun --timeout 1100 -- bash tools/gpu_r03_close.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$PWD PYTHONUNBUFFERED=1
O=gpurun_out/${1:-close}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || exit 1
python -c "import json;d=json.load(open('$O/bench_driver_cmd.json'));print('C2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'], d['pipelined']['points_per_s'])"
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_c5 -o run -- python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/stats_c5.json 2> $O/stats_c5.err || { echo "stats failed"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c5.json'));r=d['roofline'];print('C5', d['value'], r['kernel_ms'], r['frac'], r['traffic'], d['cpu_baseline']['value'])"
