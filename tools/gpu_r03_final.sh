# Round-3 closing check: the whole GPU suite, smoke, and the driver's bench command.
# Usage: gpurun --timeout 900 -- bash tools/gpu_r03_final.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD
O=gpurun_out/${1:-final}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || exit 1
python -c "import json;d=json.load(open('$O/bench_driver_cmd.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'], d['pipelined']['points_per_s'])"
