# Whole GPU suite + smoke + the C2 metric line and the C5 line (quick health check of a tree).
# Usage: gpurun --timeout 900 -- bash tools/gpu_r03_check.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD
TAG=${1:-chk}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
for f in $O/bench_*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', d['value'], r['kernel_ms'], r['frac'], r.get('exec_over_useful'))"; done
