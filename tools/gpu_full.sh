# Full GPU test suite + the default bench line (C2, with cpu_baseline and end_to_end).
# Usage: gpurun --timeout 1200 -- bash tools/gpu_full.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-full}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench failed"; tail -20 $O/bench_c2.err; exit 1; }
echo "done rc=0"
cat $O/bench_c2.json
