# Boundary-path check: the host-buffer tests + a full C2 bench line (host_path,
# end_to_end, cpu_baseline).  Usage: gpurun --timeout 900 -- bash tools/gpu_boundary.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-boundary}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_boundary.py -v -s --timeout 120 --timeout-method thread > $O/pytest_boundary.log 2>&1 || { echo "boundary tests failed"; tail -30 $O/pytest_boundary.log; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench failed"; tail -20 $O/bench_c2.err; exit 1; }
echo "done rc=0"
cat $O/bench_c2.json
