# C3 4-op parity tests + C3 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-c3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py -x -v --timeout 240 --timeout-method thread > $O/pytest_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 1 > $O/bench_c3.json 2> $O/bench_c3.err
echo "exit=$?"
