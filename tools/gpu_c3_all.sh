# All GPU tests + C3 and C2 bench lines (kernel changes touching the smooth-JP path)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-c3all}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
echo "exit=$?"
