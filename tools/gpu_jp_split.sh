# Smooth-JP split path: all GPU tests, then C3 bench lines (split occ 4 / occ 3 / fused)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-jpsplit}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err && \
RYD_JP_SPLIT=0 true && \
RYD_JP_SPLIT=0 timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c3_fused.json 2> $O/bench_c3_fused.err
echo "exit=$?"
