# bench + profile first (independent of test status), then debug + gpu tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --method cheb_vector --no-cpu-baseline > gpurun_out/bench_vector.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rocprof.log 2>&1 && \
timeout -k 10 300 python tools/dbg_dopri.py > gpurun_out/dbg_dopri.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
echo "exit=$?"
