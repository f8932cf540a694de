set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
nproc > gpurun_out/nproc.txt
rocminfo 2>/dev/null | grep -E "Marketing Name|gfx" | head -4 > gpurun_out/rocminfo.txt || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rocprof.log 2>&1
echo "exit=$?"
