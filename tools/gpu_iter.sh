# Iteration check: GPU tests, benches (C2/C3/C4), C2 HBM traffic passes.
# Usage: gpurun --timeout 900 -- bash tools/gpu_iter.sh TAG [notest]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-iter}
mkdir -p $O
if [ "$2" != "notest" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
fi
for W in c2 c3 c4; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_${W}.json 2> $O/bench_${W}.err || exit 1
done
for V in build_var/*.so; do
  [ -e "$V" ] || continue
  b=$(basename $V .so)
  for W in c2 c3; do
    RYD_ENGINE_LIB=$PWD/$V timeout -k 10 300 python -u bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_${W}_$b.json 2> $O/bench_${W}_$b.err || exit 1
  done
done
# the in-tree lib again (box clock drift between the first and the variant runs)
timeout -k 10 300 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c2_again.json 2> $O/bench_c2_again.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c2 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch_c2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c2 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/write_c2.log 2>&1
echo "done rc=$?"
