# sym16 kernel check: gpu tests on the in-tree lib, then C2/C3 benches for
# the in-tree lib, a variant lib (build_var/), and the old kernels (RYD_SYM16=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-s16}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest rc=$?" > $O/rc.txt
for W in c2 c3 c4; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_${W}.json 2> $O/bench_${W}.err || exit 1
  for V in build_var/*.so; do
    b=$(basename $V .so)
    RYD_ENGINE_LIB=$PWD/$V timeout -k 10 300 python -u bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_${W}_$b.json 2> $O/bench_${W}_$b.err || exit 1
  done
  RYD_SYM16=0 timeout -k 10 300 python -u bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_${W}_old.json 2> $O/bench_${W}_old.err || exit 1
done
echo done
