# sym16 iteration on one MI355X: phase timeline (RYD_S16_PROF variant in build/), the GPU
# suite, and C2/C3/C4 bench lines.  Usage: gpurun --timeout 900 -- bash tools/gpu_s16iter.sh TAG [tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-s16iter}
T=${2:-tests}
mkdir -p $O
if [ -f build/libryd_prof.so ]; then
  RYD_ENGINE_LIB=$PWD/build/libryd_prof.so timeout -k 10 200 python -u tools/phase_prof.py c2 4096 10000 > $O/phase_c2.log 2>&1 && RYD_ENGINE_LIB=$PWD/build/libryd_prof.so timeout -k 10 200 python -u tools/phase_prof.py c3 4096 > $O/phase_c3.log 2>&1 || { echo "phase failed"; tail -20 $O/phase_c*.log; exit 1; }
fi
timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for W in c2 c3 c4; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_$W.json 2> $O/bench_$W.err || { echo "bench $W failed"; tail -20 $O/bench_$W.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/bench_$W.json')); r=d['roofline']; print('$W', '%.3e'%d['value'], 'kernel_ms', round(r['kernel_ms'],4), 'frac', round(r['frac'],4))"
done
cat $O/phase_c2.log $O/phase_c3.log 2>/dev/null
echo done
