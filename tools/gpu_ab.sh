# A/B of build variants (build_var/*.so) against the in-tree library, interleaved, in one
# box session (clocks differ between boxes).  Usage: gpurun -- bash tools/gpu_ab.sh TAG "c2 c3"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}
mkdir -p $O
WS=${2:-c2}
for rep in 1 2; do
  for V in base build_var/*.so; do
    b=$(basename $V .so)
    for W in $WS; do
      if [ "$V" = base ]; then
        timeout -k 10 300 python -u bench.py --workload $W --steps 30 --warmup 3 --no-cpu-baseline > $O/${W}_${b}_$rep.json 2> $O/${W}_${b}_$rep.err || exit 1
      else
        RYD_ENGINE_LIB=$PWD/$V timeout -k 10 300 python -u bench.py --workload $W --steps 30 --warmup 3 --no-cpu-baseline > $O/${W}_${b}_$rep.json 2> $O/${W}_${b}_$rep.err || exit 1
      fi
    done
  done
done
python - <<'PY'
import glob, json, os, sys
O = sys.argv[1] if len(sys.argv) > 1 else None
PY
for f in $O/*.json; do python -c "
import json,sys; d=json.load(open('$f')); r=d['roofline']; print('$(basename $f)', round(d['ms_per_step'],4), round(r['kernel_ms'],4), round(r['frac'],4), round(r['exec_over_useful'],3))"; done
echo done
