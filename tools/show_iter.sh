# print the headline numbers of a gpu_iter.sh run
D=gpurun_out/$1
tail -1 $D/pytest_gpu.log 2>/dev/null
for f in $D/bench_*.json; do python -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$f'.split('/')[-1], 'ms', round(d['ms_per_step'],4), 'pts/s %.3g'%d['value'], 'frac', round(r['frac'],3), 'kernel_ms', round(r['kernel_ms'],4))"; done
python - <<PY 2>/dev/null
import sys; sys.path.insert(0,'tools')
from pmc_summary import collect
f,_=collect('$D/fetch_c2','sym16'); w,_=collect('$D/write_c2','sym16')
F=f['FETCH_SIZE']*2048; W=w['WRITE_SIZE']*1024
print('c2 traffic MB fetch %.2f write %.2f total %.2f ratio %.2f' % (F/1e6, W/1e6, (F+W)/1e6, (F+W)/10.76e6))
PY
