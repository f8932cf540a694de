#!/bin/bash
# C5 A/B of the default build against build/libryd_<v>.so variants, plus the phase profile
set -o pipefail
O=gpurun_out/${2:-c5abp}
mkdir -p $O
export PYTHONPATH=$PWD
bash tools/gpu_ab_c5.sh "$1" ${2:-c5abp} || exit 1
RYD_ENGINE_LIB=$PWD/build/libryd_tprof.so timeout -k 10 200 python -u tools/traj_prof.py > $O/phase.log 2>&1 || exit 1
cat $O/phase.log
