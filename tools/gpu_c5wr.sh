#!/bin/bash
# C5 exact kernel with LDS-assembled outputs: trajectory tests, A/B against the previous build, phases
set -o pipefail
O=gpurun_out/${1:-c5wr}
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_trajectories.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab_c5p.sh "prev" $1 || exit 1
