#!/bin/bash
# all trajectory GPU tests (ladder kernels after the helper refactor + the exact kernel)
set -o pipefail
O=gpurun_out/trajfull
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_trajectories.py \
  > $O/pytest.log 2>&1; rc=$?
tail -22 $O/pytest.log
exit $rc
