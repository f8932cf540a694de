# GPU suite, then the round-3 measurement pass (tools/gpu_r03_bench.sh).
# Usage: gpurun --timeout 1500 -- bash tools/gpu_r03_all.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03all}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/$TAG/pytest.log
tail -3 gpurun_out/$TAG/pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r03_bench.sh $TAG
