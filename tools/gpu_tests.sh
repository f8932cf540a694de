# Run a subset of the GPU tests: gpurun -- bash tools/gpu_tests.sh TAG [pytest args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-tests}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/$TAG/pytest.log 2>&1
echo "pytest exit=$?" >> gpurun_out/$TAG/pytest.log
tail -3 gpurun_out/$TAG/pytest.log
