# pytest -k selection on the GPU with prints (-s).  Usage: gpurun -- bash tools/gpu_k.sh "<expr>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "$1" > gpurun_out/k_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|rel|Error" gpurun_out/k_tests.log | tail -30
exit $rc
