# Quick GPU check: a pytest -k selection plus the default bench.  Usage: gpurun -- bash tools/gpu_quick.sh "<pytest -k expr>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$1" > gpurun_out/quick_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-sample 0 > gpurun_out/bench_quick.log 2>&1
rc=$?
tail -2 gpurun_out/quick_tests.log; tail -1 gpurun_out/bench_quick.log | cut -c1-300
exit $rc
