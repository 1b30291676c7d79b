# GPU parity suite + default bench on one box.  Usage: gpurun --timeout 1200 -- bash tools/gpu_tests.sh [pytest -k expr]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${1:+-k "$1"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_wavlm.log 2>&1
rc=$?
tail -3 gpurun_out/gputests.log; tail -1 gpurun_out/bench_wavlm.log | cut -c1-600
exit $rc
