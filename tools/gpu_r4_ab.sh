# Round-4 GPU check: GEMM probe, a pytest -k selection, then a same-box A/B of ab/base.so vs the tree.
# Usage: gpurun -- bash tools/gpu_r4_ab.sh "<pytest -k expr>" [rounds] [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=$1; N=${2:-3}; shift 2
if [ -x tools/_build/gemm8_probe ]; then
  timeout -k 10 200 tools/_build/gemm8_probe > gpurun_out/probe.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/probe.txt; exit 1; }
  grep -E "differ|full |deferred|M=" gpurun_out/probe.txt | head -40
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$SEL" > gpurun_out/check_tests.log 2>&1
rc=$?
tail -3 gpurun_out/check_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh ab/base.so $N "$@"
