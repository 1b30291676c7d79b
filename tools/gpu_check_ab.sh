# GPU tests (pytest -k selection) then a same-box A/B of ab/base.so vs the tree's libsse.so.
# Usage: gpurun -- bash tools/gpu_check_ab.sh "<pytest -k expr>" [rounds] [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=$1; N=${2:-3}; shift 2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$SEL" > gpurun_out/check_tests.log 2>&1
rc=$?
tail -3 gpurun_out/check_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh ab/base.so $N "$@"
