# Round-4 combined GPU check (one box): the full GPU suite, then a same-box A/B of ab/base.so vs the tree,
# then bench lines (tools/gpu_r4_lines.sh).  Usage: gpurun -- bash tools/gpu_r4_check.sh <tag> <ab rounds> [lines...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; N=$2; shift 2
if [ -x tools/_build/attn_probe ]; then
  timeout -k 10 120 tools/_build/attn_probe > gpurun_out/${TAG}_attn_probe.txt 2>&1 || { echo "attn probe failed"; tail -5 gpurun_out/${TAG}_attn_probe.txt; exit 1; }
  cat gpurun_out/${TAG}_attn_probe.txt | grep -v "^  mismatch" 
fi
if [ -x tools/_build/gemm8mx_probe ]; then
  timeout -k 10 120 tools/_build/gemm8mx_probe > gpurun_out/${TAG}_mx_probe.txt 2>&1 || { echo "mx probe failed"; tail -5 gpurun_out/${TAG}_mx_probe.txt; exit 1; }
  cat gpurun_out/${TAG}_mx_probe.txt
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/${TAG}_tests.log | head -20; exit $rc; }
bash tools/ab.sh ab/base.so $N || exit 1
bash tools/gpu_r4_lines.sh $TAG "$@"
