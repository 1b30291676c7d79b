# Quick GPU check: attention probe, a pytest -k selection with output, an optional bench A/B of one option.
# Usage: gpurun -- bash tools/gpu_r4_quick.sh <tag> "<pytest -k expr>" [opt=val rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; SEL=$2
timeout -k 10 120 tools/_build/attn_probe > gpurun_out/${TAG}_attn_probe.txt 2>&1 || { echo "attn probe failed"; exit 1; }
grep -v "^  mismatch" gpurun_out/${TAG}_attn_probe.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -k "$SEL" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "rel-L2|rel |passed|failed|FAILED" gpurun_out/${TAG}_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
if [ -n "$3" ]; then bash tools/ab_opt.sh $3 ${4:-2}; fi
