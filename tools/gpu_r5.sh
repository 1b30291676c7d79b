# Round-5 GPU step: a pytest -k selection (or "all"), then optionally the default bench line.
# Usage: gpurun -- bash tools/gpu_r5.sh <tag> "<pytest -k expr | all | none>" [bench]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; SEL=$2
if [ "$SEL" != "none" ]; then
  if [ "$SEL" = "all" ]; then K=(); else K=(-k "$SEL"); fi
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -s -x --timeout 300 --timeout-method thread "${K[@]}" > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  grep -E "rel-L2|rel |passed|failed|FAILED|Error" gpurun_out/${TAG}_tests.log | tail -40
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$3" = "bench" ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
  tail -1 gpurun_out/${TAG}_bench.log | cut -c1-600
fi
