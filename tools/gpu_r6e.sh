# Round-6 GPU step e: interleaved same-box bench A/B of the WavLM batch split: default (two streams sharing every
# CU), CU-masked halves (split_cumask 1: low / high CUs, 2: even / odd), and one stream (no_split 1).
# Usage: gpurun -- bash tools/gpu_r6e.sh <tag> [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; N=${2:-3}
ms() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])"; }
for i in $(seq $N); do
  for v in base split_cumask=1 split_cumask=2 no_split=1; do
    o=""; [ "$v" = base ] || o="--opt $v"
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-profile --steps 20 $o > gpurun_out/${TAG}_${v}_$i.log 2>&1 || { tail -3 gpurun_out/${TAG}_${v}_$i.log; exit 1; }
    echo "round $i $v $(ms gpurun_out/${TAG}_${v}_$i.log)"
  done
done
