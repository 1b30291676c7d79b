# Interleaved same-box A/B of one sse_set_option switch on the default bench (no profiling pass):
# R rounds over the values, clips/s and ms/step per run.  Usage: gpurun -- bash tools/gpu_ab_opt.sh <option> "<v1 v2 ...>" [R] [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OPT=$1; VALS=$2; R=${3:-3}; shift 3
for r in $(seq $R); do
  for v in $VALS; do
    timeout -k 10 200 python -u bench.py --cpu-sample 0 --no-profile --steps 20 --warmup 5 --opt $OPT=$v "$@" > gpurun_out/ab_${OPT}_$v.log 2>&1 || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab_${OPT}_$v.log').read().strip().splitlines()[-1]); print('$OPT=$v', d['value'], d['ms_per_step'])"
  done
done
