# Sweep one sse_set_option switch over values, one profiled bench run each; prints ms/step and the
# per-role device ms/step.  Usage: gpurun -- bash tools/gpu_sweep.sh <option> "<v1 v2 ...>" [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OPT=$1; VALS=$2; shift 2
for v in $VALS; do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 10 --opt $OPT=$v "$@" > gpurun_out/sweep_${OPT}_$v.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/sweep_${OPT}_$v.log').read().strip().splitlines()[-1])
print('$OPT=$v', d['ms_per_step'], {k:round(v['ms']/d['steps'],3) for k,v in d['roofline']['roles'].items()})"
done
