# Same-box A/B of another libsse.so build against the tree with the per-role timings (profiled pass) printed.
# Usage: gpurun -- bash tools/gpu_ab_lib_roles.sh <tag> <other.so> <rounds> "<role regex>" [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; LIB=$2; N=$3; RX=$4; shift 4
show() { python3 -c "
import json, re; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']['roles']; s=d['steps']
print('$2', d['value'], d['ms_per_step'], {k: round(v['ms']/s, 3) for k, v in r.items() if re.search(r'$RX', k)})"; }
for i in $(seq $N); do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 20 --lib $LIB "$@" > gpurun_out/${TAG}_o$i.log 2>&1 || exit 1
  show gpurun_out/${TAG}_o$i.log "round $i other"
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 20 "$@" > gpurun_out/${TAG}_t$i.log 2>&1 || exit 1
  show gpurun_out/${TAG}_t$i.log "round $i tree "
done
