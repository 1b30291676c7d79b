# Round 6: does a small batch's conv0 output stay in the Infinity Cache?  conv0 time per clip at B = 8 / 16 / 24 / 256
# (single stream).  Usage: gpurun -- bash tools/gpu_r6p.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for B in 8 16 24 32 256; do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --batch $B --steps 20 --warmup 5 --opt no_split=1 > gpurun_out/$1_b$B.log 2>&1 || { tail -5 gpurun_out/$1_b$B.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/$1_b$B.log').read().strip().splitlines()[-1]); r=d['roofline']['roles']; s=d['steps']; B=$B
print('B', B, 'ms/step', d['ms_per_step'], {k: round(1e3*v['ms']/s/B, 3) for k, v in r.items() if k in ('conv0_gn', 'gemm:conv', 'gemm_conv:posconv', 'attn')}, 'us/clip')"
done
echo done
