# Round 6: MX-fp8 out-projection on the fp8 Whisper path -- parity (attention MX output, Whisper fp8 fixtures)
# and the wlv2_fp8 line A/B (f8_oproj = 1: MX-fp8 attention output, MX out-projection).  Usage: gpurun -- bash tools/gpu_r6m.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_f8attn.py tests/test_gpu_whisper.py -m gpu -q -rA -k "mx_output or mx_oproj" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
grep -E "rel-L2|passed|failed" gpurun_out/${TAG}_tests.log | tail -30
for o in 0 1 0 1; do
  timeout -k 10 400 python -u bench.py --cpu-sample 0 --model whisper-large-v2 --dtype fp8 --steps 5 --warmup 2 --opt f8_oproj=$o > gpurun_out/${TAG}_f8_$o.log 2>&1 || { tail -5 gpurun_out/${TAG}_f8_$o.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_f8_$o.log').read().strip().splitlines()[-1]); r=d['roofline']; print('f8_oproj=$o', d['value'], d['ms_per_step'], d.get('model_flops_frac'), {k: round(v['ms']/d['steps'],2) for k,v in r['roles'].items() if 'oproj' in k or 'attn' in k})"
done
echo done
