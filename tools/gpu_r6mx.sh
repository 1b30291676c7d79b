# Round 6: fp8 Whisper-large-v2 with the two-phase MX schedule (default) vs four phases (gemm_4phase = 1), three rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for o in 0 1; do
    timeout -k 10 400 python -u bench.py --cpu-sample 0 --model whisper-large-v2 --dtype fp8 --steps 5 --warmup 2 --opt gemm_4phase=$o > gpurun_out/$1_f$o.log 2>&1 || { tail -5 gpurun_out/$1_f$o.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/$1_f$o.log').read().strip().splitlines()[-1]); r=d['roofline']; s=d['steps']; print('round $r gemm_4phase=$o', d['value'], d['ms_per_step'], {k: round(v['ms']/s,2) for k,v in r['roles'].items() if k.startswith('gemm')})"
  done
done
