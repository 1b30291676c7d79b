# Round 6: WavLM-base with the residual GEMM in two phases too (default) vs four phases (gemm_4phase = 1), three rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for o in 1 0; do
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 30 --warmup 5 --opt gemm_4phase=$o > gpurun_out/$1_b$o.log 2>&1 || { tail -5 gpurun_out/$1_b$o.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/$1_b$o.log').read().strip().splitlines()[-1]); r=d['roofline']; s=d['steps']; print('round $r gemm_4phase=$o', d['value'], d['ms_per_step'], {k: round(v['ms']/s,3) for k,v in r['roles'].items() if k in ('gemm:oproj','gemm:ffn2')})"
  done
done
