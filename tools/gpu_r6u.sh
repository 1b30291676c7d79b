# Round 6: residual GEMM in two phases (default) vs four phases (gemm_4phase = 1) on the other lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {   # tag, args
  local n=$1; shift
  timeout -k 10 400 python -u bench.py --cpu-sample 0 "$@" > gpurun_out/$TAG_$n.log 2>&1 || { tail -5 gpurun_out/$TAG_$n.log; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/$TAG_$n.log').read().strip().splitlines()[-1]); r=d['roofline']; s=d['steps']; print('$n', d['value'], d['ms_per_step'], {k: round(v['ms']/s,2) for k,v in r['roles'].items() if k in ('gemm:oproj','gemm:ffn2','gemm_mx:ffn2')})"
}
TAG=$1
for r in 1 2; do
  for o in 1 0; do
    run f8_o$o --model whisper-large-v2 --dtype fp8 --steps 5 --warmup 2 --opt gemm_4phase=$o || exit 1
    run wb_o$o --model whisper-large-v2 --steps 5 --warmup 2 --opt gemm_4phase=$o || exit 1
    run lg_o$o --model wavlm-large --steps 10 --opt gemm_4phase=$o || exit 1
  done
done
echo done
