# Round 6: two-phase persistent GEMM (option gemm_2phase): bit-identity + per-shape timing, then the default bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_2phase_ab.py > gpurun_out/$1_gemm.log 2>&1 || { tail -20 gpurun_out/$1_gemm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$1_gemm.log | grep -v "^{"
for r in 1 2; do
  for o in 0 1; do
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 30 --warmup 5 --opt gemm_2phase=$o > gpurun_out/$1_b$o.log 2>&1 || { tail -5 gpurun_out/$1_b$o.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/$1_b$o.log').read().strip().splitlines()[-1]); r=d['roofline']; s=d['steps']; print('round $r gemm_2phase=$o', d['value'], d['ms_per_step'], {k: round(v['ms']/s,3) for k,v in r['roles'].items() if k.startswith('gemm')})"
  done
done
echo done
