# Round 6: two-phase schedule in all 8-wave GEMMs (persistent, residual, MX): whole-model bit identity, GEMM/MX tests,
# then WavLM-base and Whisper-large-v2 fp8 bench A/B (gemm_4phase = 1: four phases).  Usage: gpurun -- bash tools/gpu_r6s.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/phase_model_ab.py > gpurun_out/$1_ident.log 2>&1 || { tail -20 gpurun_out/$1_ident.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$1_ident.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_guard.py tests/test_gpu_mx.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$1_tests.log 2>&1 || { tail -30 gpurun_out/$1_tests.log; exit 1; }
tail -1 gpurun_out/$1_tests.log
for r in 1 2; do
  for o in 0 1; do
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 30 --warmup 5 --opt gemm_4phase=$o > gpurun_out/$1_b$o.log 2>&1 || { tail -5 gpurun_out/$1_b$o.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/$1_b$o.log').read().strip().splitlines()[-1]); r=d['roofline']; s=d['steps']; print('round $r wavlm gemm_4phase=$o', d['value'], d['ms_per_step'], {k: round(v['ms']/s,3) for k,v in r['roles'].items() if k.startswith('gemm')})"
  done
done
for r in 1 2; do
  for o in 0 1; do
    timeout -k 10 400 python -u bench.py --cpu-sample 0 --model whisper-large-v2 --dtype fp8 --steps 5 --warmup 2 --opt gemm_4phase=$o > gpurun_out/$1_f$o.log 2>&1 || { tail -5 gpurun_out/$1_f$o.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/$1_f$o.log').read().strip().splitlines()[-1]); r=d['roofline']; s=d['steps']; print('round $r fp8 gemm_4phase=$o', d['value'], d['ms_per_step'], {k: round(v['ms']/s,2) for k,v in r['roles'].items() if k.startswith('gemm')})"
  done
done
echo done
