# Round-6: WavLM-large bf16 QKV pre-LN fold -- parity (guard FNT 4, folded vs materialised, golden) and the
# large_bf16 line A/B (no_lnfold=1 = the LayerNorm kernel before every QKV).  Usage: gpurun -- bash tools/gpu_r6j.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
timeout -k 10 400 python -u -m pytest tests/test_gpu_guard.py tests/test_gpu_wavlm.py -m gpu -q -k "fnt or large" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -15 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for o in 0 1; do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --model wavlm-large --steps 10 --opt no_lnfold=$o > gpurun_out/${TAG}_large_$o.log 2>&1 || { tail -5 gpurun_out/${TAG}_large_$o.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_large_$o.log').read().strip().splitlines()[-1]); print('no_lnfold=$o', d['value'], d['ms_per_step'], d.get('model_flops_frac'))"
done
timeout -k 10 300 python -u bench.py --cpu-sample 0 --model wavlm-large --steps 10 > gpurun_out/${TAG}_large_again.log 2>&1 && python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_large_again.log').read().strip().splitlines()[-1]); print('again', d['value'], d['ms_per_step'])"
echo done
