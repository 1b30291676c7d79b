# Round-6 GPU step b: short-T attention probe (full / pipe / pipe2, bitwise + timed), the attention and fp8-attention
# tests, the fp16-vs-bf16 operand-power probe, then a same-box A/B of the default bench (attn_short 0 vs 2).
# Usage: gpurun -- bash tools/gpu_r6b.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
timeout -k 10 300 pbin/attn_probe > gpurun_out/${TAG}_attn_probe.txt 2>&1 || { tail -5 gpurun_out/${TAG}_attn_probe.txt; exit 1; }
cat gpurun_out/${TAG}_attn_probe.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -k "attention_pipe or f8attn" > gpurun_out/${TAG}_sel.log 2>&1
rc=$?
grep -E "sink|passed|failed|FAILED" gpurun_out/${TAG}_sel.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u tools/fp16_power_probe.py 3 > gpurun_out/${TAG}_fp16_power.txt 2>&1 || { tail -5 gpurun_out/${TAG}_fp16_power.txt; exit 1; }
head -5 gpurun_out/${TAG}_fp16_power.txt
bash tools/ab_opt.sh attn_short=2 3 || exit 1
echo done
