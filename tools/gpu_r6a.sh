# Round-6 first GPU step: the fp8-attention / MX-residual selection with its printed numbers, the full GPU
# suite, the default bench line, then SQ counters of the two attention kernels VERDICT r5 names
# (attention_pipe_kernel on WavLM-base B = 256, attention_f8_kernel on Whisper-large-v2 fp8).
# Usage: gpurun -- bash tools/gpu_r6a.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
if [ -x pbin/gemm8_probe ]; then
  timeout -k 10 300 pbin/gemm8_probe h 3 > gpurun_out/${TAG}_gemm8h_probe.txt 2>&1 || { tail -5 gpurun_out/${TAG}_gemm8h_probe.txt; exit 1; }
  cat gpurun_out/${TAG}_gemm8h_probe.txt
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -k "f8attn or residual_in_place" > gpurun_out/${TAG}_sel.log 2>&1
grep -E "f8 attention|passed|failed|FAILED" gpurun_out/${TAG}_sel.log | tail -45
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-500
bash tools/pmc_kernel.sh ${TAG}_attn_pipe attention_pipe || exit 1
bash tools/pmc_kernel.sh ${TAG}_attn_f8 attention_f8 --model whisper-large-v2 --dtype fp8 --batch 32 || exit 1
echo done
