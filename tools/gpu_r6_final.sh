# Round-6 final-tree measurements (one box per part).
#   a: the full GPU suite, smoke(), the default bench line, its rocprofv3 kernel trace (+ kt_reduce) and stats
#   b: PMC traffic (WavLM-base bf16 single-stream, Whisper-large-v2 fp8) and the other bench lines
# Usage: gpurun -- bash tools/gpu_r6_final.sh <tag> a|b
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; PART=$2
R=$GRAFT_REPO_ROOT
if [ "$PART" = "a" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -5 gpurun_out/${TAG}_tests.log; grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -1 gpurun_out/${TAG}_smoke.log
  timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
  tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_kt -o kt --output-format csv -- python3 $R/bench.py --cpu-sample 0 --steps 10 > $R/gpurun_out/${TAG}_kt.log 2>&1 || { echo "kernel trace failed"; tail -3 $R/gpurun_out/${TAG}_kt.log; exit 1; }
  cd $R
  tail -1 gpurun_out/${TAG}_kt.log | cut -c1-300
  python3 tools/kt_reduce.py gpurun_out/${TAG}_kt/kt_kernel_trace.csv --steps 10 --json gpurun_out/${TAG}_kt_reduce.json | head -16
  echo done
  exit 0
fi
bash tools/pmc_traffic.sh gpurun_out/${TAG}_pmc_wavlm gpurun_out/${TAG}_pmc_traffic_wavlm_base_bf16.json --steps 2 --warmup 1 --opt no_split=1 || { echo "pmc wavlm failed"; exit 1; }
bash tools/pmc_traffic.sh gpurun_out/${TAG}_pmc_f8 gpurun_out/${TAG}_pmc_traffic_whisper_large_v2_fp8.json --model whisper-large-v2 --dtype fp8 --steps 2 --warmup 1 || { echo "pmc fp8 failed"; exit 1; }
bash tools/gpu_r4_lines.sh ${TAG} wlv2_fp8 wlv2_bf16 fp16 fp16x3 large_bf16 small_fp8 small_bf16 logmel || exit 1
echo done
