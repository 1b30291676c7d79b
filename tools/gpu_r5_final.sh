# Round-5 final-tree measurement (one box): the full GPU suite, smoke(), the default bench line,
# its rocprofv3 kernel trace (+ kt_reduce), WavLM-base PMC traffic, the Whisper-large-v2 fp8 / bf16 lines.
# Usage: gpurun -- bash tools/gpu_r5_final.sh <tag> [a|b|all]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; PART=${2:-all}   # a: tests, smoke, bench, kernel trace; b: PMC traffic and the Whisper lines
R=$GRAFT_REPO_ROOT
if [ "$PART" != "b" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -5 gpurun_out/${TAG}_tests.log; grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_kt -o kt --output-format csv -- python3 $R/bench.py --cpu-sample 0 --steps 10 > $R/gpurun_out/${TAG}_kt.log 2>&1 || { echo "kernel trace failed"; tail -3 $R/gpurun_out/${TAG}_kt.log; exit 1; }
cd $R
python3 tools/kt_reduce.py gpurun_out/${TAG}_kt/kt_kernel_trace.csv --steps 10 --json gpurun_out/${TAG}_kt_reduce.json | head -16
fi
[ "$PART" = "a" ] && { echo done; exit 0; }
bash tools/pmc_traffic.sh gpurun_out/${TAG}_pmc_wavlm gpurun_out/${TAG}_pmc_traffic_wavlm_base_bf16.json --steps 2 --warmup 1 --opt no_split=1 || { echo "pmc wavlm failed"; exit 1; }
bash tools/gpu_r4_lines.sh ${TAG} wlv2_fp8 wlv2_bf16 || exit 1
echo done
