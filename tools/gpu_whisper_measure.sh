# Whisper-large-v2 bench lines (bf16 B=64, fp8 B=128) and the fp8 kernel-trace stats.
# Usage: gpurun --timeout 900 -- bash tools/gpu_whisper_measure.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --model whisper-large-v2 --dtype fp8 --steps 4 --warmup 2 --cpu-sample 0 > gpurun_out/bench_wfp8.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model whisper-large-v2 --dtype bf16 --steps 4 --warmup 2 --cpu-sample 0 > gpurun_out/bench_wbf16.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_wfp8 -o wfp8 -- python3 $R/bench.py --model whisper-large-v2 --dtype fp8 --steps 2 --warmup 1 --cpu-sample 0 --no-profile > $R/gpurun_out/prof_wfp8.log 2>&1
rc=$?
tail -c 300 $R/gpurun_out/bench_wfp8.log; tail -c 300 $R/gpurun_out/bench_wbf16.log
exit $rc
