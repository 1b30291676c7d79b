# Whisper-large-v2 benches (bf16 B=64 configs[2], fp8 B=128 configs[4]) + kernel-trace stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --model whisper-large-v2 --dtype fp8 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_whisper_fp8.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model whisper-large-v2 --dtype bf16 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_whisper_bf16.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_whisper_fp8 -o whisper_fp8 -- python3 $GRAFT_REPO_ROOT/bench.py --model whisper-large-v2 --dtype fp8 --steps 2 --warmup 1 --cpu-sample 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/prof_whisper_fp8.log 2>&1
