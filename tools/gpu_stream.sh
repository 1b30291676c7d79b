# Streaming (pinned H2D double-buffered) benches: Whisper fp8 B=128 and WavLM.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --model whisper-large-v2 --dtype fp8 --steps 4 --warmup 2 --cpu-sample 0 --stream > gpurun_out/bench_whisper_fp8_stream.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-sample 0 --stream > gpurun_out/bench_wavlm_stream.log 2>&1
