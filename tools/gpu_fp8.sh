# fp8 Whisper: MX + Whisper tests, fp8 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_whisper.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --model whisper-large-v2 --dtype fp8 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_whisper_fp8.log 2>&1
