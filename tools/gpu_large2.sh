# WavLM-large: parity tests + bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wavlm.py -x -v -s --timeout 200 --timeout-method thread -k "large" > gpurun_out/large_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model wavlm-large --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/bench_wavlm_large.log 2>&1
