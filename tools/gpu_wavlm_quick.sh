# WavLM bring-up: WavLM + drop-in GPU tests, then the default bench (twice).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wavlm.py tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wavlm_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --cpu-sample 0 > gpurun_out/bench_wavlm_1.log 2>&1 &&
timeout -k 10 200 python -u bench.py --cpu-sample 0 > gpurun_out/bench_wavlm_2.log 2>&1
