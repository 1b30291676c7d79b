# narrow-row bf16 LayerNorm: WavLM tests (base + large), both WavLM benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wavlm.py tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ln_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model wavlm-large --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/bench_wavlm_large.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-sample 0 > gpurun_out/bench_wavlm_1.log 2>&1
