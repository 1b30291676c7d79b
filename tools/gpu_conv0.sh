# conv0 on the matrix cores: WavLM GPU tests, then the default bench with the MFMA and VALU conv0.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wavlm.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/conv0_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --cpu-sample 0 > gpurun_out/bench_conv0_mfma.log 2>&1 &&
SSE_CONV0_VALU=1 timeout -k 10 200 python -u bench.py --cpu-sample 0 > gpurun_out/bench_conv0_valu.log 2>&1 &&
timeout -k 10 200 python -u bench.py --cpu-sample 0 > gpurun_out/bench_conv0_mfma2.log 2>&1
