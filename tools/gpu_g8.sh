set -o pipefail
cd $GRAFT_REPO_ROOT
make -C stuttering-speech-representation_amd/csrc -j16 > gpurun_out/make.log 2>&1 &&
timeout -k 10 180 python -m pytest tests/test_gpu_kernels.py -q -x -k configs_agree > gpurun_out/g8test.log 2>&1 &&
timeout -k 10 240 python tools/gemm_bench.py 0 4 > gpurun_out/gemm.log 2>&1
