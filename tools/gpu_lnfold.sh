set -o pipefail
cd $GRAFT_REPO_ROOT
make -C stuttering-speech-representation_amd/csrc -j16 > gpurun_out/make.log 2>&1 &&
timeout -k 10 300 python -m pytest tests/test_gpu_wavlm.py tests/test_gpu_kernels.py -q -x > gpurun_out/gputests.log 2>&1 &&
bash tools/ab_bench.sh "SSE_NO_LNFOLD=1" "" 2 > gpurun_out/ab.log 2>&1
