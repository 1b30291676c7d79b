# MX-fp8 bring-up on one GPU box: new MX tests, then the GEMM kernel tests (bf16 regression).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx.py -v --timeout 120 --timeout-method thread -s > gpurun_out/mx_tests.log 2>&1 ;
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kernel_tests.log 2>&1
