# GEMM kernel tests, epilogue microbench (default / non-persistent), A/B bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/kt.log 2>&1 &&
timeout -k 10 200 python tools/gemm_epi_bench.py > gpurun_out/epi_default.log 2>&1 &&
SSE_GEMM_PERSIST=0 timeout -k 10 200 python tools/gemm_epi_bench.py > gpurun_out/epi_np.log 2>&1 &&
bash tools/ab_bench.sh "" "SSE_GEMM_PERSIST=0" 2 > gpurun_out/ab.log 2>&1
