# A/B of SSE_GEMM_RESP (residual GEMMs on the persistent acc-init kernel): tests, then interleaved benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "residual_persistent" > gpurun_out/resp_tests.log 2>&1 || exit 1
for i in 1 2; do
  for v in 0 1; do
    SSE_GEMM_RESP=$v timeout -k 10 200 python -u bench.py --cpu-sample 0 > gpurun_out/resp_bench_${v}_$i.log 2>&1 || exit 1
  done
done
