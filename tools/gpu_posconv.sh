# posconv kernel bring-up: WavLM tests, then interleaved A/B benches (SSE_POSCONV_GEMM=0/1).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wavlm.py -x -q --timeout 200 --timeout-method thread > gpurun_out/posconv_tests.log 2>&1 || exit 1
for i in 1 2; do
  for v in 0 1; do
    SSE_POSCONV_GEMM=$v timeout -k 10 200 python -u bench.py --cpu-sample 0 > gpurun_out/pc_bench_${v}_$i.log 2>&1 || exit 1
  done
done
