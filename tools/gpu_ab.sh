# GEMM kernel tests + interleaved A/B bench on one box.  Usage: gpurun -- bash tools/gpu_ab.sh "<envA>" "<envB>" [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/kt.log 2>&1 &&
bash tools/ab_bench.sh "$1" "$2" ${3:-3} > gpurun_out/ab.log 2>&1
