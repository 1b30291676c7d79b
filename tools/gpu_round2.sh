set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_wavlm.log 2>&1 &&
timeout -k 10 300 python -u tools/gemm_bench.py 0 > gpurun_out/gemm_bench.log 2>&1
rc=$?
tail -3 gpurun_out/gputests.log; tail -1 gpurun_out/bench_wavlm.log | cut -c1-300; cat gpurun_out/gemm_bench.log | tail -2
exit $rc
