set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "fp16x3 or lnfold or embed_matches" > gpurun_out/x3_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --dtype fp16x3 --cpu-sample 0 --steps 5 --warmup 2 > gpurun_out/bench_x3.log 2>&1 &&
timeout -k 10 300 python -u bench.py --dtype fp32 --cpu-sample 0 --steps 3 --warmup 1 > gpurun_out/bench_fp32.log 2>&1
rc=$?
grep -E "PASS|FAIL|rel" gpurun_out/x3_tests.log | tail -12; tail -1 gpurun_out/bench_x3.log | cut -c1-200; tail -1 gpurun_out/bench_fp32.log | cut -c1-200
exit $rc
