# Round-2 measurement set: PMC passes of the headline bench (tools/pmc_bench.sh), then the fp16x3 and
# headline bench lines.  Usage: gpurun --timeout 1100 -- bash tools/gpu_r2_measure.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/pmc_bench.sh r2_bf16 > gpurun_out/pmc_r2.log 2>&1 &&
cd $R && timeout -k 10 300 python -u bench.py --dtype fp16x3 --steps 10 --warmup 3 > gpurun_out/bench_fp16x3.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_bf16.log 2>&1
rc=$?
tail -2 gpurun_out/pmc_r2.log; tail -c 400 gpurun_out/bench_bf16.log
exit $rc
