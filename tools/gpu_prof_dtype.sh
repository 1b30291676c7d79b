# rocprofv3 kernel stats of one bench configuration.  Usage: gpurun -- bash tools/gpu_prof_dtype.sh <tag> [bench args...]
# -> gpurun_out/prof_<tag>/**/kernel_stats.csv and gpurun_out/bench_<tag>.log
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --cpu-sample 0 "$@" > gpurun_out/bench_$TAG.log 2>&1
rc=$?
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
exit $rc
