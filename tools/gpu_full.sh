# Full GPU tests, then an A/B bench against ab/head.so (previous commit), then the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 &&
bash tools/ab_bench.sh "" "SSE_LIB_PATH=ab/head.so" 2 > gpurun_out/ab.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_wavlm.log 2>&1
