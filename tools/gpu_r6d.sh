# Round-6 GPU step d: kernel trace of the default (two-stream) bench's timed region -> per-step wall / idle / one
# queue / both queues busy (kt_overlap.py), and the single-stream profiled pass (kt_reduce.py).
# Usage: gpurun -- bash tools/gpu_r6d.sh <tag> [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_kt2 -o kt --output-format csv -- python3 $R/bench.py --cpu-sample 0 --no-profile --steps 10 "$@" > $R/gpurun_out/${TAG}_kt2.log 2>&1 || { echo "trace failed"; tail -3 $R/gpurun_out/${TAG}_kt2.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_kt -o kt --output-format csv -- python3 $R/bench.py --cpu-sample 0 --steps 10 "$@" > $R/gpurun_out/${TAG}_kt.log 2>&1 || { echo "trace failed"; tail -3 $R/gpurun_out/${TAG}_kt.log; exit 1; }
cd $R
tail -1 gpurun_out/${TAG}_kt2.log | cut -c1-200
python3 tools/kt_overlap.py gpurun_out/${TAG}_kt2/kt_kernel_trace.csv --steps 10 | tee gpurun_out/${TAG}_overlap.txt
python3 tools/kt_reduce.py gpurun_out/${TAG}_kt/kt_kernel_trace.csv --steps 10 --json gpurun_out/${TAG}_kt_reduce.json | head -30
echo done
