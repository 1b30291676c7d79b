# Round 6: rocprofv3 kernel trace + stats of the fp8 Whisper-large-v2 line (B = 128, 4 steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$1_kt -o kt --output-format csv -- python3 $R/bench.py --cpu-sample 0 --model whisper-large-v2 --dtype fp8 --steps 4 --warmup 1 > $R/gpurun_out/$1_kt.log 2>&1 || { tail -5 $R/gpurun_out/$1_kt.log; exit 1; }
cd $R
tail -1 gpurun_out/$1_kt.log | cut -c1-200
head -14 gpurun_out/$1_kt/kt_kernel_stats.csv | cut -c1-160
