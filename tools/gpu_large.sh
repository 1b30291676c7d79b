# WavLM-large (the reference's default model) bench + kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --model wavlm-large --steps 5 --warmup 2 --cpu-sample 8 > gpurun_out/bench_wavlm_large.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_large -o large -- python3 $GRAFT_REPO_ROOT/bench.py --model wavlm-large --steps 3 --warmup 1 --cpu-sample 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/prof_large.log 2>&1
