# Round validation on one GPU box: GPU parity tests, smoke(), WavLM bench, kernel-trace stats.
# Usage (from this container): gpurun --timeout 1000 -- bash tools/gpu_round.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_wavlm.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_wavlm -o wavlm -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --cpu-sample 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/prof_wavlm.log 2>&1 &&
python3 $GRAFT_REPO_ROOT/tools/trace_gaps.py $GRAFT_REPO_ROOT/gpurun_out/prof_wavlm/wavlm_kernel_trace.csv > $GRAFT_REPO_ROOT/gpurun_out/gaps.txt
