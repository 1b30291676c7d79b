# Round-end measurement on one GPU box: every GPU test, smoke(), the three bench lines and the
# rocprofv3 kernel-trace stats of the WavLM and Whisper-fp8 benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_wavlm.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model whisper-large-v2 --steps 3 --warmup 1 > gpurun_out/bench_whisper_bf16.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model whisper-large-v2 --dtype fp8 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_whisper_fp8.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_wavlm -o wavlm -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --cpu-sample 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/prof_wavlm.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_whisper_fp8 -o whisper_fp8 -- python3 $GRAFT_REPO_ROOT/bench.py --model whisper-large-v2 --dtype fp8 --steps 2 --warmup 1 --cpu-sample 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/prof_whisper_fp8.log 2>&1 &&
python3 $GRAFT_REPO_ROOT/tools/trace_gaps.py $GRAFT_REPO_ROOT/gpurun_out/prof_wavlm/wavlm_kernel_trace.csv > $GRAFT_REPO_ROOT/gpurun_out/gaps.txt
