# Round-3 measurement set: every GPU test, smoke(), the default bench line (with the CPU baseline),
# a rocprofv3 kernel-stats pass of the default bench, and fp16 / fp16x3 bench lines.
# Usage: gpurun -- bash tools/gpu_r3_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3final}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { tail -5 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-200
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-sample 0 --steps 10 > $GRAFT_REPO_ROOT/$O/bench_rocprof.log 2>&1) || exit 1
timeout -k 10 300 python -u bench.py --cpu-sample 0 --dtype fp16 > $O/bench_fp16.log 2>&1 || exit 1
tail -1 $O/bench_fp16.log | cut -c1-200
timeout -k 10 300 python -u bench.py --cpu-sample 0 --dtype fp16x3 > $O/bench_fp16x3.log 2>&1 || exit 1
tail -1 $O/bench_fp16x3.log | cut -c1-200
timeout -k 10 400 python -u bench.py --cpu-sample 0 --model wavlm-large > $O/bench_wavlm_large_bf16.log 2>&1 || exit 1
tail -1 $O/bench_wavlm_large_bf16.log | cut -c1-200
timeout -k 10 400 python -u bench.py --cpu-sample 0 --model whisper-large-v2 > $O/bench_whisper_bf16.log 2>&1 || exit 1
tail -1 $O/bench_whisper_bf16.log | cut -c1-200
timeout -k 10 400 python -u bench.py --cpu-sample 0 --model whisper-large-v2 --dtype fp8 > $O/bench_whisper_fp8.log 2>&1 || exit 1
tail -1 $O/bench_whisper_fp8.log | cut -c1-200
timeout -k 10 300 python -u bench.py --cpu-sample 0 --logmel > $O/bench_logmel.log 2>&1 || exit 1
tail -1 $O/bench_logmel.log | cut -c1-200
