# Round-2 validation + measurement set: full GPU suite, smoke, default bench, its kernel-trace stats,
# Whisper-large-v2 bf16 / MX-fp8 bench lines, log-mel line.  Usage: gpurun --timeout 1200 -- bash tools/gpu_round2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench_wavlm.log 2>&1 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-sample 0 --steps 10 > $GRAFT_REPO_ROOT/$O/bench_wavlm_rocprof.log 2>&1) &&
timeout -k 10 300 python -u bench.py --model whisper-large-v2 --dtype bf16 --steps 6 --warmup 2 --cpu-sample 0 > $O/bench_whisper_bf16.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model whisper-large-v2 --dtype fp8 --batch 128 --steps 6 --warmup 2 --cpu-sample 0 > $O/bench_whisper_fp8.log 2>&1 &&
timeout -k 10 300 python -u bench.py --logmel --steps 10 --warmup 3 > $O/bench_logmel.log 2>&1
rc=$?
tail -2 $O/gputests.log; tail -1 $O/smoke.log; for f in bench_wavlm bench_whisper_bf16 bench_whisper_fp8 bench_logmel; do tail -1 $O/$f.log | cut -c1-200; done
exit $rc
