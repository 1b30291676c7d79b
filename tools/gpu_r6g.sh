# Round-6 GPU step g: the LN -> MX producer test and the fp8 Whisper tests after the paired 16-B fp8 stores of the
# LayerNorm producer, then a same-box A/B of the fp8 Whisper-large-v2 line against ab/base_r6.so.
# Usage: gpurun -- bash tools/gpu_r6g.sh <tag> [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; N=${2:-3}
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "mx or f8 or whisper" > gpurun_out/${TAG}_sel.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_sel.log
grep -E "FAILED|Error" gpurun_out/${TAG}_sel.log | head -20
[ $rc -eq 0 ] || exit $rc
bash tools/ab_lib.sh ab/base_r6.so $N --model whisper-large-v2 --dtype fp8 --steps 6 --warmup 2 || exit 1
echo done
