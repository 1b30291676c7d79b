# MX GEMM check: probe, MX / GEMM / Whisper tests, the fp8 Whisper-large-v2 line.  Usage: gpurun -- bash tools/gpu_r4_mx.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=$1
timeout -k 10 120 tools/_build/gemm8mx_probe > gpurun_out/${TAG}_mx_probe.txt 2>&1 || { echo "mx probe failed"; exit 1; }
grep -E "^[a-z]|full|no-epi" gpurun_out/${TAG}_mx_probe.txt | head -20
timeout -k 10 700 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -k "mx or gemm or whisper or outlier" > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" gpurun_out/${TAG}_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4_lines.sh $TAG wlv2_fp8
