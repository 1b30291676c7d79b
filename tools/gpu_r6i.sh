# Round-6 GPU step i: fp8 Whisper-large-v2 A/B of the tree against ab/base_r6.so (the 16-B fp8 stores, GEMM + LN -> MX),
# then tools/gpu_r6h.sh (static-priority GEMM build ab/prio.so vs the tree, WavLM-base and fp8 Whisper).
set -o pipefail
cd $GRAFT_REPO_ROOT
echo "fp8 stores: other = ab/base_r6.so"
bash tools/ab_lib.sh ab/base_r6.so 2 --model whisper-large-v2 --dtype fp8 --steps 6 --warmup 2 || exit 1
bash tools/gpu_r6h.sh ab/prio.so 3 2 || exit 1
