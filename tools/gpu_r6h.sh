# Round-6 GPU step h: same-box A/B of a library build (default ab/prio.so: static s_setprio 1 for the GEMMs' wave
# group 1) against the tree, on the WavLM-base default line and the fp8 Whisper-large-v2 line.
# Usage: gpurun -- bash tools/gpu_r6h.sh [other.so] [rounds] [fp8 rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
LIB=${1:-ab/prio.so}; N=${2:-3}
echo "wavlm-base bf16 (other = $LIB)"
bash tools/ab_lib.sh $LIB $N || exit 1
echo "whisper-large-v2 fp8 (other = $LIB)"
bash tools/ab_lib.sh $LIB ${3:-$N} --model whisper-large-v2 --dtype fp8 --steps 6 --warmup 2 || exit 1
echo done
