# Round 6: every bench line on the two-phase tree (one box)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_r4_lines.sh $1 base wlv2_fp8 wlv2_bf16 fp16 fp16x3 large_bf16 large_fp16x3 small_fp8 small_bf16 small_fp16x3 wlv2_fp16x3 || exit 1
echo done
