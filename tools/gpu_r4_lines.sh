# Round-4 bench lines (one box): each line to gpurun_out/<tag>_<name>.json.  Usage: bash tools/gpu_r4_lines.sh <tag> [names...]
# names: base fp16 fp16x3 large_fp16x3 large_bf16 wlv2_bf16 wlv2_fp8 wlv2_fp16x3 small_bf16 small_fp8 small_fp16x3 logmel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py --cpu-sample 0 "$@" > gpurun_out/${TAG}_$n.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/${TAG}_$n.log; return 1; }
  tail -1 gpurun_out/${TAG}_$n.log > gpurun_out/${TAG}_$n.json
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_$n.json')); print('$n', d['value'], d['ms_per_step'], d.get('model_flops_frac'))"
}
for n in "$@"; do
  case $n in
    base) run base --steps 20 --warmup 5 ;;
    fp16) run fp16 --dtype fp16 --steps 20 --warmup 5 ;;
    fp16x3) run fp16x3 --dtype fp16x3 --steps 10 ;;
    large_fp16x3) run large_fp16x3 --model wavlm-large --dtype fp16x3 --steps 5 ;;
    large_bf16) run large_bf16 --model wavlm-large --steps 10 ;;
    wlv2_bf16) run wlv2_bf16 --model whisper-large-v2 --steps 5 --warmup 2 ;;
    wlv2_fp8) run wlv2_fp8 --model whisper-large-v2 --dtype fp8 --steps 5 --warmup 2 ;;
    wlv2_fp16x3) run wlv2_fp16x3 --model whisper-large-v2 --dtype fp16x3 --steps 3 --warmup 1 ;;
    small_bf16) run small_bf16 --model whisper-small --steps 5 --warmup 2 ;;
    small_fp8) run small_fp8 --model whisper-small --dtype fp8 --steps 5 --warmup 2 ;;
    small_fp16x3) run small_fp16x3 --model whisper-small --dtype fp16x3 --steps 5 --warmup 2 ;;
    logmel) run logmel --logmel --steps 20 ;;
    *) echo "unknown line $n"; exit 2 ;;
  esac || exit 1
done
