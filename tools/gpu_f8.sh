# fp8 attention step: the fp8 / Whisper GPU tests, then the Whisper-large-v2 fp8 bench with the fp8 attention
# (default) and with the bf16 attention (fp8_attn_bf16=1), interleaved.
# Usage: gpurun -- bash tools/gpu_f8.sh <tag> "<pytest -k expr | all | none>" [rounds] [option, default fp8_attn_bf16]
#        [option values, default "0 1"]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; SEL=$2; ROUNDS=${3:-1}; OPT=${4:-fp8_attn_bf16}; VALS=${5:-"0 1"}
if [ "$SEL" != "none" ]; then
  if [ "$SEL" = "all" ]; then K=(); else K=(-k "$SEL"); fi
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -s -x --timeout 300 --timeout-method thread "${K[@]}" > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  grep -E "rel-L2|rel |passed|failed|FAILED|Error" gpurun_out/${TAG}_tests.log | tail -40
  [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 $ROUNDS); do
  for o in $VALS; do
    timeout -k 10 300 python -u bench.py --model whisper-large-v2 --dtype fp8 --steps 6 --warmup 2 --cpu-sample 0 \
      --opt $OPT=$o > gpurun_out/${TAG}_bench_$o.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench_$o.log; exit 1; }
    echo "round $r $OPT=$o: $(tail -1 gpurun_out/${TAG}_bench_$o.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], {k: v for k, v in d.get("roles", {}).items() if "attn" in k or "qk" in k or ":v" in k})')"
  done
done
