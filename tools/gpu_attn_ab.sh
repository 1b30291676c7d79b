# Kernel-trace A/B of one libsse option on one bench configuration: per-kernel mean durations, default vs
# --opt NAME=VALUE.  Usage: gpurun -- bash tools/gpu_attn_ab.sh <tag> NAME=VALUE [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; OPT=$2; shift 2
for side in off on; do
  extra=""; [ $side = on ] && extra="--opt $OPT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_$side -o kt --output-format csv -- \
    python3 -u bench.py --cpu-sample 0 --no-profile --steps 5 --warmup 2 "$@" $extra > gpurun_out/${TAG}_$side.log 2>&1 || exit 1
  f=$(find gpurun_out/${TAG}_$side -name "kt_kernel_stats.csv" | head -1)
  echo "== $side $OPT"; python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:8]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} x {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:90]}')
PY
done
