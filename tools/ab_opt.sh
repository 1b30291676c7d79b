# Same-box A/B of one libsse option (interleaved bench runs: default vs --opt NAME=VALUE).
# Usage: gpurun -- bash tools/ab_opt.sh NAME=VALUE [rounds] [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OPT=$1; N=${2:-3}; shift 2
TAG=$(echo $OPT | tr '=' '_')
ms() { python3 -c "import json,sys; print(json.loads(open('$1').read().strip().splitlines()[-1])['ms_per_step'])"; }
for i in $(seq $N); do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-profile --steps 20 "$@" > gpurun_out/abo_${TAG}_off_$i.log 2>&1 &&
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-profile --steps 20 --opt $OPT "$@" > gpurun_out/abo_${TAG}_on_$i.log 2>&1 || exit 1
  echo "$OPT round $i off $(ms gpurun_out/abo_${TAG}_off_$i.log) on $(ms gpurun_out/abo_${TAG}_on_$i.log)"
done
