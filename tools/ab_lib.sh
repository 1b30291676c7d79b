# Same-box A/B of two libsse.so builds (interleaved bench runs): the in-tree library vs --lib <other>.
# Usage: gpurun -- bash tools/ab_lib.sh <other.so> [rounds] [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
LIB=$1; N=${2:-3}; shift 2
ms() { python3 -c "import json,sys; print(json.loads(open('$1').read().strip().splitlines()[-1])['ms_per_step'])"; }
for i in $(seq $N); do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-profile --steps 20 --lib $LIB "$@" > gpurun_out/abl_other_$i.log 2>&1 &&
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-profile --steps 20 "$@" > gpurun_out/abl_tree_$i.log 2>&1 || exit 1
  echo "round $i other $(ms gpurun_out/abl_other_$i.log) tree $(ms gpurun_out/abl_tree_$i.log)"
done
