# Same-box A/B of two libsse.so builds (interleaved bench runs).  Build B first here:
#   git stash; make -C <pkg>/csrc; cp <pkg>/libsse.so ab/base.so; git stash pop; make ...
# Usage: gpurun -- bash tools/ab.sh ab/base.so [rounds] [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
BASE=$1; N=${2:-3}; shift 2
for i in $(seq $N); do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-profile --steps 20 --lib $BASE "$@" > gpurun_out/ab_base_$i.log 2>&1 &&
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-profile --steps 20 "$@" > gpurun_out/ab_new_$i.log 2>&1 || exit 1
  echo "round $i base $(python3 -c "import json,sys; print(json.loads(open('gpurun_out/ab_base_$i.log').read().strip().splitlines()[-1])['ms_per_step'])") new $(python3 -c "import json,sys; print(json.loads(open('gpurun_out/ab_new_$i.log').read().strip().splitlines()[-1])['ms_per_step'])")"
done
