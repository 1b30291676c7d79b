#!/bin/bash
# A/B two configurations on ONE box, interleaved in separate processes:
#   tools/ab_bench.sh "<env A>" "<env B>" <rounds> [bench args]
# e.g. "SSE_LIB_PATH=ab/old.so" "SSE_LIB_PATH=ab/new.so", or "" "SSE_NO_LNFOLD=1".
# Library builds of a git revision: tools/build_variant.sh <rev> ab/<name>.so (kept inside the
# repo so they travel to the box).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
A=$1; B=$2; R=$3; shift 3
for r in $(seq 1 $R); do
  for v in A B; do
    envs=$A; [ $v = B ] && envs=$B
    envs=${envs//SSE_LIB_PATH=/SSE_LIB_PATH=$PWD/}
    env $envs timeout -k 10 300 python bench.py --cpu-sample 0 "$@" > gpurun_out/ab_${v}_$r.log 2>&1 || exit 1
    echo "$v $r $(tail -1 gpurun_out/ab_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], json.dumps({k: round(v["ms"],2) for k, v in d["roofline"]["roles"].items()}))')"
  done
done
