#!/bin/bash
# A/B two builds of libsse.so on ONE box, interleaved: tools/ab_bench.sh <a.so> <b.so> <rounds> [bench args]
# (build them with tools/build_variant.sh; both must sit inside the repo so they travel to the box)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
A=$1; B=$2; R=$3; shift 3
for r in $(seq 1 $R); do
  for v in A B; do
    so=$A; [ $v = B ] && so=$B
    SSE_LIB_PATH=$PWD/$so timeout -k 10 300 python bench.py --cpu-sample 0 "$@" > gpurun_out/ab_${v}_$r.log 2>&1 || exit 1
    echo "$v $r $(tail -1 gpurun_out/ab_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], json.dumps({k: round(v["ms"],2) for k, v in d["roofline"]["roles"].items()}))')"
  done
done
