#!/bin/bash
# L2 read requests to the memory side (TCC_EA0_RDREQ) vs those "destined for DRAM (MC)" (TCC_EA0_RDREQ_DRAM)
# per kernel over a short bench run (one rocprofv3 --pmc pass, two TCC counters, no tracing domains).
# Usage: gpurun -- bash tools/pmc_dram.sh <tag> [bench args...]
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
OUT=$R/gpurun_out/pmcd_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d "$OUT/p" -o p --output-format csv -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-profile --cpu-sample 0 "$@" > "$OUT/p.log" 2>&1 || { echo "pmc failed"; tail -3 "$OUT/p.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
f = glob.glob(out + "/p/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "TCC_EA0_RDREQ_sum":
        n[k] += 1
res = {}
for k, d in acc.items():
    t, dr = d.get("TCC_EA0_RDREQ_sum", 0.0), d.get("TCC_EA0_RDREQ_DRAM_sum", 0.0)
    res[k] = {"launches": n[k], "rdreq_per_launch": t / max(n[k], 1), "rdreq_dram_per_launch": dr / max(n[k], 1),
              "dram_fraction": dr / t if t else None}
json.dump(res, open(out + "/dram.json", "w"), indent=1)
for k, v in sorted(res.items(), key=lambda kv: -kv[1]["rdreq_per_launch"] * kv[1]["launches"])[:12]:
    print(f"{v['launches']:4d} {v['rdreq_per_launch']:14.0f} {v['rdreq_dram_per_launch']:14.0f} {v['dram_fraction']}  {k[:90]}")
PY
