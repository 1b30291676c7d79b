#!/bin/bash
# HBM traffic per kernel launch over a short bench run: one rocprofv3 --pmc pass per counter
# (FETCH_SIZE, WRITE_SIZE; no tracing domains), then tools/pmc_traffic.py folds them into a JSON
# (gfx950 correction: FETCH_SIZE x 2, MI355X_MICROARCH.md "HBM").
# Usage: tools/pmc_traffic.sh <outdir> <out.json> [bench args...]
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/$1; JS=$R/$2; shift 2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python3 "$R/bench.py" --no-profile --cpu-sample 0 "$@" > "$OUT/fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- python3 "$R/bench.py" --no-profile --cpu-sample 0 "$@" > "$OUT/write.log" 2>&1
python3 "$R/tools/pmc_traffic.py" "$OUT" "$JS" "$@"
