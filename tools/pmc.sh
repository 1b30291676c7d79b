#!/bin/bash
# PMC passes over a short bench run (each pass its own rocprofv3 invocation; no tracing domains
# combined with --pmc).  Usage: tools/pmc.sh <outdir> [bench args...]
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA \
  -d "$OUT/p1" -o p1 --output-format csv -- python3 "$R/bench.py" "$@" > "$OUT/p1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/p2" -o p2 --output-format csv -- python3 "$R/bench.py" "$@" > "$OUT/p2.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d "$OUT/p3" -o p3 --output-format csv -- python3 "$R/bench.py" "$@" > "$OUT/p3.log" 2>&1
echo PMC_DONE
