#!/bin/bash
# One profiling pass set over a short bench.py run (default WavLM-base bf16 B=256): kernel-trace
# stats, two SQ counter passes (cycle accounting, instruction mix) and the HBM traffic passes
# (FETCH_SIZE, WRITE_SIZE), each its own rocprofv3 run (no tracing domains with --pmc).
# Usage: gpurun -- bash tools/pmc_bench.sh <tag> [bench args...]  -> gpurun_out/pmc_<tag>/
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 2 --warmup 1 --no-profile --cpu-sample 0 $*"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 $B > "$OUT/kt.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA -d "$OUT/p1" -o p1 --output-format csv -- python3 $B > "$OUT/p1.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d "$OUT/p2" -o p2 --output-format csv -- python3 $B > "$OUT/p2.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python3 $B > "$OUT/fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- python3 $B > "$OUT/write.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$OUT/p1" "$OUT/p2" --json "$OUT/sq.json" > "$OUT/sq.txt"
python3 "$R/tools/pmc_traffic.py" "$OUT" "$OUT/traffic.json" $* > "$OUT/traffic.txt"
echo PMC_DONE
