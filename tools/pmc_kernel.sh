#!/bin/bash
# SQ counter passes restricted to kernels matching a regex over a short bench.py run (each pass its own
# rocprofv3 run, no tracing domains).  Usage: gpurun -- bash tools/pmc_kernel.sh <tag> <regex> [bench args...]
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; RX=$2; shift 2
OUT=$R/gpurun_out/pmck_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 2 --warmup 1 --no-profile --cpu-sample 0 $*"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INSTS_MFMA"
P3="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$RX" -d "$OUT/p$i" -o p$i --output-format csv -- python3 $B > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$OUT/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$OUT/p1" "$OUT/p2" "$OUT/p3" --json "$OUT/sq.json" > "$OUT/sq.txt"
cat "$OUT/sq.txt"
