#!/bin/bash
# SQ / TCC counter passes over one GEMM shape (each pass its own rocprofv3; no tracing domains).
# Usage: tools/pmc_gemm.sh <outdir> M N K epi cfg
set -e
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS \
  -d "$R/$OUT/p1" -o p1 --output-format csv -- python3 "$R/tools/gemm_one.py" "$@" 10 > "$R/$OUT/p1.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  -d "$R/$OUT/p2" -o p2 --output-format csv -- python3 "$R/tools/gemm_one.py" "$@" 10 > "$R/$OUT/p2.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d "$R/$OUT/p3" -o p3 --output-format csv -- python3 "$R/tools/gemm_one.py" "$@" 10 > "$R/$OUT/p3.log" 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/kt" -o kt -- python3 "$R/tools/gemm_one.py" "$@" 10 > "$R/$OUT/kt.log" 2>&1
echo PMC_DONE
