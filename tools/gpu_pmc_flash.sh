# PMC passes (SQ counters) over a short Whisper-large-v2 bf16 bench: flash attention + GEMM activity.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_flash
mkdir -p $O
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
  -d $O/p1 -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model whisper-large-v2 --batch 16 --steps 1 --warmup 1 --cpu-sample 0 --no-profile > $O/p1.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F GRBM_GUI_ACTIVE \
  -d $O/p2 -o p2 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model whisper-large-v2 --batch 16 --steps 1 --warmup 1 --cpu-sample 0 --no-profile > $O/p2.log 2>&1 &&
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $O/p1 $O/p2 --json $O/summary.json > $O/summary.txt
