# PMC pass 1 (SQ counters) over a short WavLM bench: per-kernel wave/LDS/VALU/MFMA counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_attn
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS \
  -d $GRAFT_REPO_ROOT/gpurun_out/pmc_attn/p1 -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/pmc_attn/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  -d $GRAFT_REPO_ROOT/gpurun_out/pmc_attn/p2 -o p2 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/pmc_attn/p2.log 2>&1 &&
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $GRAFT_REPO_ROOT/gpurun_out/pmc_attn/p1 $GRAFT_REPO_ROOT/gpurun_out/pmc_attn/p2 --json $GRAFT_REPO_ROOT/gpurun_out/pmc_attn/summary.json > $GRAFT_REPO_ROOT/gpurun_out/pmc_attn/summary.txt
