# PMC passes over a short WavLM-base bench run (tools/pmc.sh) + HBM traffic per kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/pmc.sh gpurun_out/pmc_bench --steps 2 --warmup 1 --cpu-sample 0 --no-profile > gpurun_out/pmc_bench.log 2>&1 &&
python3 tools/pmc_summary.py gpurun_out/pmc_bench --json gpurun_out/pmc_bench/summary.json > gpurun_out/pmc_summary.txt 2>&1
