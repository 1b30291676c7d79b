# HBM traffic per launch (rocprofv3 PMC FETCH_SIZE / WRITE_SIZE, one pass each) for the WavLM bf16
# and Whisper-large-v2 fp8 benches -> profiles/r1_pmc_traffic_*.json (read by bench.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/pmc_traffic.sh gpurun_out/pmc_wavlm gpurun_out/r1_pmc_traffic_wavlm_base_bf16.json --steps 2 --warmup 1 &&
bash tools/pmc_traffic.sh gpurun_out/pmc_whisper_fp8 gpurun_out/r1_pmc_traffic_whisper_large_v2_fp8.json --model whisper-large-v2 --dtype fp8 --steps 1 --warmup 1
