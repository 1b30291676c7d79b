set -o pipefail
cd $GRAFT_REPO_ROOT
make -C stuttering-speech-representation_amd/csrc -j16 > gpurun_out/make.log 2>&1 &&
bash tools/pmc_gemm.sh gpurun_out/pmc_ffn1 38144 3072 768 gelu 0 &&
bash tools/pmc_gemm.sh gpurun_out/pmc_ffn2 38144 768 3072 res 0 &&
bash tools/pmc_gemm.sh gpurun_out/pmc_sq 8192 8192 8192 plain 0 &&
timeout -k 10 240 python tools/gemm_bench.py 0 > gpurun_out/gemm.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench_wavlm.log 2>&1
