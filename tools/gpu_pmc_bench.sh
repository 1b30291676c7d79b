set -o pipefail
cd $GRAFT_REPO_ROOT
make -C stuttering-speech-representation_amd/csrc -j16 > gpurun_out/make.log 2>&1 &&
bash tools/pmc.sh gpurun_out/pmc_bench --steps 3 --warmup 1 --cpu-sample 0 --no-profile > gpurun_out/pmc_bench.log 2>&1
