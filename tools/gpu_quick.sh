# build, GPU parity tests, WavLM bench (default workload)
set -o pipefail
cd $GRAFT_REPO_ROOT
make -C stuttering-speech-representation_amd/csrc -j16 > gpurun_out/make.log 2>&1 &&
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/bench_wavlm.log 2>&1
