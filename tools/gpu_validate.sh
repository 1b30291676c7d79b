set -o pipefail
cd $GRAFT_REPO_ROOT
make -C stuttering-speech-representation_amd/csrc -j16 > gpurun_out/make.log 2>&1 &&
timeout -k 10 240 python tools/gemm_bench.py 0 2 3 > gpurun_out/gemm2.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 300 python bench.py --model whisper-large-v2 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_whisper.log 2>&1
