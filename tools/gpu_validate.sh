# One GPU validation pass: build, GEMM microbench, GPU parity tests, both benches, kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
make -C stuttering-speech-representation_amd/csrc -j16 > gpurun_out/make.log 2>&1 &&
timeout -k 10 240 python tools/gemm_bench.py 0 3 > gpurun_out/gemm.log 2>&1 &&
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench_wavlm.log 2>&1 &&
timeout -k 10 300 python bench.py --model whisper-large-v2 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_whisper.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wavlm -o wavlm -- python bench.py --steps 5 --cpu-sample 0 > gpurun_out/prof_wavlm.log 2>&1
