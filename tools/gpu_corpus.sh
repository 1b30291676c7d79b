# configs[3] corpus mode on one GPU (50k clips), plus the torchrun launch form of the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --corpus 50000 > gpurun_out/bench_corpus.log 2>&1 &&
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/bench_torchrun.log 2>&1
