# Round 6: long-K GEMM probe (persistent / non-persistent / hipBLASLt).  Usage: gpurun -- bash tools/gpu_r6o.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_longk_probe.py > gpurun_out/$1_longk.log 2>&1 || { tail -20 gpurun_out/$1_longk.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$1_longk.log
