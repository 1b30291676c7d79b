# Round 6: where a persistent GEMM tile's time goes under the two-phase schedule (pbin/gemm8_probe, then "4": four phases)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 pbin/gemm8_probe > gpurun_out/$1_p2.txt 2>&1 || { tail -5 gpurun_out/$1_p2.txt; exit 1; }
timeout -k 10 300 pbin/gemm8_probe 4 > gpurun_out/$1_p4.txt 2>&1 || { tail -5 gpurun_out/$1_p4.txt; exit 1; }
echo done
