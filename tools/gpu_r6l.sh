# Round 6: libsse GEMMs vs hipBLASLt on the bench shapes, then the same under a rocprofv3 kernel trace (library kernel names)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/vendor_gemm_ab.py --json gpurun_out/${TAG}_vendor.json > gpurun_out/${TAG}_vendor.log 2>&1 || { tail -20 gpurun_out/${TAG}_vendor.log; exit 1; }
cat gpurun_out/${TAG}_vendor.log | grep -v amdgpu.ids
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_kt -o kt --output-format csv -- python3 $R/tools/vendor_gemm_ab.py --reps 5 > $R/gpurun_out/${TAG}_kt.log 2>&1 || { echo "trace failed"; tail -5 $R/gpurun_out/${TAG}_kt.log; exit 1; }
cd $R
cut -c1-220 gpurun_out/${TAG}_kt/kt_kernel_stats.csv | head -30
echo done
