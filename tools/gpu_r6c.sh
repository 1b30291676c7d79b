# Round-6 GPU step c: the full GPU suite, smoke(), the default bench line, and the fp16 / bf16 operand clocks
# (rocprofv3 GRBM_GUI_ACTIVE per GEMM launch, tools/fp16_power_probe.py pmc / clocks).
# Usage: gpurun -- bash tools/gpu_r6c.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_tests.log
grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $R/gpurun_out/${TAG}_clk -o c --output-format csv -- python3 $R/tools/fp16_power_probe.py pmc > $R/gpurun_out/${TAG}_clk.log 2>&1 || { echo "clock pass failed"; tail -3 $R/gpurun_out/${TAG}_clk.log; exit 1; }
cd $R
f=$(ls gpurun_out/${TAG}_clk/*counter_collection.csv | head -1)
python3 tools/fp16_power_probe.py clocks $f > gpurun_out/${TAG}_clocks.txt 2>&1 || { tail -3 gpurun_out/${TAG}_clocks.txt; exit 1; }
head -20 gpurun_out/${TAG}_clocks.txt
echo done
