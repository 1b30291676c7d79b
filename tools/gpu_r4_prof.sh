# Round-4 profile pass (one box): attention probe, a profiled WavLM-base bench (per-role ms/step), the
# rocprofv3 kernel-trace stats of the same command, and log-mel SQ counters.
# Usage: gpurun -- bash tools/gpu_r4_prof.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
if [ -x tools/_build/attn_probe ]; then
  timeout -k 10 120 tools/_build/attn_probe > gpurun_out/${TAG}_attn_probe.txt 2>&1 || { echo "attn probe failed"; exit 1; }
  grep -v "^  mismatch" gpurun_out/${TAG}_attn_probe.txt
fi
timeout -k 10 300 python -u bench.py --cpu-sample 0 > gpurun_out/${TAG}_base_prof.log 2>&1 || { tail -5 gpurun_out/${TAG}_base_prof.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_base_prof.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('profiled_ms_per_step'))
st=d['steps']
for k,v in sorted(d['roofline']['roles'].items(), key=lambda kv: -kv[1]['ms']): print('   ', k, round(v['ms']/st,3), v['tflops'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_kt -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-sample 0 --steps 10 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_kt.log 2>&1 || { echo "kernel trace failed"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/${TAG}_kt.log; exit 1; }
cd $GRAFT_REPO_ROOT
bash tools/pmc_kernel.sh ${TAG}_logmel lm_ --logmel --batch 128 || exit 1
