# Quick GPU check: the GPU tests selected by -k, then bench lines for the given dtypes (WavLM-base,
# per-role ms/step printed).  Usage: gpurun -- bash tools/gpu_quick.sh "<pytest -k>" <tag> [dtype ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K=${1:-}
TAG=${2:-quick}
shift 2
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "$K" > $O/gputests.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|rel-L2" $O/gputests.log | tail -60
  tail -3 $O/gputests.log
  [ $rc -ne 0 ] && exit $rc
fi
for dt in "$@"; do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --dtype $dt > $O/bench_$dt.log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads(open('$O/bench_$dt.log').read().strip().splitlines()[-1]); print('$dt', d['value'], d['ms_per_step'], d['roofline']['frac'], {k:(round(v['ms']/d['steps'],3),v['tflops']) for k,v in d['roofline']['roles'].items()})"
done
