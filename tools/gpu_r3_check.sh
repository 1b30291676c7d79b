# Round-3 quick check: the GPU tests selected by -k (default: all), then the default bench line with
# per-role ms/step and a corpus line (host-staged).  Usage: gpurun -- bash tools/gpu_r3_check.sh "<pytest -k>" <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K=${1:-}
TAG=${2:-r3}
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${KA[@]}" > $O/gputests.log 2>&1
rc=$?
tail -3 $O/gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --cpu-sample 0 > $O/bench.log 2>&1 || exit $?
python3 -c "
import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k:(round(v['ms']/d['steps'],3),v['tflops']) for k,v in d['roofline']['roles'].items()})"
timeout -k 10 300 python -u bench.py --corpus 20000 --cpu-sample 0 > $O/corpus.log 2>&1 || exit $?
tail -1 $O/corpus.log | cut -c1-300
