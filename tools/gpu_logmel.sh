# Log-mel A/B: GPU log-mel tests, bench --logmel for the 4-frame kernel and the round-2 kernel
# (logmel_v1=1), and a rocprofv3 kernel-stats pass of the default.  Usage: gpurun -- bash tools/gpu_logmel.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-logmel}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "logmel or whisper_tiny" > $O/gputests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|diff|err" $O/gputests.log | tail -20; [ $rc -ne 0 ] && exit $rc
for v in 0 1; do
  timeout -k 10 200 python -u bench.py --logmel --steps 20 --warmup 5 --opt logmel_v1=$v > $O/bench_v$v.log 2>&1 || exit $?
  tail -1 $O/bench_v$v.log | cut -c1-400
done
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --logmel --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/bench_prof.log 2>&1) || exit $?
python3 - <<P
import csv,glob
f=glob.glob('$O/kt/**/kt_kernel_stats.csv',recursive=True)+glob.glob('$O/kt/kt_kernel_stats.csv')
for r in csv.DictReader(open(f[0])): print(r['Name'][:60], r['Calls'], r['AverageNs'])
P
