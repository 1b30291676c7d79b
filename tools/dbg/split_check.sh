cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wavlm or ragged or corpus or kernels or dropin" > gpurun_out/split_tests.log 2>&1; rc=$?
tail -2 gpurun_out/split_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
 for o in 1 0; do
  timeout -k 10 200 python -u bench.py --cpu-sample 0 --no-profile --steps 20 --warmup 5 --opt no_split=$o > gpurun_out/sp_$o.log 2>&1 || exit $?
  echo "no_split=$o $(python3 -c "import json; d=json.loads(open('gpurun_out/sp_$o.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
 done
done
timeout -k 10 200 python -u bench.py --cpu-sample 0 > gpurun_out/sp_prof.log 2>&1 || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/sp_prof.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['profiled_ms_per_step'], {k:(round(v['ms']/d['steps'],3),v['tflops']) for k,v in d['roofline']['roles'].items()})"
