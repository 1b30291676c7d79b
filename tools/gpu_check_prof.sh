# gpu_check_ab.sh + one profiled bench run printing per-role ms/step.  Usage: gpurun -- bash tools/gpu_check_prof.sh "<pytest -k>" [rounds]
cd $GRAFT_REPO_ROOT && bash tools/gpu_check_ab.sh "$1" ${2:-2} && timeout -k 10 300 python -u bench.py --cpu-sample 0 > gpurun_out/bench_prof.log 2>&1 && python3 -c "
import json; d=json.loads(open('gpurun_out/bench_prof.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], {k:(round(v['ms']/d['steps'],3),v['tflops']) for k,v in d['roofline']['roles'].items()})"
