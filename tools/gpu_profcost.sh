set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python bench.py --cpu-sample 0 > gpurun_out/prof_on_$i.log 2>&1 &&
timeout -k 10 200 python bench.py --cpu-sample 0 --no-profile > gpurun_out/prof_off_$i.log 2>&1 || exit 1
done
