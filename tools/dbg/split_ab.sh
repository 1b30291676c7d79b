cd $GRAFT_REPO_ROOT
timeout -k 10 250 python -u tools/dbg/gemm_race.py > gpurun_out/gemm_race.log 2>&1; echo "race rc=$?"
tail -6 gpurun_out/gemm_race.log
for r in 1 2; do for sp in 1 2 4; do
timeout -k 10 200 python -u bench.py --cpu-sample 0 --no-profile --steps 20 --warmup 5 --split $sp > gpurun_out/split_$sp.log 2>&1 || exit $?
echo "split $sp: $(tail -1 gpurun_out/split_$sp.log | cut -c1-140)"
done; done
