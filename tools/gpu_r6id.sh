# Round 6: whole-model bit identity of the gemm_4phase schedules (tools/phase_model_ab.py) and the in-model test
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/phase_model_ab.py > gpurun_out/$1_ident.log 2>&1 || { tail -20 gpurun_out/$1_ident.log; exit 1; }
grep -E "identical|DIFF" gpurun_out/$1_ident.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -k schedules --timeout 200 --timeout-method thread > gpurun_out/$1_tests.log 2>&1 || { tail -20 gpurun_out/$1_tests.log; exit 1; }
tail -1 gpurun_out/$1_tests.log
