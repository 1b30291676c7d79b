# Round 6: residual GEMM's half-1 rows staged during the last K-tile -- bit identity vs the previous build (ab/old.so),
# residual / guard / WavLM tests, bench A/B with roles.  Usage: gpurun -- bash tools/gpu_r6y.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lib_ident.py save /tmp/old_emb.pt --lib ab/old.so > gpurun_out/$1_ident.log 2>&1 &&
timeout -k 10 300 python -u tools/lib_ident.py check /tmp/old_emb.pt >> gpurun_out/$1_ident.log 2>&1 || { tail -12 gpurun_out/$1_ident.log; exit 1; }
grep -E "identical|DIFF" gpurun_out/$1_ident.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_guard.py tests/test_gpu_wavlm.py tests/test_gpu_kernels.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$1_tests.log 2>&1 || { tail -30 gpurun_out/$1_tests.log; exit 1; }
tail -1 gpurun_out/$1_tests.log
bash tools/gpu_ab_lib_roles.sh $1 ab/old.so 3 "oproj|ffn2" || exit 1
echo done
