cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 tools/_build/gemm8_probe > gpurun_out/r4g_gemm_probe.txt 2>&1 || { echo probe failed; tail -3 gpurun_out/r4g_gemm_probe.txt; exit 1; }
grep -A5 "conv1" gpurun_out/r4g_gemm_probe.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -k "whisper" > gpurun_out/r4g_tests.log 2>&1; rc=$?
grep -E "rel-L2|rel |passed|failed|FAILED" gpurun_out/r4g_tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4_lines.sh r4g wlv2_bf16 wlv2_fp8 wlv2_fp16x3
