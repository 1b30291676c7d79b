cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 120 --timeout-method thread > gpurun_out/kern_tests.log 2>&1; tail -5 gpurun_out/kern_tests.log
timeout -k 10 300 python -u tools/nan_probe.py > gpurun_out/nan_probe.txt 2>&1; grep -v "^  File\|^    " gpurun_out/nan_probe.txt | tail -12
