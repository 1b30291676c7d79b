set -o pipefail
cd $GRAFT_REPO_ROOT
make -C stuttering-speech-representation_amd/csrc -j16 > gpurun_out/make.log 2>&1 &&
timeout -k 10 300 python -m pytest tests/test_gpu_ingest.py tests/test_gpu_augment.py -q -x -s > gpurun_out/ingest_tests.log 2>&1
