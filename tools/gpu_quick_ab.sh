set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_quick.sh "wavlm or dropin or corpus or augment" && bash tools/ab.sh ab/base.so 3
