set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_prof.sh r18_b128 resnet 18 128 || exit $?
bash tools/gpu_prof.sh r50_b256 resnet 50 256 || exit $?
