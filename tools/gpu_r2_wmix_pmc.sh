set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r2_wmix.sh && bash tools/gpu_r2_pmc.sh
