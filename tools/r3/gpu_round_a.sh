# GPU: copy-engine probe, then FlashAttention timings + PMC at the bench shape
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/r3/gpu_copy_probe.sh || exit 1
bash tools/r3/gpu_fa_pmc.sh || exit 1
