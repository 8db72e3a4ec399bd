# GPU: final verification after the round-5 forward / dQ DMA changes
cd $GRAFT_REPO_ROOT
RUN=r5final2 bash tools/r5/gpu_full.sh
