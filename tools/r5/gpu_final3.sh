# GPU: final verification of the round-5 tree (after the optimizer-offload changes), then mb10 host-step at ratio 0.3
cd $GRAFT_REPO_ROOT
RUN=r5final3 bash tools/r5/gpu_full.sh || exit $?
O=gpurun_out/r5final3
export HDS_BENCH_PROGRESS=1
timeout -k 10 330 python -u bench.py --micro-batch 10 --steps 4 --warmup 3 --offload-opt-states --offload-states-ratio 0.3 --offload-states-host-step > $O/mb10_offstates_hoststep_0.3.log 2>&1
echo "mb10 0.3 rc=$?" >> $O/status.txt
exit 0
