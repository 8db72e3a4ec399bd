# GPU: kernel trace of the mb10 host-step state offload (how much of the step the GPU idles through the host Adam)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5aw
mkdir -p $O
export HDS_BENCH_PROGRESS=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --micro-batch 10 --steps 2 --warmup 2 --offload-opt-states --offload-states-ratio 0.35 --offload-states-host-step > $O/prof.log 2>&1
echo "prof rc=$?" >> $O/status.txt
find $O/prof -name "*kernel_trace.csv" -size +30M -delete
exit 0
