# round 6 batch 2: qkv TunableOp, host-step auto ratio, traced mb10 async host step (GPU idle), host-cache controls
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6b2
mkdir -p $O tuning_r6
PYTORCH_TUNABLEOP_FILENAME=tuning_r6/tunableop_results%d.csv timeout -k 10 240 python tools/r6/tune_qkv.py --o > $O/tune_qkv.log 2>&1 || { echo tune failed; tail -20 $O/tune_qkv.log; }
grep -E "tflops|wrote" $O/tune_qkv.log
cp tuning_r6/tunableop_results0.csv $O/ 2>/dev/null
timeout -k 10 480 python bench.py --steps 6 --warmup 3 --micro-batch 10 --offload-opt-states --offload-states-ratio auto --offload-states-host-step > $O/mb10_auto.json 2> $O/mb10_auto.err || { echo auto bench failed; tail -30 $O/mb10_auto.err; exit 1; }
python -c "import json;d=json.loads([l for l in open('$O/mb10_auto.json') if l.startswith('{')][-1]);print('auto', d['value'], d['extra']['peak_mem_gib'], d['extra']['offload_opt_states'].get('auto_ratio'))"
timeout -k 10 480 rocprofv3 --kernel-trace --stats -d $O/prof -o mb10 -- python3 bench.py --steps 2 --warmup 2 --micro-batch 10 --offload-opt-states --offload-states-ratio 0.35 --offload-states-host-step > $O/mb10_trace.log 2>&1 || { echo trace failed; tail -20 $O/mb10_trace.log; exit 1; }
DB=$(find $O/prof -name "*.db" | head -1)
python tools/r5/step_kernels.py $DB $O/mb10_async_step_kernels.txt | head -8
find $O/prof -name "*.db" -size +30M -delete
bash tools/r6/gpu_controls.sh
