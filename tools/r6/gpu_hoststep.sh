# Async host step (round 6): GPU tests of the host-step tails, then mb10 host-step A/B (async vs sync) on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6host
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_host_tier_gpu.py -k "host_step or twin" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
R=${RATIO:-0.35}
timeout -k 10 480 python bench.py --steps 8 --warmup 3 --micro-batch 10 --offload-opt-states --offload-states-ratio $R --offload-states-host-step > $O/mb10_async_$R.json 2> $O/mb10_async_$R.err || { echo async bench failed; tail -30 $O/mb10_async_$R.err; exit 1; }
python -c "import json;d=json.loads([l for l in open('$O/mb10_async_$R.json') if l.startswith('{')][-1]);print('async', d['value'], d['extra']['peak_mem_gib'], d['extra'].get('offload_opt_states'))"
HDS_ASYNC_HOST_STEP=0 timeout -k 10 480 python bench.py --steps 8 --warmup 3 --micro-batch 10 --offload-opt-states --offload-states-ratio $R --offload-states-host-step > $O/mb10_sync_$R.json 2> $O/mb10_sync_$R.err || { echo sync bench failed; tail -30 $O/mb10_sync_$R.err; exit 1; }
python -c "import json;d=json.loads([l for l in open('$O/mb10_sync_$R.json') if l.startswith('{')][-1]);print('sync', d['value'], d['extra']['peak_mem_gib'])"
