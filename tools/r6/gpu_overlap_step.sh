# Overlapped ZeRO-3 step (the fused Adam per unit on a side stream under the next forward): the bit-exactness GPU
# test, then the headline with / without it interleaved on one box, then a kernel trace of the overlapped headline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6ovl
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_overlap_step_gpu.py tests/test_host_tier_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for t in 1 0 1 0; do
  HDS_OVERLAP_STEP=$t timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_ovl${t}_$RANDOM.json 2> $O/err_$t.log || { echo "bench $t failed"; tail -20 $O/err_$t.log; exit 1; }
done
for f in $O/bench_ovl*.json; do python -c "import json;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f', d['value'])"; done
