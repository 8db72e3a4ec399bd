# round-6 final verification: GPU suite, smoke, headline bench, rocprof step table of the headline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r6final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 || { echo "suite failed rc=$?"; tail -40 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
grep '^{' $O/bench.json | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 2 > $O/prof_bench.log 2>&1 || { echo prof failed; tail -20 $O/prof_bench.log; exit 1; }
DB=$(find $O/prof -name "*.db" | head -1)
python tools/r5/step_kernels.py $DB $O/headline_kernels.txt | head -12
find $O/prof -name "*.db" -size +30M -delete
