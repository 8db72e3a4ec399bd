# GPU: full GPU test suite, smoke(), headline bench (round-4 verification)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${RUN:-r4full}
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $D/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> $D/status.txt
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 200 python -u __graft_entry__.py smoke > $D/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $D/status.txt
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $D/bench.log 2>&1
echo "bench rc=$?" >> $D/status.txt
