# GPU: round-5 verification -- full GPU test suite, smoke(), headline bench, kernel profile of the headline step,
# 32k x mb2 plan under the default budget (timed-step peak)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${RUN:-r5final}
mkdir -p $D
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $D/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> $D/status.txt
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 200 python -u __graft_entry__.py smoke > $D/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $D/status.txt
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $D/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $D/status.txt
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 bench.py --steps 3 --warmup 3 > $D/prof.log 2>&1
rc=$?; echo "prof rc=$rc" >> $D/status.txt
case $rc in 124|134|137|139) exit $rc;; esac
find $D/prof -name "*kernel_trace.csv" -size +30M -delete
export HDS_BENCH_PROGRESS=1
timeout -k 10 420 python -u bench.py --seq 32768 --micro-batch 2 --steps 4 --warmup 6 --host-act-cache --act-cache-policy plan --act-cache-spill-overlap 0.8 > $D/plan_32768_mb2.log 2>&1
echo "plan32k rc=$?" >> $D/status.txt
exit 0
