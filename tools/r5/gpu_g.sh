# GPU: the summed-residual boundary at 128k (one saved tensor per block; round 4: 5,322 tok/s) and 320k without
# --act-cache-host-gib (round 4 needed 225 GiB pinned)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${R5G_OUT:-r5g}; O=gpurun_out/$(basename $O)
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
export HDS_BENCH_PROGRESS=1
run timeout -k 10 400 python -u bench.py --seq 131072 --micro-batch 1 --steps 3 --warmup 2 --host-act-cache --act-cache-policy ckpt_offload > $O/ckoff128k.log 2>&1
run timeout -k 10 600 python -u bench.py --seq 327680 --micro-batch 1 --steps 1 --warmup 2 --host-act-cache --act-cache-policy ckpt_offload > $O/ckoff320k.log 2>&1
exit 0
