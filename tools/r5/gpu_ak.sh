# GPU: block-A microbenchmark (S MFMAs + K reads in isolation, one wave per SIMD)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5al
mkdir -p $O
timeout -k 10 120 ./tools/r5/mfma_lds_micro > $O/micro.log 2>&1 || exit 1
cat $O/micro.log
