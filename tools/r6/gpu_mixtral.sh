# Mixtral-8x7B at 8 of 32 layers, ZeRO-3 on one MI355X (round 6, VERDICT r5 Next 8 evidence): throughput + the
# kernel table of one step (expert GEMMs' share and rate)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6mx${TAG:-}
mkdir -p $O
MB=${MB:-4}
timeout -k 10 500 python -u bench.py --model mixtral-8x7b --layers 8 --micro-batch $MB --steps 4 --warmup 2 > $O/mixtral_l8_mb$MB.json 2> $O/mixtral_l8_mb$MB.err || { echo bench failed; tail -20 $O/mixtral_l8_mb$MB.err; exit 1; }
grep '^{' $O/mixtral_l8_mb$MB.json | cut -c1-600
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --model mixtral-8x7b --layers 8 --micro-batch $MB --steps 2 --warmup 2 > $O/prof_bench.log 2>&1 || { echo prof failed; tail -20 $O/prof_bench.log; exit 1; }
DB=$(find $O/prof -name "*.db" | head -1)
python tools/r5/step_kernels.py $DB $O/mixtral_kernels_mb$MB.txt | head -16
find $O/prof -name "*.db" -size +30M -delete
