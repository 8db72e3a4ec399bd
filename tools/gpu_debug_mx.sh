set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/debug_mx.py > gpurun_out/debug_mx.log 2>&1
