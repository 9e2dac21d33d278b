set -o pipefail
mkdir -p gpurun_out/r04x
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04x/sprof -o run -- python3 $GRAFT_REPO_ROOT/tools/stream_prof.py --streams 1 --chunks 20 > $GRAFT_REPO_ROOT/gpurun_out/r04x/sprof.log 2>&1
