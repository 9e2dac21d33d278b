set -o pipefail
mkdir -p gpurun_out/r04final
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04final/gpu_suite.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r04final/bench.json 2> gpurun_out/r04final/bench.err &&
timeout -k 10 120 python tools/stream_prof.py --streams 1 --chunks 50 > gpurun_out/r04final/stream1.txt 2>&1 &&
timeout -k 10 120 python tools/stream_prof.py --streams 64 --chunks 20 > gpurun_out/r04final/stream64.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04final/sprof -o run -- python3 $GRAFT_REPO_ROOT/tools/stream_prof.py --streams 1 --chunks 20 > $GRAFT_REPO_ROOT/gpurun_out/r04final/sprof.log 2>&1
