#!/bin/bash
# end-of-round tree: full GPU suite, the default bench line, and the fast-leg kernel trace (tools/profile_fast.sh)
set -o pipefail
mkdir -p gpurun_out/r05y
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05y/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc" >> gpurun_out/r05y/gpu_suite.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/r05y/bench.json 2> gpurun_out/r05y/bench.err || exit 1
bash tools/profile_fast.sh r05y_fast
