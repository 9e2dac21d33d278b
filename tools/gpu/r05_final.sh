#!/bin/bash
# full GPU suite, the default bench line, and the fast-leg kernel trace (tools/profile_fast.sh)
set -o pipefail
mkdir -p gpurun_out/r05x
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r05x/gpu_suite.log 2>&1
echo "suite rc=$?" >> gpurun_out/r05x/gpu_suite.log
timeout -k 10 400 python bench.py > gpurun_out/r05x/bench.json 2> gpurun_out/r05x/bench.err || exit 1
bash tools/profile_fast.sh r05x_fast
