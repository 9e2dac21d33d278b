#!/bin/bash
# round 6, ninth call: pfm_run_punc_host per-call latency (graph / eager, fast / exact) and its kernel trace
set -o pipefail
mkdir -p gpurun_out/r06i
R=$(pwd)
timeout -k 10 120 python tools/punc_bench.py 30 300 fast > gpurun_out/r06i/lat.txt 2>&1 || exit $?
PFM_PUNC_GRAPH=0 timeout -k 10 120 python tools/punc_bench.py 30 300 fast >> gpurun_out/r06i/lat.txt 2>&1 || exit $?
timeout -k 10 120 python tools/punc_bench.py 30 300 exact >> gpurun_out/r06i/lat.txt 2>&1 || exit $?
cat gpurun_out/r06i/lat.txt | grep "per call"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r06i/prof -o run --output-format csv -- python3 $R/tools/punc_bench.py 30 100 fast > $R/gpurun_out/r06i/prof.log 2>&1) || exit $?
find gpurun_out/r06i/prof -name "*kernel_stats.csv" | head -2
