#!/bin/bash
# rocprofv3 kernel statistics of the fast-mode bench leg under one knob setting, run on the GPU box from the repo
# root: tools/prof_ab.sh <out-name> "<VAR=val ...>" [extra bench args]  -> gpurun_out/<out-name>/run_kernel_stats.csv
set -o pipefail
name=$1
R=$(pwd)
mkdir -p "$R/gpurun_out/$name"
for kv in $2; do export "$kv"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$name" -o run -- \
  python3 "$R/bench.py" --exact-steps 0 --cpu-utts 0 --beam-steps 0 --steps 5 --warmup 2 "${@:3}" > "$R/gpurun_out/$name/bench.log" 2>&1
rc=$?
for f in $(find "$R/gpurun_out/$name" -name "*kernel_trace.csv"); do python3 "$R/tools/trace_busy.py" "$f" > "$R/gpurun_out/$name/busy.txt" 2>&1; rm -f "$f"; done
exit $rc
