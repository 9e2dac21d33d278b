#!/bin/bash
# kernel trace of a short fast-mode bench (no side legs) under the current knobs -> gpurun_out/k2prof/
R=$(pwd)
mkdir -p "$R/gpurun_out/k2prof"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/k2prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --exact-steps 0 --cpu-utts 0 --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 > "$R/gpurun_out/k2prof/bench.log" 2>&1
rc=$?
cd "$R"
f=$(ls gpurun_out/k2prof/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && head -25 "$f"
exit $rc
