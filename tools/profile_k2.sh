#!/bin/bash
# kernel trace of a short fast-mode bench (no side legs) under the current knobs -> gpurun_out/${PROF_TAG:-k2prof}/
R=$(pwd)
D="$R/gpurun_out/${PROF_TAG:-k2prof}"
mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$D" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --exact-steps 0 --cpu-utts 0 --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 > "$D/bench.log" 2>&1
rc=$?
cd "$R"
f=$(ls "$D"/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && head -12 "$f" | cut -c1-160
exit $rc
