#!/bin/bash
# rocprofv3 kernel trace of the fast (headline) leg of bench.py alone (no exact / SenseVoice / streaming /
# punctuation / long-audio / CPU legs), run on the GPU box from the repo root:
#   tools/profile_fast.sh <out-name> [extra bench args]
# -> gpurun_out/<out-name>/{run_results.db, bench.log, stats.csv, summary.md}
# Set PFM_SUBBATCH=1 PFM_DEC_SUBBATCH=1 in the environment for a trace without concurrent streams (the kernel
# trace serialises them), whose kernel time per call is the step.
set -o pipefail
name=$1; shift
R=$(pwd)
mkdir -p "$R/gpurun_out/$name"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$name" -o run -- \
  python3 "$R/bench.py" --steps 5 --warmup 2 --exact-steps 0 --cpu-utts 0 --sv-steps 0 --stream-chunks 0 \
  --punc-steps 0 --long-audio-s 0 --beam-steps 0 "$@" > "$R/gpurun_out/$name/bench.log" 2>&1
rc=$?
cd "$R"
[ $rc -eq 0 ] && python tools/rocpd_summary.py "gpurun_out/$name/run_results.db" "gpurun_out/$name/stats.csv" \
  "gpurun_out/$name/bench.log" 2 5 > "gpurun_out/$name/summary.md"
exit $rc
