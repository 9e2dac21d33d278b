#!/bin/bash
# rocprofv3 kernel trace of the DEFAULT bench command (the one whose JSON line is reported), run on the
# GPU box from the repo root: tools/profile_default.sh <out-name>
# -> gpurun_out/<out-name>/{run_results.db, bench.log, stats.csv, summary.md}
set -o pipefail
name=$1
R=$(pwd)
mkdir -p "$R/gpurun_out/$name"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$name" -o run -- \
  python3 "$R/bench.py" > "$R/gpurun_out/$name/bench.log" 2>&1
rc=$?
cd "$R"
[ $rc -eq 0 ] && python tools/rocpd_summary.py "gpurun_out/$name/run_results.db" "gpurun_out/$name/stats.csv" \
  "gpurun_out/$name/bench.log" 2 5 > "gpurun_out/$name/summary.md"
exit $rc
