#!/bin/bash
# rocprofv3 kernel trace of the fast bench (run on the GPU box from the repo root):
#   tools/profile_bench.sh <out-name> [bench args...]
# writes gpurun_out/<out-name>/run_results.db (summarise with tools/rocpd_summary.py)
set -o pipefail
name=$1; shift
R=$(pwd)
mkdir -p "$R/gpurun_out/$name"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$name" -o run -- \
  python3 "$R/bench.py" --exact-steps 0 --cpu-utts 0 "$@" > "$R/gpurun_out/$name/bench.log" 2>&1
rc=$?
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' "$R/gpurun_out/$name/bench.log"
exit $rc
