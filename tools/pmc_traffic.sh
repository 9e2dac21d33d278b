#!/bin/bash
# HBM traffic per bf16 GEMM launch from two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) of a short
# unsplit bench (the roofline pass's kernel set), gfx950-corrected by tools/pmc_traffic.py:
#   tools/pmc_traffic.sh <out.json>
set -o pipefail
out=$1
R=$(pwd)
mkdir -p "$R/gpurun_out/pmc_traffic"
export PFM_SUBBATCH=1 PFM_DEC_SUBBATCH=1   # the roofline pass runs single-stream (profiling on)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_traffic/f" -o run -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --exact-steps 0 --cpu-utts 0 --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 > "$R/gpurun_out/pmc_traffic/f.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_traffic/w" -o run -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --exact-steps 0 --cpu-utts 0 --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 > "$R/gpurun_out/pmc_traffic/w.log" 2>&1
rc=$?
cd "$R"
[ $rc -eq 0 ] && python tools/pmc_traffic.py gpurun_out/pmc_traffic/f/run_results.db gpurun_out/pmc_traffic/w/run_results.db "$out"
exit $rc
