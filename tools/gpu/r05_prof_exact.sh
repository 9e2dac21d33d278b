#!/bin/bash
# rocprofv3 kernel trace of the EXACT (x6) leg alone: bench.py --mode exact
set -o pipefail
R=$(pwd); name=r05_exact
mkdir -p "$R/gpurun_out/$name"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$name" -o run -- \
  python3 "$R/bench.py" --mode exact --steps 2 --warmup 1 --exact-steps 0 --cpu-utts 0 --sv-steps 0 --stream-chunks 0 \
  --punc-steps 0 --long-audio-s 0 --beam-steps 0 > "$R/gpurun_out/$name/bench.log" 2>&1
