#!/bin/bash
# rocprofv3 kernel traces of the EXACT leg alone, one utterance group (PFM_SUBBATCH=1: no stream concurrency, so every
# kernel's duration is its own), hipBLASLt route on / off
set -o pipefail
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for a in 1 0; do
  name=r05_exact_sb1_blas$a
  mkdir -p "$R/gpurun_out/$name"
  PFM_SUBBATCH=1 PFM_EXACT_BLAS=$a timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$name" -o run -- \
    python3 "$R/bench.py" --mode exact --steps 2 --warmup 1 --exact-steps 0 --cpu-utts 0 --sv-steps 0 --stream-chunks 0 \
    --punc-steps 0 --long-audio-s 0 --beam-steps 0 > "$R/gpurun_out/$name/bench.log" 2>&1 || exit $?
done
