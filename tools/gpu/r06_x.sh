#!/bin/bash
# round 6: EXACT step — one encoder group with the 8-phase tile everywhere vs the default dispatch
set -o pipefail
O=gpurun_out/r06x
mkdir -p $O
timeout -k 10 1100 python tools/bench_ab.py 2 "X=0" "PFM_SUBBATCH=1" "PFM_SUBBATCH=1 PFM_GEMM_CFG=17" "PFM_GEMM_CFG=17" -- --mode exact --steps 3 --warmup 1 \
  --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 --beam-steps 0 --generate 0 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
