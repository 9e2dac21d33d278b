#!/bin/bash
# round 6: 64 concurrent streams — per-chunk latency (skinny policy default vs tiled everywhere) and a kernel trace
set -o pipefail
O=gpurun_out/r06y
mkdir -p $O
R=$(pwd)
for a in "X=0" "PFM_GEMM_SKINNY=0"; do
  env $a timeout -k 10 120 python tools/stream_prof.py 30 64 2>&1 | sed "s/^/$a /" >> $O/lat.txt || exit $?
done
cat $O/lat.txt | grep "per chunk"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/tools/stream_prof.py 30 64 > $R/$O/prof.log 2>&1) || exit $?
