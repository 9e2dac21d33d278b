#!/bin/bash
# round 6: kernel trace of one streaming stream (the per-chunk launch chain)
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
R=$(pwd)
timeout -k 10 120 python tools/stream_prof.py 50 > $O/lat.txt 2>&1 || exit $?
cat $O/lat.txt | tail -1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/tools/stream_prof.py 50 > $R/$O/prof.log 2>&1) || exit $?
tail -1 $O/prof.log
