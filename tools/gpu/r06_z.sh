#!/bin/bash
# round 6: the M > 64 skinny GEMM with 2 / 4 column strips per workgroup — op tests, streaming tests, 64-stream latency
set -o pipefail
O=gpurun_out/r06z
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_streaming.py \
  tests/test_gpu_stream_beam.py -k "skinny or stream or gemm_bf16" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 0 1; do
for a in "PFM_SKINNY_NS=0" "PFM_SKINNY_NS=1" "PFM_SKINNY_NS=2"; do
  env $a timeout -k 10 120 python tools/stream_prof.py 30 64 2>&1 | sed "s/^/$a /" >> $O/lat.txt || exit $?
done
done
for a in "PFM_SKINNY_NS=0" "PFM_SKINNY_NS=1"; do
  env $a timeout -k 10 120 python tools/stream_prof.py 30 16 2>&1 | sed "s/^/$a S=16 /" >> $O/lat.txt || exit $?
  env $a timeout -k 10 120 python tools/stream_prof.py 30 1 2>&1 | sed "s/^/$a S=1 /" >> $O/lat.txt || exit $?
done
cat $O/lat.txt | grep "per chunk"
