#!/bin/bash
# round 6: EXACT x6 tile policy 1 (C17 wide / C16 narrow) — EXACT parity tests, then an interleaved A/B of the EXACT step
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
#timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_automodel.py \
#  -k "exact or Exact or EXACT or tile_policy or dp_shards" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
#tail -2 $O/tests.txt
timeout -k 10 1000 python tools/bench_ab.py 2 "PFM_X6_POLICY=0" "PFM_X6_POLICY=2" "PFM_X6_POLICY=3" -- --mode exact --steps 3 --warmup 1 \
  --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 --beam-steps 0 --generate 0 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
