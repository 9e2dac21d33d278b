#!/bin/bash
# round 6: punctuation graphs over 16-word buckets (fast mode) — tests, per-call latency, long audio (graphs on / off)
set -o pipefail
O=gpurun_out/r06pg
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_punc.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for n in 30 100 200; do
  PFM_PUNC_GRAPH=1 timeout -k 10 120 python tools/punc_bench.py $n 200 fast >> $O/lat.txt 2>&1 || exit $?
  PFM_PUNC_GRAPH=0 timeout -k 10 120 python tools/punc_bench.py $n 200 fast >> $O/lat.txt 2>&1 || exit $?
done
grep "per call" $O/lat.txt
for r in 0 1; do
  PFM_PUNC_GRAPH=1 timeout -k 10 300 python tools/long_audio_prof.py > $O/la_g$r.txt 2>&1 || exit $?
  PFM_PUNC_GRAPH=0 timeout -k 10 300 python tools/long_audio_prof.py > $O/la_e$r.txt 2>&1 || exit $?
done
for f in $O/la_*.txt; do echo $f; grep '"value"' $f | head -1 | sed 's/.*"value"/"value"/' | cut -c1-110; done
