#!/bin/bash
# round 6: the one-workgroup punctuation forward — punctuation tests, per-call latency (fused / multi-launch), long audio
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_punc.py \
  > $O/tests.txt 2>&1 || { grep -E "n=|PASS|FAIL|Error|error" $O/tests.txt | tail -30; exit 1; }
grep -E "n=[0-9]+:|passed|failed" $O/tests.txt | tail -14
for n in 30 100 200; do
  timeout -k 10 120 python tools/punc_bench.py $n 200 fast >> $O/lat.txt 2>&1 || exit $?
  PFM_PUNC_FUSED=0 timeout -k 10 120 python tools/punc_bench.py $n 200 fast 2>&1 | sed 's/^/multi /' >> $O/lat.txt || exit $?
done
grep "per call" $O/lat.txt
timeout -k 10 300 python tools/long_audio_prof.py > $O/long_audio.txt 2>&1 || exit $?
grep '"value"' $O/long_audio.txt | sed 's/.*"value"/"value"/' | cut -c1-200
