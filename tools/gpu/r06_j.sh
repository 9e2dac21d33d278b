#!/bin/bash
# round 6, tenth call: small-head attention with 16 key lanes per query row — punctuation tests, per-call latency
# at 30 / 100 / 200 words (new vs the previous library), the long-audio leg
set -o pipefail
mkdir -p gpurun_out/r06j
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_punc.py \
  > gpurun_out/r06j/punc_tests.txt 2>&1 || { tail -30 gpurun_out/r06j/punc_tests.txt; exit 1; }
tail -2 gpurun_out/r06j/punc_tests.txt
for n in 30 100 200; do
  for m in fast exact; do
    timeout -k 10 120 python tools/punc_bench.py $n 100 $m >> gpurun_out/r06j/lat.txt 2>&1 || exit $?
    PFM_LIB=$(pwd)/abvar/puncold/libpfm_hip.so timeout -k 10 120 python tools/punc_bench.py $n 100 $m 2>&1 | sed 's/^/old /' >> gpurun_out/r06j/lat.txt || exit $?
  done
done
grep "per call" gpurun_out/r06j/lat.txt
timeout -k 10 300 python tools/long_audio_prof.py > gpurun_out/r06j/long_audio.txt 2>&1 || exit $?
grep '"value"' gpurun_out/r06j/long_audio.txt | sed 's/.*"value"/"value"/'
grep -E "run_punc_host|runtime.py.*\(run\)|vad.py.*inference" gpurun_out/r06j/long_audio.txt
