#!/bin/bash
# round 6, twelfth call: punctuation graphs off by default — punctuation tests, long-audio leg x2 (eager; graphs)
set -o pipefail
mkdir -p gpurun_out/r06l
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_punc.py \
  > gpurun_out/r06l/tests.txt 2>&1 || { tail -30 gpurun_out/r06l/tests.txt; exit 1; }
tail -1 gpurun_out/r06l/tests.txt
timeout -k 10 300 python tools/long_audio_prof.py > gpurun_out/r06l/long_audio.txt 2>&1 || exit $?
PFM_PUNC_GRAPH=1 timeout -k 10 300 python tools/long_audio_prof.py > gpurun_out/r06l/long_audio_graph.txt 2>&1 || exit $?
grep '"value"' gpurun_out/r06l/long_audio.txt gpurun_out/r06l/long_audio_graph.txt | sed 's/{.*"value"/"value"/'
