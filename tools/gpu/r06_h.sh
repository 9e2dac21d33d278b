#!/bin/bash
# round 6, eighth call: pfm_run_punc_host through per-(mode, word count) HIP graphs — the punctuation tests, then
# the long-audio leg with graphs (default) and without (PFM_PUNC_GRAPH=0)
set -o pipefail
mkdir -p gpurun_out/r06h
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_punc.py \
  > gpurun_out/r06h/punc_tests.txt 2>&1 || { tail -30 gpurun_out/r06h/punc_tests.txt; exit 1; }
tail -3 gpurun_out/r06h/punc_tests.txt
timeout -k 10 300 python tools/long_audio_prof.py > gpurun_out/r06h/long_audio_graph.txt 2>&1 || exit $?
PFM_PUNC_GRAPH=0 timeout -k 10 300 python tools/long_audio_prof.py > gpurun_out/r06h/long_audio_nograph.txt 2>&1 || exit $?
grep -h '"value"' gpurun_out/r06h/long_audio_*.txt | cut -c1-40,240-400
