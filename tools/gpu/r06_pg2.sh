#!/bin/bash
# round 6: bucketed punctuation graphs as the fast-mode default — punctuation / VAD pipeline / AutoModel tests, long audio
set -o pipefail
O=gpurun_out/r06pg2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_punc.py tests/test_gpu_vad.py \
  tests/test_gpu_automodel.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python tools/long_audio_prof.py > $O/la.txt 2>&1 || exit $?
grep '"value"' $O/la.txt | head -1 | sed 's/.*"value"/"value"/' | cut -c1-110
