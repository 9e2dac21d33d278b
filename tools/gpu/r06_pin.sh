#!/bin/bash
# round 6: pinned staging for waveform uploads — frontend / VAD / streaming / AutoModel tests, long audio, VAD pass
set -o pipefail
O=gpurun_out/r06pin
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_frontend.py tests/test_gpu_vad.py \
  tests/test_gpu_streaming.py tests/test_gpu_automodel.py tests/test_gpu_sensevoice.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python tools/vad_prof.py > $O/vad.txt 2>&1 || exit $?
grep "VAD pass" $O/vad.txt
timeout -k 10 300 python tools/long_audio_prof.py > $O/la.txt 2>&1 || exit $?
grep '"value"' $O/la.txt | head -1 | sed 's/.*"value"/"value"/' | cut -c1-110
