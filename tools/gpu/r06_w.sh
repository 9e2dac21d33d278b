#!/bin/bash
# round 6: punctuation launch folds (LN1 in the embedding, FSMN in the attention, after_norm in the head)
set -o pipefail
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_punc.py tests/test_gpu_vad.py \
  tests/test_gpu_ops.py -k "punc or vad or attention" > $O/tests.txt 2>&1 || { grep -E "n=|FAIL|Error|error" $O/tests.txt | tail -30; exit 1; }
grep -E "folded|passed|failed" $O/tests.txt | tail -10
for n in 30 100 200; do
  timeout -k 10 120 python tools/punc_bench.py $n 200 fast >> $O/lat.txt 2>&1 || exit $?
  PFM_PUNC_FOLD=0 timeout -k 10 120 python tools/punc_bench.py $n 200 fast 2>&1 | sed 's/^/unfolded /' >> $O/lat.txt || exit $?
done
grep "per call" $O/lat.txt
timeout -k 10 300 python tools/long_audio_prof.py > $O/long_audio.txt 2>&1 || exit $?
grep '"value"' $O/long_audio.txt | sed 's/.*"value"/"value"/' | cut -c1-200
