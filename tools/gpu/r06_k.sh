#!/bin/bash
# round 6, eleventh call: LayerNorm folded into the CT-Transformer's skinny QKV / w1 launches (K = 256, beyond 64 rows)
set -o pipefail
mkdir -p gpurun_out/r06k
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_punc.py tests/test_gpu_ops.py \
  > gpurun_out/r06k/tests.txt 2>&1 || { tail -30 gpurun_out/r06k/tests.txt; exit 1; }
grep -E "max \|fast|passed|failed" gpurun_out/r06k/tests.txt | tail -6
for n in 30 100 200; do
  timeout -k 10 120 python tools/punc_bench.py $n 100 fast >> gpurun_out/r06k/lat.txt 2>&1 || exit $?
done
grep "per call" gpurun_out/r06k/lat.txt
timeout -k 10 300 python tools/long_audio_prof.py > gpurun_out/r06k/long_audio.txt 2>&1 || exit $?
grep '"value"' gpurun_out/r06k/long_audio.txt | sed 's/.*"value"/"value"/'
grep -E "run_punc_host|runtime.py.*\(run\)|vad.py.*inference|punc_inference" gpurun_out/r06k/long_audio.txt
