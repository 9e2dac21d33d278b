set -o pipefail
mkdir -p gpurun_out/r04g
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_ops.py -k "ffn" > gpurun_out/r04g/tests.log 2>&1 &&
timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_sensevoice.py >> gpurun_out/r04g/tests.log 2>&1 &&
timeout -k 10 700 python tools/bench_ab.py 3 "X=0" "PFM_LIB=funasr_amd/_lib/var/pd6/libpfm_hip.so" -- --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 --beam-steps 0 > gpurun_out/r04g/ab.txt 2>&1
