set -o pipefail
mkdir -p gpurun_out/r04e
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_beam.py tests/test_gpu_stream_beam.py > gpurun_out/r04e/tests.log 2>&1 &&
timeout -k 10 300 $T tests/test_gpu_ops.py -k "attention or fsmn" >> gpurun_out/r04e/tests.log 2>&1 &&
timeout -k 10 400 $T tests/test_gpu_parity.py >> gpurun_out/r04e/tests.log 2>&1 &&
timeout -k 10 60 ./tools/beam_bench_prev 64 230 500 10 > gpurun_out/r04e/beam.txt 2>&1 &&
timeout -k 10 60 ./tools/beam_bench 64 230 500 10 >> gpurun_out/r04e/beam.txt 2>&1 &&
timeout -k 10 500 python tools/bench_ab.py 2 "X=0" "PFM_LIB=funasr_amd/_lib/var/prev/libpfm_hip.so" -- --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 --exact-steps 0 > gpurun_out/r04e/ab.txt 2>&1
