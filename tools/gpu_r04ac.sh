set -o pipefail
mkdir -p gpurun_out/r04ac
P=funasr_amd/_lib/var/prev/libpfm_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ac/tests.log 2>&1 &&
timeout -k 10 600 python tools/bench_ab.py 3 "X=0" "PFM_LIB=$P" -- --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 --beam-steps 0 > gpurun_out/r04ac/ab.txt 2>&1
