set -o pipefail
mkdir -p gpurun_out/r04af
P=funasr_amd/_lib/var/prev/libpfm_hip.so
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04af/tests.log 2>&1 &&
timeout -k 10 600 python tools/bench_ab.py 3 "X=0" "PFM_LIB=$P" -- --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 --beam-steps 0 > gpurun_out/r04af/ab.txt 2>&1
