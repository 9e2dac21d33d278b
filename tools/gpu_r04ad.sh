set -o pipefail
mkdir -p gpurun_out/r04ad
timeout -k 10 900 python tools/bench_ab.py 3 "X=0" "PFM_LIB=funasr_amd/_lib/var/kvg8/libpfm_hip.so" "PFM_LIB=funasr_amd/_lib/var/kvg16/libpfm_hip.so" -- --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 --beam-steps 0 > gpurun_out/r04ad/ab.txt 2>&1
