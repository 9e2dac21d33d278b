set -o pipefail
mkdir -p gpurun_out/sub
timeout -k 10 900 python tools/bench_ab.py 3 "X=0" "PFM_SUBBATCH=1" "PFM_DEC_SUBBATCH=1" "PFM_SUBBATCH=1 PFM_DEC_SUBBATCH=1" -- --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 --beam-steps 0 > gpurun_out/sub/ab.txt 2>&1
