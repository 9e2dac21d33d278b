set -o pipefail
timeout -k 10 300 python bench.py --exact-steps 0 --cpu-utts 0 --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 --beam-steps 0 > gpurun_out/r05_bench_fastonly.json 2> gpurun_out/r05_bench_fastonly.err &&
bash tools/profile_fast.sh r05a_fast &&
PFM_SUBBATCH=1 PFM_DEC_SUBBATCH=1 bash tools/profile_fast.sh r05a_fast_sb1
