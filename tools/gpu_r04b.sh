set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 120 ./tools/ffn2_bench 16000 32000 > gpurun_out/r04b/ffn2_bench.txt 2>&1 &&
FFN2_ONLY=4 bash tools/pmc_ffn2.sh m4 32000 &&
bash tools/profile_fast.sh r04b_fast &&
timeout -k 10 600 python bench.py > gpurun_out/r04b/bench.json 2> gpurun_out/r04b/bench.err
