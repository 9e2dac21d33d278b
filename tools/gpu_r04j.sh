set -o pipefail
mkdir -p gpurun_out/r04j
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04j/gpu_suite.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r04j/bench.json 2> gpurun_out/r04j/bench.err &&
bash tools/profile_fast.sh r04j_fast &&
bash tools/pmc_bench.sh gpurun_out/r04j/pmc_bench.json > gpurun_out/r04j/pmc_bench.log 2>&1 &&
timeout -k 10 60 ./tools/beam_bench 64 230 500 10 > gpurun_out/r04j/beam.txt 2>&1 &&
timeout -k 10 120 python tools/stream_prof.py --streams 1 --chunks 50 > gpurun_out/r04j/stream1.txt 2>&1
