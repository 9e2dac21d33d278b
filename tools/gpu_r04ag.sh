set -o pipefail
mkdir -p gpurun_out/r04ag
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ag/gpu_suite.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r04ag/bench.json 2> gpurun_out/r04ag/bench.err
