set -o pipefail
mkdir -p gpurun_out/r05full
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05full/gpu_suite.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r05full/bench.json 2> gpurun_out/r05full/bench.err
