set -o pipefail
mkdir -p gpurun_out/r05fb
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py tests/test_gpu_automodel.py tests/test_gpu_vad.py tests/test_gpu_streaming.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r05fb/tests.log 2>&1
