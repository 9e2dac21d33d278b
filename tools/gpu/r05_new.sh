set -o pipefail
mkdir -p gpurun_out/r05new
timeout -k 10 400 python -u -m pytest tests/test_gpu_output_dir.py tests/test_gpu_automodel.py tests/test_gpu_beam.py tests/test_gpu_stream_beam.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r05new/tests.log 2>&1
