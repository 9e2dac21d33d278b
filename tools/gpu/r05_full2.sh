set -o pipefail
mkdir -p gpurun_out/r05full
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_streaming.py::test_stream_large_fast_regret > gpurun_out/r05full/gpu_suite2.log 2>&1 ;
timeout -k 10 120 python -u -m pytest tests/test_gpu_streaming.py -m gpu -q --timeout 120 --timeout-method thread -k large_fast > gpurun_out/r05full/gpu_stream.log 2>&1 ;
timeout -k 10 300 python bench.py > gpurun_out/r05full/bench.json 2> gpurun_out/r05full/bench.err
