set -o pipefail
mkdir -p gpurun_out/r05xw
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -k "split or qkv or gemm or ffn" > gpurun_out/r05xw/ops.log 2>&1 &&
timeout -k 10 400 python -u tools/xw_ab.py 0 7 15 > gpurun_out/r05xw/ab.txt 2>&1
