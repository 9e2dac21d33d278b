#!/bin/bash
# ffn2 stream timing (sustained), the C-ABI host code under ASan on the device, the FFN op and parity tests
set -o pipefail
timeout -k 10 200 env FFN2_ANAT=2 ./tools/ffn2_bench 32000 2>&1 | tee gpurun_out/r05m_anat.txt || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_host_sanitize.py -m gpu \
  2>&1 | tee gpurun_out/r05m_asan.log || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py \
  tests/test_gpu_parity.py 2>&1 | tee gpurun_out/r05m_tests.log
