#!/bin/bash
# round 6: C18 (4-wave 128x128 wave tiles) — GEMM op tests (every config incl. 18, bit identity vs C15 / C16), then the
# per-shape scan of the EXACT x6 shapes and the fast shapes
set -o pipefail
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "gemm_bf16 or 4wave" \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
SCAN_X6=1 timeout -k 10 300 python tools/gemm_cfg_scan.py 15 16 17 18 > $O/scan_x6.txt 2>&1 || exit $?
cat $O/scan_x6.txt | grep -v amdgpu.ids
timeout -k 10 300 python tools/gemm_cfg_scan.py 0 4 15 17 18 > $O/scan_fast.txt 2>&1 || exit $?
SCAN_GROUP=1 timeout -k 10 300 python tools/gemm_cfg_scan.py 0 15 17 18 >> $O/scan_fast.txt 2>&1 || exit $?
cat $O/scan_fast.txt | grep -v amdgpu.ids
