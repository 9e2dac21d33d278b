#!/bin/bash
# round 6, second call: EXACT batch invariance (one MFMA shape for every x6 GEMM), the parity suite, the bench line
set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 300 python -u -m pytest tests/test_gpu_automodel.py tests/test_gpu_parity.py -q --timeout 240 --timeout-method thread -x > gpurun_out/r06b/suite_a.log 2>&1
rc=$?; echo "suite_a rc=$rc" >> gpurun_out/r06b/suite_a.log; tail -6 gpurun_out/r06b/suite_a.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r06b/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r06b/gpu_suite.log; tail -8 gpurun_out/r06b/gpu_suite.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 500 python bench.py --cpu-utts 0 > gpurun_out/r06b/bench.json 2> gpurun_out/r06b/bench.err
