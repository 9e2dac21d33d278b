#!/bin/bash
# round 6, first call: the sanitizer driver's host-pointer refusals (first: a refusal that failed would fault), the
# full GPU suite, the default bench line
set -o pipefail
mkdir -p gpurun_out/r06a
bash tools/gpu/r05_asan_drv.sh > gpurun_out/r06a/asan.log 2>&1
rc=$?
echo "asan rc=$rc" >> gpurun_out/r06a/asan.log
tail -5 gpurun_out/r06a/asan.log
case $rc in 0|1|86) ;; *) exit $rc ;; esac
grep -q "^error" gpurun_out/asan_drv.txt && grep "^error" gpurun_out/asan_drv.txt | head
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06a/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc" >> gpurun_out/r06a/gpu_suite.log
tail -15 gpurun_out/r06a/gpu_suite.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 500 python bench.py > gpurun_out/r06a/bench.json 2> gpurun_out/r06a/bench.err
rc=$?
tail -3 gpurun_out/r06a/bench.err
exit $rc
