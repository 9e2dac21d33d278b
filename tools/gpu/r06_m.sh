#!/bin/bash
# round 6, thirteenth call: the large streaming-beam fast test with emulation-derived bounds (printing its statistics)
set -o pipefail
mkdir -p gpurun_out/r06m
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_stream_beam.py -k large \
  > gpurun_out/r06m/tests.txt 2>&1; rc=$?
grep -E "chunk|stream beam|passed|failed|Error" gpurun_out/r06m/tests.txt | tail -24
exit $rc
