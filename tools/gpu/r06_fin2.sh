#!/bin/bash
# round 6, final call (bucketed punctuation graphs): the whole GPU suite, smoke(), the sanitizer driver on the GPU (host-pointer refusals), the
# default bench line, and a single-group rocprofv3 trace of the fast leg (reconciles with its own bench line)
set -o pipefail
O=gpurun_out/r06fin2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> $O/gpu_suite.log; tail -8 $O/gpu_suite.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
bash tools/gpu/r05_asan_drv.sh > $O/asan_wrap.log 2>&1; arc=$?
cp gpurun_out/asan_drv.txt $O/asan_drv.txt; echo "asan rc=$arc"; grep -c "^ok" $O/asan_drv.txt; grep -E "FAIL|SUMMARY" $O/asan_drv.txt | head -3
case $arc in 0|86) ;; *) exit $arc ;; esac
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('generate_value'), d['long_audio']['value'], d['exact_mode']['ms_per_step'])"
PFM_SUBBATCH=1 PFM_DEC_SUBBATCH=1 bash tools/profile_fast.sh r06fin2_fast_sb1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
head -3 gpurun_out/r06fin2_fast_sb1/summary.md
