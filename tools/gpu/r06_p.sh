#!/bin/bash
# round 6: EXACT-mode kernel trace (single group: per-kernel times reconcile with the step)
set -o pipefail
PFM_SUBBATCH=1 PFM_DEC_SUBBATCH=1 bash tools/profile_fast.sh r06p_exact_sb1 --mode exact > /dev/null 2>&1 || { tail -20 gpurun_out/r06p_exact_sb1/bench.log; exit 1; }
head -30 gpurun_out/r06p_exact_sb1/summary.md
