#!/bin/bash
# kernel time of the fused FFN diagnostic variants (PFM_FFN_VAR 0..3): tools/ffn_var.sh [M]
R=$(pwd); M=${1:-16000}
mkdir -p $R/gpurun_out/ffnvar
cd /tmp && export TMPDIR=/tmp
for v in ${VARS:-0 1 2 4}; do
  PFM_FFN_VAR=$v timeout -k 10 90 rocprofv3 --kernel-trace -d $R/gpurun_out/ffnvar/v$v -o run -- python3 $R/tools/ffn_one.py $M > $R/gpurun_out/ffnvar/v$v.log 2>&1 || exit $?
  python3 -c "
import sqlite3; c=sqlite3.connect('$R/gpurun_out/ffnvar/v$v/run_results.db')
for r in c.execute(\"select count(*), avg(duration), min(duration) from kernels where name like '%ffn_fused%'\"): print('VAR $v', r)
"
done
