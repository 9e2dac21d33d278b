#!/bin/bash
# kernel time of the fused FFN kernel (pfm_op_ffn, M rows) under several PFM_* environment arms:
#   M=32000 tools/ffn_arms.sh "PFM_FFN_PD=2" "PFM_FFN_PD=3" ...
R=$(pwd); M=${M:-32000}
mkdir -p $R/gpurun_out/ffnarms
cd /tmp && export TMPDIR=/tmp
i=0
for arm in "$@"; do
  i=$((i+1))
  ( export $arm; timeout -k 10 90 rocprofv3 --kernel-trace -d $R/gpurun_out/ffnarms/a$i -o run -- python3 $R/tools/ffn_one.py $M 10 > $R/gpurun_out/ffnarms/a$i.log 2>&1 ) || exit $?
  python3 -c "
import sqlite3, glob
db = glob.glob('$R/gpurun_out/ffnarms/a$i/**/*.db', recursive=True)[0]
c = sqlite3.connect(db)
for r in c.execute(\"select count(*), avg(duration), min(duration) from kernels where name like '%ffn_fused%'\"): print('$arm', 'M $M', r)
"
done
