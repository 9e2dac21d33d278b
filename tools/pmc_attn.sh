set -o pipefail
R=$(pwd); mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmc/kt -o run -- python3 $R/tools/attn_ab.py > $R/gpurun_out/pmc/kt.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc/p1 -o run -- python3 $R/tools/attn_ab.py > $R/gpurun_out/pmc/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC GRBM_COUNT -d $R/gpurun_out/pmc/p2 -o run -- python3 $R/tools/attn_ab.py > $R/gpurun_out/pmc/p2.log 2>&1
rc=$?
cd $R
python tools/pmc_dump.py gpurun_out/pmc/p1/run_results.db attn > gpurun_out/pmc/attn_p1.txt
python tools/pmc_dump.py gpurun_out/pmc/p2/run_results.db attn > gpurun_out/pmc/attn_p2.txt
python -c "
import sqlite3; c=sqlite3.connect('gpurun_out/pmc/kt/run_results.db')
print(c.execute('pragma table_info(kernels)').fetchall())
" > gpurun_out/pmc/kt_schema.txt
exit $rc
