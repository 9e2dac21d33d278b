#!/bin/bash
# PMC passes on one GEMM shape: tools/pmc_gemm.sh M N K tag
set -o pipefail
R=$(pwd); M=$1; N=$2; K=$3; tag=$4
mkdir -p $R/gpurun_out/pmcg
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $R/gpurun_out/pmcg/$tag -o run -- python3 $R/tools/gemm_one.py $M $N $K > $R/gpurun_out/pmcg/$tag.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC GRBM_COUNT -d $R/gpurun_out/pmcg/${tag}2 -o run -- python3 $R/tools/gemm_one.py $M $N $K > $R/gpurun_out/pmcg/${tag}2.log 2>&1 &&
timeout -k 10 90 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmcg/${tag}kt -o run -- python3 $R/tools/gemm_one.py $M $N $K > $R/gpurun_out/pmcg/${tag}kt.log 2>&1
rc=$?
cd $R
python tools/pmc_dump.py gpurun_out/pmcg/$tag/run_results.db gemm > gpurun_out/pmcg/$tag.txt
python tools/pmc_dump.py gpurun_out/pmcg/${tag}2/run_results.db gemm >> gpurun_out/pmcg/$tag.txt
python -c "
import sqlite3; c=sqlite3.connect('gpurun_out/pmcg/${tag}kt/run_results.db')
for r in c.execute(\"select name, count(*), avg(duration), vgpr_count, accum_vgpr_count, lds_size, grid_x, workgroup_x from kernels where name like '%gemm%' group by name\"): print(r)
" >> gpurun_out/pmcg/$tag.txt
exit $rc
