#!/bin/bash
# PMC passes + kernel trace of the fused FFN kernel alone: tools/pmc_ffn.sh tag [M]
set -o pipefail
R=$(pwd); tag=$1; M=${2:-16000}
mkdir -p $R/gpurun_out/pmcf
cd /tmp && export TMPDIR=/tmp
timeout -k 10 90 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmcf/${tag}kt -o run -- python3 $R/tools/ffn_one.py $M > $R/gpurun_out/pmcf/${tag}kt.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmcf/$tag -o run -- python3 $R/tools/ffn_one.py $M > $R/gpurun_out/pmcf/$tag.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmcf/${tag}2 -o run -- python3 $R/tools/ffn_one.py $M > $R/gpurun_out/pmcf/${tag}2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d $R/gpurun_out/pmcf/${tag}3 -o run -- python3 $R/tools/ffn_one.py $M > $R/gpurun_out/pmcf/${tag}3.log 2>&1
rc=$?
cd $R
for s in "" 2 3; do python tools/pmc_dump.py gpurun_out/pmcf/$tag$s/run_results.db ffn_fused >> gpurun_out/pmcf/$tag.txt; done
python -c "
import sqlite3; c=sqlite3.connect('gpurun_out/pmcf/${tag}kt/run_results.db')
for r in c.execute(\"select name, count(*), avg(duration), vgpr_count, accum_vgpr_count, lds_size, grid_x, workgroup_x from kernels where name like '%ffn%' group by name\"): print(r)
" >> gpurun_out/pmcf/$tag.txt
exit $rc
