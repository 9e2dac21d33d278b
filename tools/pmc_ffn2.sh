#!/bin/bash
# PMC passes of the 128-row fused FFN kernel alone (tools/ffn2_bench with FFN2_ONLY: the OP kernel, 3 + 5 launches):
#   [FFN2_ONLY=4] tools/pmc_ffn2.sh tag [M]   -> gpurun_out/pmcf2/<tag>.txt   (4: the OP + next-QKV kernel)
# Each pass is its own rocprofv3 run (counter slots per pass: MI355X_MICROARCH "rocprofv3 PMC slots").
set -o pipefail
R=$(pwd); tag=$1; M=${2:-32000}
D=$R/gpurun_out/pmcf2
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && export FFN2_ONLY=${FFN2_ONLY:-1}
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $D/${tag}kt -o run -- $R/tools/ffn2_bench $M > $D/${tag}kt.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $D/$tag -o run -- $R/tools/ffn2_bench $M > $D/$tag.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE -d $D/${tag}2 -o run -- $R/tools/ffn2_bench $M > $D/${tag}2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d $D/${tag}3 -o run -- $R/tools/ffn2_bench $M > $D/${tag}3.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum -d $D/${tag}4 -o run -- $R/tools/ffn2_bench $M > $D/${tag}4.log 2>&1
rc=$?
cd $R
for s in "" 2 3 4; do python tools/pmc_dump.py $D/$tag$s/run_results.db ffn2_kernel >> $D/$tag.txt; done
exit $rc
