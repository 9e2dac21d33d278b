#!/bin/bash
# PMC evidence for bench.py's roofline kernel set (the GEMM class: bf16 GEMMs + fused FFN kernels) on the headline
# leg alone: three separate rocprofv3 passes of the same short bench (one counter group each, no traces combined):
#   FETCH_SIZE | WRITE_SIZE | SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE + SQ_BUSY_CYCLES
# then tools/pmc_traffic.py (gfx950 corrections, MFMA busy = MFMA-busy cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)):
#   tools/pmc_bench.sh <out.json>
set -o pipefail
out=$1
R=$(pwd)
D=$R/gpurun_out/pmc_bench
mkdir -p $D
ARGS="--steps 3 --warmup 1 --exact-steps 0 --cpu-utts 0 --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 --beam-steps 0"
export PFM_SUBBATCH=1 PFM_DEC_SUBBATCH=1   # the roofline pass runs single-stream (profiling on)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $D/f -o run -- python3 $R/bench.py $ARGS > $D/f.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $D/w -o run -- python3 $R/bench.py $ARGS > $D/w.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $D/m -o run -- python3 $R/bench.py $ARGS > $D/m.log 2>&1
rc=$?
cd $R
[ $rc -eq 0 ] && python tools/pmc_traffic.py $D/f/run_results.db $D/w/run_results.db "$out" $D/m/run_results.db
exit $rc
