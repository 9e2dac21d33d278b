#!/bin/bash
# round 6, seventh call: the bf16 attention's softmax variants alone (tools/attn_bench: base, MFMA row sums, C = -max
# start, both), their PMC VALU / MFMA ratio (base vs MFMA row sums), and the long-audio leg's host profile
set -o pipefail
mkdir -p gpurun_out/r06g
for b in attn_bench attn_bench_l attn_bench_c attn_bench_cl; do
  echo "== $b" >> gpurun_out/r06g/attn_bench.txt
  timeout -k 10 60 ./tools/$b 30 >> gpurun_out/r06g/attn_bench.txt 2>&1 || exit $?
done
cat gpurun_out/r06g/attn_bench.txt | grep -E "==|B=" | head -40
R=$(pwd)
for v in base attnl; do
  if [ $v = attnl ]; then export PFM_LIB=$R/abvar/attnl/libpfm_hip.so; fi
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE -d $R/gpurun_out/r06g/pmc_$v -o run -- python3 $R/tools/attn_ab.py > $R/gpurun_out/r06g/pmc_$v.log 2>&1) || exit $?
  python tools/pmc_dump.py gpurun_out/r06g/pmc_$v/run_results.db attn > gpurun_out/r06g/pmc_$v.txt
done
unset PFM_LIB
tail -5 gpurun_out/r06g/pmc_base.txt gpurun_out/r06g/pmc_attnl.txt
timeout -k 10 300 python tools/long_audio_prof.py > gpurun_out/r06g/long_audio_prof.txt 2>&1
