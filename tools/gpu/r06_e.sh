#!/bin/bash
# round 6, fifth call: the unsplit 128-row decoder FFN (k_ffn2.hip MODE 9 / 10) op tests, an interleaved A/B against
# the 64-row k_ffn.hip kernel, and the attention's MFMA row sums (variant library)
set -o pipefail
mkdir -p gpurun_out/r06e
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -q -k "ffn_fused_decoder" --timeout 120 --timeout-method thread -x > gpurun_out/r06e/ops.log 2>&1
rc=$?; echo "ops rc=$rc" >> gpurun_out/r06e/ops.log; tail -4 gpurun_out/r06e/ops.log
case $rc in 0) ;; *) exit 1 ;; esac
AB="--sv-steps 0 --stream-chunks 0 --punc-steps 0 --beam-steps 0 --long-audio-s 0 --generate 0 --steps 10"
timeout -k 10 400 python tools/bench_ab.py 3 "PFM_DEC_FFN_FUSED=1" "PFM_DEC_FFN_FUSED=3" "PFM_DEC_FFN_FUSED=3 PFM_DEC_SUBBATCH=1" -- $AB > gpurun_out/r06e/ab_dec.txt 2>&1
rc=$?; tail -4 gpurun_out/r06e/ab_dec.txt
case $rc in 0) ;; *) exit $rc ;; esac
timeout -k 10 300 python tools/bench_ab.py 3 "X=0" "PFM_LIB=/root/repo/abvar/attnl/libpfm_hip.so" -- $AB > gpurun_out/r06e/ab_attn.txt 2>&1
rc=$?; tail -3 gpurun_out/r06e/ab_attn.txt
case $rc in 0) ;; *) exit $rc ;; esac
PFM_LIB=/root/repo/abvar/attnl/libpfm_hip.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -s -k "headline_fast_default_dispatch or fused_fsmn" --timeout 120 --timeout-method thread > gpurun_out/r06e/attn_var_parity.log 2>&1
rc=$?; echo "attn variant parity rc=$rc" >> gpurun_out/r06e/attn_var_parity.log; tail -3 gpurun_out/r06e/attn_var_parity.log
