#!/bin/bash
# round 6, third call: the split decoder FFN (k_ffn2.hip MODE 7 / 8) op tests first, then the parity suites, an
# interleaved A/B of the decoder kernels / group splits and of the attention's C = -max start (variant library),
# then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -q -k "ffn_fused_decoder" --timeout 120 --timeout-method thread -x > gpurun_out/r06c/ops.log 2>&1
rc=$?; echo "ops rc=$rc" >> gpurun_out/r06c/ops.log; tail -4 gpurun_out/r06c/ops.log
case $rc in 0) ;; *) exit 1 ;; esac
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_automodel.py -q --timeout 240 --timeout-method thread > gpurun_out/r06c/parity.log 2>&1
rc=$?; echo "parity rc=$rc" >> gpurun_out/r06c/parity.log; tail -8 gpurun_out/r06c/parity.log
case $rc in 0|1) ;; *) exit $rc ;; esac
AB="--sv-steps 0 --stream-chunks 0 --punc-steps 0 --beam-steps 0 --long-audio-s 0 --generate 0 --steps 10"
timeout -k 10 400 python tools/bench_ab.py 3 "PFM_DEC_FFN_FUSED=1" "PFM_DEC_FFN_FUSED=2" "PFM_DEC_FFN_FUSED=2 PFM_SUBBATCH=1 PFM_DEC_SUBBATCH=1" -- $AB > gpurun_out/r06c/ab_dec.txt 2>&1
rc=$?; tail -4 gpurun_out/r06c/ab_dec.txt
case $rc in 0) ;; *) exit $rc ;; esac
timeout -k 10 300 python tools/bench_ab.py 3 "X=0" "PFM_LIB=/root/repo/abvar/attncsub/libpfm_hip.so" -- $AB > gpurun_out/r06c/ab_attn.txt 2>&1
rc=$?; tail -3 gpurun_out/r06c/ab_attn.txt
case $rc in 0) ;; *) exit $rc ;; esac
PFM_LIB=/root/repo/abvar/attncsub/libpfm_hip.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -s -k "headline_fast_default_dispatch and 7 or fused_fsmn" --timeout 120 --timeout-method thread > gpurun_out/r06c/attn_var_parity.log 2>&1
rc=$?; echo "attn variant parity rc=$rc" >> gpurun_out/r06c/attn_var_parity.log; tail -3 gpurun_out/r06c/attn_var_parity.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r06c/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r06c/gpu_suite.log; tail -8 gpurun_out/r06c/gpu_suite.log
