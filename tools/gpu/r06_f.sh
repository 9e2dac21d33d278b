#!/bin/bash
# round 6, sixth call: the attention's MFMA row sums (variant library) A/B + parity; VAD frame energies, host
# punctuation entry and the VAD pipeline tests; the long-audio leg
set -o pipefail
mkdir -p gpurun_out/r06f
timeout -k 10 300 python -u -m pytest tests/test_gpu_vad.py tests/test_gpu_punc.py -q --timeout 120 --timeout-method thread > gpurun_out/r06f/vad_punc.log 2>&1
rc=$?; echo "vad/punc rc=$rc" >> gpurun_out/r06f/vad_punc.log; tail -5 gpurun_out/r06f/vad_punc.log
case $rc in 0|1) ;; *) exit $rc ;; esac
AB="--sv-steps 0 --stream-chunks 0 --punc-steps 0 --beam-steps 0 --long-audio-s 0 --generate 0 --steps 10"
timeout -k 10 300 python tools/bench_ab.py 3 "X=0" "PFM_LIB=/root/repo/abvar/attnl/libpfm_hip.so" -- $AB > gpurun_out/r06f/ab_attn.txt 2>&1
rc=$?; tail -3 gpurun_out/r06f/ab_attn.txt
case $rc in 0) ;; *) exit $rc ;; esac
PFM_LIB=/root/repo/abvar/attnl/libpfm_hip.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -s -k "headline_fast_default_dispatch or fused_fsmn" --timeout 120 --timeout-method thread > gpurun_out/r06f/attn_var_parity.log 2>&1
rc=$?; echo "attn variant parity rc=$rc" >> gpurun_out/r06f/attn_var_parity.log; tail -3 gpurun_out/r06f/attn_var_parity.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python bench.py --steps 5 --exact-steps 0 --cpu-utts 0 --sv-steps 0 --stream-chunks 0 --beam-steps 0 > gpurun_out/r06f/bench_la.json 2> gpurun_out/r06f/bench_la.err
rc=$?; tail -2 gpurun_out/r06f/bench_la.err
exit $rc
