set -o pipefail
bash tools/gpu_steps.sh "ffnops:300:python -u -m pytest tests/test_gpu_ops.py -q --timeout 120 --timeout-method thread -k ffn_fused" \
 "headline:300:python -u -m pytest tests/test_gpu_parity.py -q -s --timeout 120 --timeout-method thread -k 'headline or large_fast or folded_outproj or fused_decoder or fused_ffn'" \
 "ab:400:python tools/bench_ab.py 2 PFM_FFN_KERNEL=1 PFM_FFN_KERNEL=2 'PFM_FFN_KERNEL=2 PFM_SUBBATCH=1' -- --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0" \
 "prof:300:bash tools/profile_k2.sh"
