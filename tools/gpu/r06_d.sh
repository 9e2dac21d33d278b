#!/bin/bash
# round 6, fourth call: kernel traces (one stream per stage, so the trace's kernel time per call is the step) of the
# decoder FFN as k_ffn2.hip split (2) and k_ffn.hip (1); cProfile of the long-audio leg
set -o pipefail
mkdir -p gpurun_out/r06d
PFM_SUBBATCH=1 PFM_DEC_SUBBATCH=1 PFM_DEC_FFN_FUSED=2 bash tools/profile_fast.sh r06d_dec2 --generate 0 || exit $?
PFM_SUBBATCH=1 PFM_DEC_SUBBATCH=1 PFM_DEC_FFN_FUSED=1 bash tools/profile_fast.sh r06d_dec1 --generate 0 || exit $?
timeout -k 10 300 python tools/long_audio_prof.py > gpurun_out/r06d/long_audio_prof.txt 2>&1
rc=$?; tail -45 gpurun_out/r06d/long_audio_prof.txt | head -50
exit $rc
