set -o pipefail
mkdir -p gpurun_out/r04aa
P=funasr_amd/_lib/var/prev/libpfm_hip.so
PFM_LIB=$P timeout -k 10 200 python tools/stream_tokens_dump.py gpurun_out/r04aa/tok_prev.npy 4 40 > gpurun_out/r04aa/dump.txt 2>&1 &&
PFM_ATTN_WAVES=4 PFM_LIB=$P timeout -k 10 200 python tools/stream_tokens_dump.py gpurun_out/r04aa/tok_prev_w4.npy 4 40 >> gpurun_out/r04aa/dump.txt 2>&1
