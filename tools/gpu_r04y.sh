set -o pipefail
mkdir -p gpurun_out/r04y
for k in 1 2 3; do
timeout -k 10 120 python tools/stream_prof.py --streams 1 --chunks 50 > gpurun_out/r04y/stream1_w8_$k.txt 2>&1 &&
PFM_ATTN_WAVES=4 timeout -k 10 120 python tools/stream_prof.py --streams 1 --chunks 50 > gpurun_out/r04y/stream1_w4_$k.txt 2>&1 || exit 1
done
