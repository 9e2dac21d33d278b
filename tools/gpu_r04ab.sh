set -o pipefail
mkdir -p gpurun_out/r04ab
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
P=funasr_amd/_lib/var/prev/libpfm_hip.so
timeout -k 10 400 $T tests/test_gpu_streaming.py tests/test_gpu_stream_beam.py tests/test_gpu_ops.py tests/test_gpu_parity.py -k "stream or attn or attention or cif" > gpurun_out/r04ab/tests.log 2>&1 &&
timeout -k 10 200 python tools/stream_tokens_dump.py gpurun_out/r04ab/tok_new.npy 4 40 > gpurun_out/r04ab/dump.txt 2>&1 &&
PFM_LIB=$P timeout -k 10 200 python tools/stream_tokens_dump.py gpurun_out/r04ab/tok_prev.npy 4 40 >> gpurun_out/r04ab/dump.txt 2>&1 &&
for k in 1 2 3; do
timeout -k 10 120 python tools/stream_prof.py --streams 1 --chunks 50 > gpurun_out/r04ab/stream1_new_$k.txt 2>&1 &&
PFM_LIB=$P timeout -k 10 120 python tools/stream_prof.py --streams 1 --chunks 50 > gpurun_out/r04ab/stream1_prev_$k.txt 2>&1 || exit 1
done &&
timeout -k 10 120 python tools/stream_prof.py --streams 64 --chunks 20 > gpurun_out/r04ab/stream64.txt 2>&1
