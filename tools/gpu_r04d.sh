set -o pipefail
mkdir -p gpurun_out/r04d
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -k "ln_gemm or skinny or outproj" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04d/tests.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_streaming.py tests/test_gpu_stream_beam.py tests/test_gpu_beam.py -x -q --timeout 120 --timeout-method thread >> gpurun_out/r04d/tests.log 2>&1 &&
PFM_LIB=funasr_amd/_lib/var/p3i/libpfm_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -k "outproj_qkv or headline" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04d/p3i_tests.log 2>&1 &&
timeout -k 10 120 ./tools/ffn2_bench 32000 > gpurun_out/r04d/ffn2.txt 2>&1 &&
timeout -k 10 120 ./tools/ffn2_bench_p3i 32000 >> gpurun_out/r04d/ffn2.txt 2>&1 &&
timeout -k 10 120 python tools/stream_prof.py --streams 1 --chunks 50 > gpurun_out/r04d/stream1.txt 2>&1 &&
timeout -k 10 60 ./tools/beam_bench_prev 64 230 500 10 > gpurun_out/r04d/beam.txt 2>&1 &&
timeout -k 10 60 ./tools/beam_bench 64 230 500 10 >> gpurun_out/r04d/beam.txt 2>&1 &&
timeout -k 10 60 ./tools/beam_bench_tab 64 230 500 10 >> gpurun_out/r04d/beam.txt 2>&1 &&
timeout -k 10 500 python tools/bench_ab.py 2 "X=0" "PFM_LIB=funasr_amd/_lib/var/p3i/libpfm_hip.so" -- --sv-steps 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 --beam-steps 0 > gpurun_out/r04d/ab.txt 2>&1 &&
bash tools/profile_fast.sh r04c_fast &&
bash tools/pmc_bench.sh gpurun_out/r04_pmc_bench.json > gpurun_out/r04d/pmc_bench.log 2>&1
