set -o pipefail
python - <<'PY'
from tests.test_host_sanitize import _write_model
from funasr_amd.config import paraformer_streaming_tiny, paraformer_tiny
cfg = paraformer_tiny(enc_blocks=2, dec_blocks=1, vocab_size=64); cfg.ctc_weight = 0.3
scfg = paraformer_streaming_tiny(enc_blocks=2, dec_blocks=1, vocab_size=64); scfg.ctc_weight = 0.3
_write_model("/tmp/m.bin", cfg, 3); _write_model("/tmp/m.bin.stream", scfg, 4)
print("models written", flush=True)
PY
printf "leak:libamdhip64\nleak:libhsa-runtime64\nleak:libhsakmt\n" > /tmp/lsan.supp
ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:exitcode=86:verify_asan_link_order=0 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 LSAN_OPTIONS=suppressions=/tmp/lsan.supp timeout -k 10 150 stdbuf -oL ./tests/asan/api_driver gpu /tmp/m.bin > gpurun_out/asan_drv.txt 2>&1
rc=$?
tail -30 gpurun_out/asan_drv.txt
exit $rc
