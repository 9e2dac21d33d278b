"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU, no GPU): the FSMN-VAD state machine
(funasr_amd/csrc/vad_detector.hip, the host-only part of libpfm_hip.so) built alone with
g++ -fsanitize=address,undefined and driven (tests/asan/vad_driver.cc) by
  * the reference's per-chunk posteriors / decibels (tests/golden/vad.npz): the reference's segments exactly;
  * seeded random posteriors / decibels in random chunkings, offline and streaming, with final flags: the same
    segments as the Python statement of the reference's state machine (funasr_amd/vad.py).
Any sanitizer report aborts the driver (-fno-sanitize-recover), which fails the test."""
import json
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

from funasr_amd.config import fsmn_vad
from funasr_amd.vad import VadDetector

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("asan") / "vad_driver")
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "include"), "-x", "c++",
           os.path.join(ROOT, "funasr_amd", "csrc", "vad_detector.hip"), os.path.join(ROOT, "tests", "asan", "vad_driver.cc"),
           "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def _run(driver, path, chunks, streaming):
    with open(path, "wb") as f:
        f.write(struct.pack("<ii", len(chunks), int(streaming)))
        for db, ps, fin in chunks:
            db = np.ascontiguousarray(db, dtype=np.float64)
            ps = np.ascontiguousarray(ps, dtype=np.float32)
            f.write(struct.pack("<ii", db.size, ps.size))
            f.write(db.tobytes())
            f.write(ps.tobytes())
            f.write(struct.pack("<i", int(fin)))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=86",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([driver, path], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln]
    assert not any(ln.startswith("error") for ln in lines), lines
    return [[int(a) for a in ln.split()] for ln in lines]


def test_opts_match_config():
    """The driver uses pfm_vad_opts_default, which the golden runs use (fsmn_vad().vad_opts)."""
    o = fsmn_vad().vad_opts
    assert o["max_end_silence_time"] == 800 and o["window_size_ms"] == 200 and o["speech_noise_thres"] == 0.6


@pytest.mark.parametrize("name", ["v1", "v2"])
def test_vad_state_machine_asan_reference_segments(driver, tmp_path, name):
    gj = json.load(open(f"{GOLD}/vad.json"))[name]
    g = np.load(f"{GOLD}/vad.npz")
    p0, po = g[f"{name}_p0"], g[f"{name}_p0_off"]
    db, do = g[f"{name}_db"], g[f"{name}_db_off"]
    chunks = [(db[do[c]:do[c + 1]], p0[po[c]:po[c + 1]], c == len(po) - 2) for c in range(len(po) - 1)]
    assert _run(driver, str(tmp_path / "in.bin"), chunks, False) == gj["segments"]


@pytest.mark.parametrize("seed", range(6))
def test_vad_state_machine_asan_random(driver, tmp_path, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(50, 4000))
    # speech-like runs: posteriors switching between low / high silence probability, decibels with quiet gaps
    flips = np.cumsum(rng.integers(5, 300, size=64))
    state = (np.searchsorted(flips, np.arange(n)) % 2).astype(bool)
    ps = np.where(state, rng.uniform(0.0, 0.3, n), rng.uniform(0.7, 1.0, n)).astype(np.float32)
    db = np.where(state, rng.uniform(40, 90, n), rng.uniform(-120, 30, n))
    for streaming in (False, True):
        cuts = np.sort(rng.choice(np.arange(1, n), size=int(rng.integers(0, 8)), replace=False)) if n > 8 else []
        bounds = [0] + list(cuts) + [n]
        chunks = [(db[a:b], ps[a:b], i == len(bounds) - 2) for i, (a, b) in enumerate(zip(bounds[:-1], bounds[1:]))]
        segs = _run(driver, str(tmp_path / f"in{int(streaming)}.bin"), chunks, streaming)
        # the same segments as the Python statement of the reference's state machine (funasr_amd/vad.py)
        det = VadDetector(fsmn_vad().vad_opts)
        want = []
        for d, p, fin in chunks:
            det.decibel.extend(np.asarray(d, dtype=np.float64).tolist())
            det.p_sil.extend(np.asarray(p, dtype=np.float32).tolist())
            det.frm_cnt += len(p)
            det.detect_chunk(len(p), fin)
            want += det.segments(fin, streaming)
        assert segs == want, (streaming, segs[:5], want[:5])


# ---- the library's C-ABI host code (pfm_api.hip: argument validation, workspace sizing, weight re-layout) under
# ASan + UBSan: tests/asan/api_driver.cc linked with pfm_api.hip / vad_detector.hip built with -Xarch_host
# -fsanitize=address,undefined (tests/asan/build_api_driver.py; the device code and the other objects as shipped)
API_ENV = {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:exitcode=86:verify_asan_link_order=0",
           "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}


@pytest.fixture(scope="module")
def api_driver():
    sys_path = os.path.join(ROOT, "tests", "asan")
    from tests.asan.build_api_driver import OUT, build_api_driver
    from funasr_amd.build import OBJ_DIR
    if os.path.isdir(OBJ_DIR) and any(f.endswith(".o") for f in os.listdir(OBJ_DIR)):
        try:
            return build_api_driver()   # (incremental) where the library's objects are (the build container)
        except (RuntimeError, OSError, subprocess.CalledProcessError) as e:
            pytest.fail(f"building {sys_path}/api_driver failed: {getattr(e, 'stderr', e)}")
    if os.path.exists(OUT):
        return OUT   # the GPU box: objects do not travel, the binary built by __graft_entry__.build() does
    pytest.fail("tests/asan/api_driver missing and the library objects to build it are absent")


def _api_run(drv, args, tmp_path, timeout=300):
    supp = tmp_path / "lsan.supp"
    # the HIP / HSA runtimes keep process-lifetime allocations; leaks from the library itself still fail
    supp.write_text("leak:libamdhip64\nleak:libhsa-runtime64\nleak:libhsakmt\nleak:librocprofiler\n")
    env = dict(os.environ, **API_ENV)
    env["LSAN_OPTIONS"] = f"suppressions={supp}"
    r = subprocess.run([drv] + args, capture_output=True, text=True, env=env, timeout=timeout)
    fails = [ln for ln in r.stdout.splitlines() if ln.startswith("error")]
    assert r.returncode == 0 and "PASSED" in r.stdout, (r.returncode, fails[:20], r.stderr[-3000:])
    return r.stdout


def test_api_validation_asan(api_driver, tmp_path):
    """Every C-ABI entry point with null / out-of-range arguments (a PFM_E_* code and a message, no launch),
    pfm_create's configuration checks (13 bad configs), the config defaults and the host VAD detector, with the
    host code under ASan + UBSan (no device needed: pfm_create stops at the device query here)."""
    out = _api_run(api_driver, ["cpu"], tmp_path)
    assert out.count("\nok ") > 100


def _write_model(path, cfg, seed):
    from funasr_amd.runtime import PfmConfig
    from funasr_amd.weights import make_weights
    sd = make_weights(cfg, seed=seed)
    with open(path, "wb") as f:
        f.write(b"PFMW")
        f.write(bytes(PfmConfig.from_config(cfg)))
        f.write(struct.pack("<I", len(sd)))
        for k, v in sd.items():
            v = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
            name = k.encode()
            f.write(struct.pack("<I", len(name)) + name + struct.pack("<I", v.ndim))
            f.write(np.asarray(v.shape, dtype=np.int64).tobytes())
            f.write(v.tobytes())


@pytest.mark.gpu
def test_api_end_to_end_asan_gpu(api_driver, tmp_path):
    """The host code under ASan + UBSan driving a tiny Paraformer (2 encoder / 1 decoder blocks, CTC head,
    64-token vocabulary) on the device: every weight through pfm_set_weight (host Conv1d / FSMN-tap re-layouts)
    and pfm_set_weight_device, the refusals of unknown keys / rank / shape / dtype, reserve and growth past it,
    exact / fast / beam runs on a ragged batch (outputs in range, exact deterministic), profiling, then a streaming
    model (dec_sanm_shift 5) through streams create / step / tail / reset / duplicate-slot refusal / beam step and
    teardown."""
    from funasr_amd.config import paraformer_streaming_tiny, paraformer_tiny
    cfg = paraformer_tiny(enc_blocks=2, dec_blocks=1, vocab_size=64)
    cfg.ctc_weight = 0.3
    scfg = paraformer_streaming_tiny(enc_blocks=2, dec_blocks=1, vocab_size=64)
    scfg.ctc_weight = 0.3
    path = str(tmp_path / "model.bin")
    _write_model(path, cfg, 3)
    _write_model(path + ".stream", scfg, 4)
    out = _api_run(api_driver, ["gpu", path], tmp_path)
    for check in ("run fast", "run exact", "exact run deterministic", "run_beam", "stream_step", "stream_step_beam",
                  "destroy streaming"):
        assert f"ok {check}\n" in out, check
