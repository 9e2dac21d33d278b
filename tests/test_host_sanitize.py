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
