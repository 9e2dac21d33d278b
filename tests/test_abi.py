"""The C-ABI library builds/loads on a host without a GPU and exports exactly what include/pfm.h
declares; the ctypes config struct matches the header's pfm_config field order and types."""
import ctypes
import os
import re
import subprocess

import pytest

from funasr_amd import runtime as rt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pfm.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pfm_[a-z_0-9]+)\s*\(", src)))


def test_library_present_and_loads():
    if not os.path.exists(rt.LIB_PATH):
        from funasr_amd.build import build
        build()
    lib = rt.load_library()
    assert lib is not None


def test_exports_every_declared_symbol():
    rt.load_library()
    declared = _declared_functions()
    assert set(declared) == set(rt.ABI_SYMBOLS), (set(declared) ^ set(rt.ABI_SYMBOLS))
    out = subprocess.run(["nm", "-D", "--defined-only", rt.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (pfm_[a-z_0-9]+)$", out, flags=re.M))
    missing = set(declared) - exported
    assert not missing, missing


def test_config_struct_matches_header():
    src = open(HEADER).read()
    body = re.search(r"typedef struct pfm_config \{(.*?)\} pfm_config;", src, re.S).group(1)
    fields = re.findall(r"(int32_t|float)\s+(\w+);", body)
    py = [(n, t) for n, t in rt.PfmConfig._fields_]
    assert [f[1] for f in fields] == [n for n, _ in py]
    for (ctype, _), (_, pytype) in zip(fields, py):
        assert (pytype is ctypes.c_int32) == (ctype == "int32_t")


def test_config_default_is_paraformer_large():
    lib = rt.load_library()
    c = rt.PfmConfig()
    lib.pfm_config_default(ctypes.byref(c))
    from funasr_amd.config import paraformer_large
    want = rt.PfmConfig.from_config(paraformer_large())
    for name, _ in rt.PfmConfig._fields_:
        assert getattr(c, name) == pytest.approx(getattr(want, name)), name


def test_errors_are_reported_not_thrown():
    lib = rt.load_library()
    c = rt.PfmConfig()
    lib.pfm_config_default(ctypes.byref(c))
    c.heads = 3   # d_model 512 / 3 is not a 128-wide head
    h = ctypes.c_void_p()
    rc = lib.pfm_create(ctypes.byref(c), 0, ctypes.byref(h))
    assert rc == -1
    assert b"head" in lib.pfm_last_error()
    assert lib.pfm_lfr_frames(80000) == 83
    assert lib.pfm_lfr_frames(480000) == 500
    assert lib.pfm_lfr_frames(399) == 0


def test_product_path_does_not_import_oracle():
    """The shipped package never references the test oracle (no CPU fallback)."""
    pkg = os.path.join(ROOT, "funasr_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dirpath, f), encoding="utf-8").read()
                assert "oracle" not in re.sub(r"#.*|//.*", "", txt).replace("oracle/", ""), f


def test_config_sensevoice_is_sensevoice_small():
    lib = rt.load_library()
    c = rt.PfmConfig()
    lib.pfm_config_sensevoice(ctypes.byref(c))
    from funasr_amd.config import sense_voice_small
    want = rt.PfmConfig.from_config(sense_voice_small())
    for name in ("input_size", "d_model", "heads", "ffn", "enc_blocks", "kernel_size", "enc_sanm_shift", "vocab_size",
                 "ln_eps", "arch", "tp_blocks", "n_embed"):
        assert getattr(c, name) == pytest.approx(getattr(want, name)), name
    assert c.arch == rt.ARCH_SENSEVOICE and c.dec_blocks == 0
