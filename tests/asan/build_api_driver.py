"""Build tests/asan/api_driver: the library's host code (pfm_api.hip, vad_detector.hip) compiled with the host
half under AddressSanitizer + UndefinedBehaviorSanitizer (-Xarch_host: the device code is built as usual; GPU
sanitizers are not used on this pool), linked with the library's other objects (funasr_amd/_lib/obj, built by
funasr_amd.build) and the driver tests/asan/api_driver.cc. Test infrastructure: __graft_entry__.build() runs it so
the binary travels with the tree to the GPU box (objects do not).

    python tests/asan/build_api_driver.py
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from funasr_amd.build import ARCH, CSRC, OBJ_DIR, build, hipcc  # noqa: E402

OUT = os.path.join(HERE, "api_driver")
BUILD = os.path.join(HERE, "_build")
SANITIZED = ("pfm_api.hip", "vad_detector.hip")
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-Xarch_host",
       "-fno-sanitize-recover=all", "-Xarch_host", "-fno-omit-frame-pointer"]


def _newer(out, deps):
    return not os.path.exists(out) or any(os.path.getmtime(d) > os.path.getmtime(out) for d in deps)


def build_api_driver() -> str:
    build()   # the library's objects
    os.makedirs(BUILD, exist_ok=True)
    cc = hipcc()
    inc = ["-I", os.path.join(ROOT, "include")]
    hdrs = [os.path.join(ROOT, "include", "pfm.h")] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    objs = []
    for name in SANITIZED:
        src, obj = os.path.join(CSRC, name), os.path.join(BUILD, name + ".asan.o")
        if _newer(obj, [src] + hdrs):
            subprocess.run([cc, "-O1", "-g", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}"] + SAN + inc +
                           ["-c", src, "-o", obj], check=True, capture_output=True, text=True)
        objs.append(obj)
    drv_src, drv_obj = os.path.join(HERE, "api_driver.cc"), os.path.join(BUILD, "api_driver.o")
    if _newer(drv_obj, [drv_src] + hdrs):
        subprocess.run([cc, "-O1", "-g", "-std=c++17", f"--offload-arch={ARCH}"] + SAN + inc +
                       ["-c", drv_src, "-o", drv_obj], check=True, capture_output=True, text=True)
    lib_objs = sorted(os.path.join(OBJ_DIR, f) for f in os.listdir(OBJ_DIR)
                      if f.endswith(".o") and f[:-2] not in SANITIZED)
    deps = objs + [drv_obj] + lib_objs
    if _newer(OUT, deps):
        subprocess.run([cc, f"--offload-arch={ARCH}", "-fsanitize=address,undefined", "-fno-gpu-sanitize", "-o",
                        OUT + ".tmp"] + deps,
                       check=True, capture_output=True, text=True)
        os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build_api_driver())
