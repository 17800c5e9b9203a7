"""Build recipe for libpacgpu.so (hipcc, gfx950 only).

    python -m pac_amd.build          (or pac_amd.build.build())

The library is built in-tree next to this file so it travels with the repo
snapshot to the GPU box.  -ffp-contract=off: no implicit FMA contraction; the
kernels use explicit fma only where the derivation says so.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "pac_abi.hip")
DEPS = [os.path.join(HERE, "csrc", f) for f in
        ("pac_abi.hip", "pac_kernels.hip", "pac_kernels.h", "pac_wave.h", "pac_common.h",
         "pac_master.hip", "pac_decode.hip", "pac_wav.hip", "pac_bs.h")] + [os.path.join(HERE, "..", "include", "pac_gpu.h")]
LIB = os.path.join(HERE, "libpacgpu.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def cmd():
    return [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-ffp-contract=off",
            "-fPIC", "-shared", "-Wno-unused-value", "-Wno-unused-result", "-o", LIB, SRC]


def source_hash():
    """sha256 (16 hex digits) of the kernel + C-ABI sources: profiles record
    it so that bench.py can refuse counters taken on a different build"""
    import hashlib
    h = hashlib.sha256()
    for d in DEPS:
        with open(d, "rb") as f:
            h.update(os.path.basename(d).encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in DEPS if os.path.exists(d))


def build(force=False, verbose=False):
    if not force and up_to_date():
        return LIB
    c = cmd()
    if verbose:
        print(" ".join(c))
    r = subprocess.run(c, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + r.stderr[-4000:])
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
