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
# per-kernel VGPRs / LDS / the compiler's occupancy limit of this build
# (-Rpass-analysis=kernel-resource-usage), written beside the library; bench.py
# reports it next to the achieved occupancy of the PMC profile
RESOURCES = os.path.join(HERE, "libpacgpu.resources.json")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def cmd():
    return [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-ffp-contract=off",
            "-fPIC", "-shared", "-Wno-unused-value", "-Wno-unused-result", "-Rpass-analysis=kernel-resource-usage",
            "-o", LIB, SRC]


def parse_resources(text):
    """{kernel: {vgprs, sgprs, lds_bytes, occupancy_waves_per_simd, ...}} from
    the kernel-resource-usage remarks (demangled names, template args dropped)"""
    import re
    out, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = demangle(m.group(1))
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[([^\]]+)\])?: (\S+) \[-Rpass", line)
        if m and cur:
            key = {"TotalSGPRs": "sgprs", "VGPRs": "vgprs", "AGPRs": "agprs", "Occupancy": "occupancy_waves_per_simd",
                   "LDS Size": "lds_bytes", "ScratchSize": "scratch_bytes_per_lane", "VGPRs Spill": "vgpr_spill",
                   "SGPRs Spill": "sgpr_spill"}.get(m.group(1).strip())
            if key:
                v = m.group(3)
                out[cur][key] = int(v) if v.isdigit() else v
    return out


def demangle(sym):
    """k_master_front<true> style names as rocprofv3 prints them (no arguments)"""
    try:
        r = subprocess.run(["c++filt", sym], capture_output=True, text=True)
        name = r.stdout.strip() or sym
    except OSError:
        import re
        m = re.match(r"_Z(\d+)", sym)
        name = sym[m.end():m.end() + int(m.group(1))] if m else sym
    name = name.split("(")[0]
    return name[5:] if name.startswith("void ") else name


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
    import json
    with open(RESOURCES, "w") as f:
        json.dump({"src_hash": source_hash(), "kernels": parse_resources(r.stderr)}, f, indent=1, sort_keys=True)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
