"""Build an A/B variant of libpacgpu.so: copy csrc/ to a temp dir, apply
literal (old -> new) replacements, compile to ab/libpacgpu_<name>.so.
Select it at run time with PAC_LIB=ab/libpacgpu_<name>.so.

    python tools/build_variant.py NAME FILE 'old' 'new' [FILE 'old' 'new' ...]
    python tools/build_variant.py NAME FILE @FILE path/to/replacement
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "perceptual-audio-codec_amd", "csrc")


def main(name, edits):
    tmp = tempfile.mkdtemp()
    src = os.path.join(tmp, "pkg", "csrc")
    shutil.copytree(CSRC, src)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    for f, old, new in edits:
        p = os.path.join(src, os.path.basename(f))
        s = open(p).read()
        if old == "@FILE":                 # replace the whole file by the one at path `new`
            shutil.copyfile(new, p)
            continue
        if old not in s:
            raise SystemExit("edit not found in %s: %r" % (f, old[:60]))
        open(p, "w").write(s.replace(old, new))
    out = os.path.join(ROOT, "ab", "libpacgpu_%s.so" % name)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
           "-shared", "-Wno-unused-value", "-Wno-unused-result", "-I" + os.path.join(ROOT, "include"),
           "-o", out, os.path.join(src, "pac_abi.hip")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr[-3000:])
    print(out)


if __name__ == "__main__":
    a = sys.argv[2:]
    main(sys.argv[1], [(a[i], a[i + 1], a[i + 2]) for i in range(0, len(a), 3)])
