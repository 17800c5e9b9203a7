"""Decode goldens: the reference's own decoder (PACFile.ReadDataBlock +
codec.Decode + PCMFile.WriteDataBlock, driven as pacfile.py's __main__ does)
run through the /tmp shim (refshim.py) on the committed encode goldens and
fixtures; records the sha256 and frame count of every output WAV in
decode_manifest.json.  Run by hand in the build container:

    python tests/golden/make_decode_golden.py

The 12 master decodes the reference itself committed (outputs/*.wav) are
recorded as well, hashed straight from /root/reference.
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
SHIM = "/tmp/pac_refshim"
PINNED = ["piano_test2", "harmonic_test2", "harmonic_test4", "percussion_test1", "percussion_test2",
          "percussion_test3", "piano_test3", "pop_test2", "rock", "rock_test2", "speech_test2",
          "speech_test3"]


def sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def shim_decode(inp, profile):
    out = tempfile.mktemp(suffix=".wav")
    code = ("import sys; sys.path.insert(0, %r); import refdriver; refdriver.decode(%r, %r, %r)"
            % (os.path.join(SHIM, profile), inp, out, profile))
    subprocess.run([sys.executable, "-c", code], check=True, cwd=os.path.join(SHIM, profile))
    h = sha(out)
    n = (os.path.getsize(out) - 44) // 4
    os.remove(out)
    return h, n


def main():
    subprocess.run([sys.executable, os.path.join(HERE, "refshim.py")], check=True)
    man = {"shim": {}, "reference_outputs": {}}
    for name in sorted(os.listdir(HERE)):
        if name.endswith(".pac") or name.endswith(".wak"):
            prof = "origin" if name.endswith(".pac") else "master"
            h, n = shim_decode(os.path.join(HERE, name), prof)
            man["shim"][name] = {"sha256": h, "frames_x_ch_over_2": n}
            print(name, h[:16])
    for name in ("harpsichord.pac", "piano_test2.wak"):
        prof = "origin" if name.endswith(".pac") else "master"
        h, n = shim_decode(os.path.join(ROOT, "tests", "fixtures", name), prof)
        man["shim"]["fixtures/" + name] = {"sha256": h, "frames_x_ch_over_2": n}
        print(name, h[:16])
    for n in PINNED:
        man["reference_outputs"][n] = sha(os.path.join(REF, "outputs", n + ".wav"))
    with open(os.path.join(HERE, "decode_manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
