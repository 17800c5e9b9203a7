"""Reference encodes of the M/S-extreme streams (tests/golden/msx/).

Run by hand in the build container (needs /root/reference; never at test
time):  python tests/golden/make_msx_golden.py

The inputs are generated, not stored: `pac_amd.synth.ms_extreme_pcm(kind,
MSX_FRAMES, fs, MSX_SEED)` -- dual-mono (S == 0), anti-phase (M == 0), one
silent channel, sparse +-1 LSB differences, DC pairs and a stream cycling
through all of them.  Each is written as a WAV file in /tmp and encoded by the
reference's own PACFile driver (the shim of refshim.py, master and Origin
coders); the coded files land in tests/golden/msx/ and msx_manifest.json keeps
the sha256 of every input's PCM bytes (the tests regenerate the input and
check it against this hash before comparing) and of every coded file.

Reference: codec/codec.py:94-102 (LRMS from the raw FFTs), psychoac.py:549-591
(M/S lines, the six calcBTHR calls, MLD), :662-682 (band selection).
"""
import hashlib
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
import pac_amd  # noqa: E402,F401
from pac_amd import synth  # noqa: E402
from make_golden import write_wav, SHIM  # noqa: E402

MSX_FRAMES = 200 * 1024 - 317      # 201 blocks with the Close() flush, ragged last hop
MSX_SEED = 2026
OUT = os.path.join(HERE, "msx")


def case_list():
    return [(kind, fs, prof) for kind in synth.MS_EXTREMES for fs in (44100, 48000)
            for prof in ("master", "origin")]


def case_name(kind, fs, prof):
    return "%s_%dk_%s.%s" % (kind, fs // 1000, prof, "wak" if prof == "master" else "pac")


def sha(b):
    return hashlib.sha256(b).hexdigest()


def encode_one(case):
    kind, fs, prof = case
    pcm = synth.ms_extreme_pcm(kind, MSX_FRAMES, fs, MSX_SEED)
    wav = "/tmp/msx_%s_%d_%s.wav" % (kind, fs, prof)
    out = "/tmp/msx_%s_%d_%s.coded" % (kind, fs, prof)
    write_wav(wav, fs, pcm)
    code = ("import sys, os; os.chdir(%r); sys.path.insert(0, %r); import refdriver; "
            "refdriver.encode(%r, %r, %r)" % (os.path.join(SHIM, prof), os.path.join(SHIM, prof), wav, out, prof))
    subprocess.run([sys.executable, "-c", code], check=True)
    with open(out, "rb") as f:
        coded = f.read()
    with open(os.path.join(OUT, case_name(*case)), "wb") as f:
        f.write(coded)
    os.remove(wav)
    os.remove(out)
    return case, sha(pcm.astype("<i2").tobytes()), sha(coded)


def main():
    subprocess.run([sys.executable, os.path.join(HERE, "refshim.py")], check=True)
    os.makedirs(OUT, exist_ok=True)
    man = {"generated_by": "tests/golden/make_msx_golden.py (reference shim)", "frames": MSX_FRAMES,
           "seed": MSX_SEED, "cases": {}}
    with ThreadPoolExecutor(max(1, min(8, os.cpu_count() or 1))) as ex:
        for (kind, fs, prof), pcm_sha, coded_sha in ex.map(encode_one, case_list()):
            man["cases"][case_name(kind, fs, prof)] = {"kind": kind, "fs": fs, "profile": prof,
                                                       "pcm_sha256": pcm_sha, "sha256": coded_sha}
            print(kind, fs, prof, flush=True)
    with open(os.path.join(HERE, "msx_manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
