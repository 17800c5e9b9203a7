"""Generate the golden vectors under tests/golden/ from the reference itself.

Run by hand in the build container (needs /root/reference; never at test
time):  python tests/golden/make_golden.py

Builds the Python-3 shim of the reference in /tmp (refshim.py), encodes small
synthetic / edge-case inputs with the reference's own PACFile/codec code, and
records:
  * <case>.in.npy       int16 [frames, channels] input PCM
  * <case>.pac|.wak     the reference's data section + header (whole file)
  * stages_<case>.npz   per-stage values for a few blocks (MDCT before the
                        overall scale, masking thresholds, SMRs, bit allocation,
                        scale factors) captured by wrapping the reference's
                        functions
  * manifest.json       sha256 of every file above and of the reference
                        fixtures the tests rely on
"""
import hashlib
import json
import os
import struct
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
import pac_amd  # noqa: E402
from pac_amd import synth  # noqa: E402

SHIM = "/tmp/pac_refshim"


def write_wav(path, fs, pcm):
    pcm = np.ascontiguousarray(pcm, dtype="<i2")
    n, nch = pcm.shape
    data = pcm.tobytes()
    with open(path, "wb") as f:
        f.write(struct.pack("<4sL4s4sLHHLLHH4sL", b"RIFF", 36 + len(data), b"WAVE", b"fmt ", 16, 1,
                            nch, fs, fs * nch * 2, nch * 2, 16, b"data", len(data)))
        f.write(data)


def cases():
    n = 12 * 1024
    t = np.arange(n)
    sq = np.where((t // 37) % 2 == 0, 32767, -32768).astype(np.int16)
    # impulses 397 samples apart with distinct amplitudes: every window holds
    # several, so no two FFT magnitudes tie exactly (a lone impulse gives a
    # flat |FFT| and findpeaks then depends on FFT rounding -- DESIGN.md)
    imp = np.zeros(n, np.int16)
    k = np.arange(0, n, 397)
    imp[k] = (30000 - 523 * (np.arange(len(k)) % 37)).astype(np.int16)
    return [
        ("origin_white48k", "origin", 48000, synth.white_pcm(24 * 1024 + 333, 2, seed=1234)),
        ("origin_zero48k", "origin", 48000, np.zeros((5 * 1024, 2), np.int16)),
        ("origin_square44k", "origin", 44100, np.stack([sq, imp], 1)),
        ("origin_mono44k", "origin", 44100, synth.white_pcm(8 * 1024 + 17, 1, seed=5, scale=0.1)),
        ("master_pinktones48k", "master", 48000, synth.pink_tones_pcm(24 * 1024 + 100, 48000, seed=1234)),
        ("master_zero48k", "master", 48000, np.zeros((5 * 1024, 2), np.int16)),
        ("master_square44k", "master", 44100, np.stack([sq, imp], 1)),
        ("master_white48k", "master", 48000, synth.white_pcm(16 * 1024, 2, seed=99)),
    ]


STAGE_BLOCKS = (1, 3, 10)


def run_case(name, prof, fs, pcm):
    """Encode with the reference shim; capture per-stage values of a few blocks."""
    d = os.path.join(SHIM, prof)
    sys.path.insert(0, d)
    for m in ("codec", "psychoac", "mdct", "window", "quantize", "bitalloc", "pacfile",
              "pcmfile", "bitpack", "audiofile", "Huffman", "refdriver"):
        sys.modules.pop(m, None)
    cwd = os.getcwd()
    os.chdir(d)
    try:
        import codec as rc
        import psychoac as rp
        import refdriver
        cap = {"mdct": [], "thr": [], "smr": [], "ba": [], "sf": [], "overall": [], "lrms": []}
        state = {"blk": 0}
        orig_mdct = rc.MDCT

        def MDCT(*a, **k):
            out = orig_mdct(*a, **k)
            if state["blk"] in STAGE_BLOCKS:
                cap["mdct"].append((state["blk"], out[:1024].copy()))
            return out
        rc.MDCT = MDCT
        if prof == "origin":
            orig_thr = rp.getMaskedThreshold

            def gmt(*a, **k):
                out = orig_thr(*a, **k)
                if state["blk"] in STAGE_BLOCKS:
                    cap["thr"].append((state["blk"], out.copy()))
                return out
            rp.getMaskedThreshold = gmt
            orig_esc = rc.EncodeSingleChannel

            def esc(data, cp):
                s, b, m, o = orig_esc(data, cp)
                if state["blk"] in STAGE_BLOCKS:
                    cap["ba"].append((state["blk"], np.array(b).copy()))
                    cap["sf"].append((state["blk"], np.array(s).copy()))
                    cap["overall"].append((state["blk"], o))
                return s, b, m, o
            rc.EncodeSingleChannel = esc
            orig_smr = rc.CalcSMRs

            def csmr(*a, **k):
                out = orig_smr(*a, **k)
                if state["blk"] in STAGE_BLOCKS:
                    cap["smr"].append((state["blk"], np.array(out).copy()))
                return out
            rc.CalcSMRs = csmr
            orig_enc = rc.Encode

            def enc(data, cp):
                out = orig_enc(data, cp)
                state["blk"] += 1
                return out
            rc.Encode = enc
        else:
            orig_bthr = rp.calcBTHR

            def cb(*a, **k):
                out = orig_bthr(*a, **k)
                if state["blk"] in STAGE_BLOCKS:
                    cap["thr"].append((state["blk"], out.copy()))
                return out
            rp.calcBTHR = cb
            orig_gsmt = rp.getStereoMaskThreshold

            def gsmt(*a, **k):
                smr, lines = orig_gsmt(*a, **k)
                if state["blk"] in STAGE_BLOCKS:
                    cap["smr"].append((state["blk"], np.array(smr).copy()))
                return smr, lines
            rc.getStereoMaskThreshold = gsmt
            orig_edc = rc.EncodeDualChannel

            def edc(data, cp, lrms, h):
                s, b, m, o = orig_edc(data, cp, lrms, h)
                if state["blk"] in STAGE_BLOCKS:
                    cap["ba"].append((state["blk"], np.array(b).copy()))
                    cap["sf"].append((state["blk"], np.array(s).copy()))
                    cap["overall"].append((state["blk"], np.array(o)))
                    cap["lrms"].append((state["blk"], np.array(lrms).copy()))
                return s, b, m, o
            rc.EncodeDualChannel = edc
            orig_enc = rc.Encode

            def enc(data, cp, h):
                out = orig_enc(data, cp, h)
                state["blk"] += 1
                return out
            rc.Encode = enc
        wav = "/tmp/golden_%s.wav" % name
        write_wav(wav, fs, pcm)
        out = "/tmp/golden_%s.%s" % (name, "pac" if prof == "origin" else "wak")
        refdriver.encode(wav, out, prof)
        with open(out, "rb") as f:
            coded = f.read()
    finally:
        os.chdir(cwd)
        sys.path.remove(d)
    return coded, cap


def pack_stages(cap):
    out = {}
    for k, v in cap.items():
        if not v:
            continue
        out[k + "_block"] = np.array([b for b, _ in v])
        out[k] = np.array([np.asarray(x, dtype=np.float64) for _, x in v])
    return out


def sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main():
    subprocess.run([sys.executable, os.path.join(HERE, "refshim.py")], check=True)
    manifest = {"generated_by": "tests/golden/make_golden.py (reference shim, numpy %s)"
                % np.__version__, "files": {}, "reference_fixtures": {}}
    for name, prof, fs, pcm in cases():
        coded, cap = run_case(name, prof, fs, pcm)
        np.save(os.path.join(HERE, name + ".in.npy"), pcm)
        ext = "pac" if prof == "origin" else "wak"
        with open(os.path.join(HERE, "%s.%s" % (name, ext)), "wb") as f:
            f.write(coded)
        np.savez_compressed(os.path.join(HERE, "stages_%s.npz" % name), fs=fs, **pack_stages(cap))
        for fn in (name + ".in.npy", "%s.%s" % (name, ext), "stages_%s.npz" % name):
            manifest["files"][fn] = sha(os.path.join(HERE, fn))
        print(name, len(coded), "bytes")
    ref = "/root/reference"
    verified = ["coded/harpsichord.pac", "coded/german.pac", "coded/trumpet.pac"] + [
        "coded/%s.wak" % n for n in ("piano_test2 harmonic_test2 harmonic_test4 percussion_test1 "
                                     "percussion_test2 percussion_test3 piano_test3 pop_test2 rock "
                                     "rock_test2 speech_test2 speech_test3").split()] + [
        "coded/withHuffman/speech_test3.wak"]
    for v in verified:
        manifest["reference_fixtures"][v] = sha(os.path.join(ref, v))
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
