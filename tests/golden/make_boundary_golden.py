"""Decision-boundary cases (tests/golden/boundary.py) and the reference's own
encodes of them.

Run by hand in the build container (needs /root/reference for the reference
encodes; never at test time):  python tests/golden/make_boundary_golden.py

1. Search (CPU oracle): windows of stereo reference inputs; a gain of one
   channel (lrms) or of both (alloc, mld) scanned, and every change of the
   oracle's decisions bisected until the two streams differ in one sample by
   one LSB; each bracket classified by the first decision that differs
   (boundary.classify / key_mld).  mld brackets are refined by one or two more
   single-LSB changes until the crossing line's MLD threshold sits within
   2^-30 of the M/S threshold (as intensities), on either side.
2. The reference coder (the refshim of refshim.py, the reference's PACFile
   driver) encodes every stream, and the dense-LSB M/S streams; the coded
   files land in tests/golden/boundary/ and the manifest keeps their sha256
   and the sha256 of every input's PCM.

Reference: codec/codec.py:94-102, bitalloc.py:129-184, psychoac.py:570-591.
"""
import hashlib
import json
import os
import subprocess
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import boundary as B  # noqa: E402

SOURCES = ["piano_test2.wav", "harmonic_test2.wav", "pop_test2.wav", "rock.wav", "speech_test2.wav",
           "percussion_test1.wav", "harpsichord.wav", "trumpet.wav", "german.wav", "rock_test2.wav",
           "speech_test3.wav", "harmonic_test4.wav"]
WANT = {"lrms": 10, "argmax": 10, "cut": 8, "budget": 3, "mld": 6, "mldneed": 4}
LSB_DENSE = [(D, fs, prof) for D in (4, 8) for fs in (44100, 48000) for prof in ("master", "origin")]


def spec(src, off, gL, gR, pert=()):
    return {"src": src, "off": int(off), "gL": float(gL).hex(), "gR": float(gR).hex(), "pert": [list(p) for p in pert]}


def bisect(fs, mk, g1, g2, key):
    """g1 < g2 with key(g1) != key(g2) -> adjacent streams (<= 1 sample apart)"""
    p1, p2 = mk(g1), mk(g2)
    k1 = key(B.oracle_blocks(fs, p1))
    for _ in range(80):
        if np.count_nonzero(p1 != p2) <= 1:
            break
        gm = 0.5 * (g1 + g2)
        if gm in (g1, g2):
            break
        pm = mk(gm)
        km = key(B.oracle_blocks(fs, pm))
        if km != k1:
            g2, p2 = gm, pm
        else:
            g1, p1 = gm, pm
    return g1, g2


def search_window(job):
    """all brackets of one (source, offset, mode) window"""
    src, off, mode = job
    fs, raw = B.source(src)
    if raw.shape[1] != 2 or off + B.FRAMES > raw.shape[0]:
        return []
    out = []
    if mode == "lrms":
        def mk(g):
            return B.make_pcm(spec(src, off, 1.0, g))
        key = B.key_lrms
        grid = np.linspace(0.55, 1.45, 19)
    elif mode == "alloc":
        def mk(g):
            return B.make_pcm(spec(src, off, g, g))
        key = B.key_alloc
        grid = np.geomspace(0.05, 1.0, 25)
    elif mode == "alloclr":            # R at a quarter of L: L/R-coded bands (the -15 dB cut)
        def mk(g):
            return B.make_pcm(spec(src, off, g, 0.25 * g))
        key = B.key_alloc
        grid = np.geomspace(0.02, 1.0, 33)
    else:
        def mk(g):
            return B.make_pcm(spec(src, off, g, g))

        def key(bl):
            return B.key_mld(bl, fs)
        grid = np.geomspace(0.1, 1.0, 25)
    ks = [key(B.oracle_blocks(fs, mk(g)[1])) for g in grid]
    for i in range(len(grid) - 1):
        if ks[i] == ks[i + 1]:
            continue
        g1, g2 = bisect(fs, lambda g: mk(g)[1], grid[i], grid[i + 1], key)
        gr = {"lrms": None, "alloclr": 0.25}.get(mode, 1.0)
        s1 = spec(src, off, 1.0, g1) if gr is None else spec(src, off, g1, gr * g1)
        s2 = spec(src, off, 1.0, g2) if gr is None else spec(src, off, g2, gr * g2)
        _, p1 = B.make_pcm(s1)
        _, p2 = B.make_pcm(s2)
        if np.count_nonzero(p1 != p2) != 1:
            continue
        b1, b2 = B.oracle_blocks(fs, p1), B.oracle_blocks(fs, p2)
        if mode == "mld":
            c = mld_class(fs, b1, b2)
        else:
            c = B.classify(fs, p1, p2, b1, b2)
        if c is None:
            continue
        out.append({"a": s1, "b": s2, **c})
    return out


def mld_class(fs, b1, b2):
    """the MLD row transition between two adjacent streams: the block, row and
    the single line whose d (boundary.mld_lines) changed sign"""
    k1, k2 = B.key_mld(b1, fs), B.key_mld(b2, fs)
    for t, (x, y) in enumerate(zip(k1, k2)):
        if x == y:
            continue
        bit = (x ^ y) & -(x ^ y)
        r = bit.bit_length() - 1
        var, row = ("S", r - 16) if r >= 16 else ("M", r)
        d1 = B.mld_lines(b1[t], fs)[var == "S"][64 * row:64 * row + 64]
        d2 = B.mld_lines(b2[t], fs)[var == "S"][64 * row:64 * row + 64]
        flip = [i for i in range(64) if (d1[i] < 0) != (d2[i] < 0)]
        if len(flip) != 1 or np.sum(d1 < 0) + np.sum(d2 < 0) != 1:
            return None             # not a clean 0 <-> 1 line transition of the row
        i = flip[0]
        line = 64 * row + i
        kind = "mldneed" if np.isnan(d1[i]) or np.isnan(d2[i]) else "mld"
        return {"kind": kind, "block": t, "detail": "MLD_%s row %d line %d" % (var, row, line),
                "mld": {"block": t, "var": var, "line": int(line)}}
    return None


def full_key(fs, bl):
    return B.key_alloc(bl), B.key_mld(bl, fs)


def refine(case, ncand=200, nverify=30):
    """Move each stream of a bracket closer to the case's threshold by one or
    two more single-LSB changes (random candidates in the deciding block's
    window, their effects on boundary.signed_margin taken as linear, the best
    combinations verified with the oracle): the sign of the margin (the
    decision) and every other decision of the stream (full_key) kept."""
    fs, _ = B.source(case["a"]["src"])
    out = dict(case)
    t = case["block"]
    lo, hi = max(0, 1024 * (t - 1)), min(B.FRAMES, 1024 * (t + 1))
    for side in ("a", "b"):
        s0 = case[side]
        _, p0 = B.make_pcm(s0)
        bl0 = B.oracle_blocks(fs, p0)
        k0, m0 = full_key(fs, bl0), B.signed_margin(case, fs, p0, bl0)
        if m0 is None:
            return None
        best = (abs(m0), s0, m0)
        rng = np.random.default_rng(11 + case["a"]["off"] + (side == "b") + 1000 * len(s0["pert"]))
        cand = sorted({(int(f), int(c), int(d)) for f, c, d in
                       zip(rng.integers(lo, hi, ncand), rng.integers(0, 2, ncand), rng.choice([-1, 1], ncand))})
        cand = [c for c in cand if (c[0], c[1]) not in {(q[0], q[1]) for q in s0["pert"]}]
        sens = []
        for pt in cand:
            sm = B.signed_margin(case, fs, B.make_pcm(dict(s0, pert=s0["pert"] + [list(pt)]))[1])
            sens.append(np.nan if sm is None else sm - m0)
        sens = np.array(sens)
        combos = []
        for a_ in range(len(cand)):
            if np.isnan(sens[a_]):
                continue
            e = m0 + sens[a_]
            if (e > 0) == (m0 > 0):
                combos.append((abs(e), [cand[a_]]))
            for b_ in range(a_ + 1, len(cand)):
                if np.isnan(sens[b_]) or (cand[a_][0], cand[a_][1]) == (cand[b_][0], cand[b_][1]):
                    continue
                e = m0 + sens[a_] + sens[b_]
                if (e > 0) == (m0 > 0):
                    combos.append((abs(e), [cand[a_], cand[b_]]))
        combos.sort(key=lambda x: x[0])
        for _, pts in combos[:nverify]:
            sp = dict(s0, pert=s0["pert"] + [list(q) for q in pts])
            _, p = B.make_pcm(sp)
            bl = B.oracle_blocks(fs, p)
            m = B.signed_margin(case, fs, p, bl)
            if m is None or (m > 0) != (m0 > 0) or full_key(fs, bl) != k0:
                continue
            if abs(m) < best[0]:
                best = (abs(m), sp, m)
        out[side] = best[1]
        out["margin_" + side] = best[2]
    out["margin"] = max(abs(out["margin_a"]), abs(out["margin_b"]))
    return out


def refine2(case):
    """two refinement passes (the second starts from the first's streams)"""
    r = refine(case)
    return refine(r) if r is not None else None


def reference_encode(job):
    """the reference coder's .wak / .pac of one int16 stream (refshim driver)"""
    name, fs, pcm, prof = job
    from make_golden import write_wav, SHIM
    wav = "/tmp/bnd_%s.wav" % name
    out = "/tmp/bnd_%s.coded" % name
    write_wav(wav, fs, pcm)
    code = ("import sys, os; os.chdir(%r); sys.path.insert(0, %r); import refdriver; "
            "refdriver.encode(%r, %r, %r)" % (os.path.join(SHIM, prof), os.path.join(SHIM, prof), wav, out, prof))
    subprocess.run([sys.executable, "-c", code], check=True)
    with open(out, "rb") as f:
        coded = f.read()
    os.remove(wav)
    os.remove(out)
    return name, coded


def main_mld():
    """--mld: redo only the MLD cases (more windows; both transition kinds),
    keeping the manifest's other cases and their reference files"""
    man = B.load_manifest()
    rng = np.random.default_rng(4049)
    jobs = []
    for src in SOURCES:
        fs, raw = B.source(src)
        if raw.shape[1] != 2:
            continue
        for off in rng.integers(0, raw.shape[0] - B.FRAMES, 8):
            jobs.append((src, int(off), "mld"))
    found = {"mld": [], "mldneed": []}
    with ProcessPoolExecutor(max(1, min(8, os.cpu_count() or 1))) as ex:
        for res in ex.map(search_window, jobs):
            for c in res:
                found[c["kind"]].append(c)
        print({k: len(v) for k, v in found.items()}, flush=True)
        new = []
        for k in ("mld", "mldneed"):
            lst = [c for c in ex.map(refine2, found[k][:3 * WANT[k]]) if c is not None]
            new += sorted(lst, key=lambda c: c["margin"])[:WANT[k]]
    keep = [c for c in man["cases"] if c["kind"] not in ("mld", "mldneed")]
    for c in man["cases"]:
        if c["kind"] in ("mld", "mldneed"):
            for side in ("a", "b"):
                os.remove(os.path.join(B.OUT, "%s_%s.wak" % (c["name"], side)))
    new = [dict(c, name="%s_%02d" % (c["kind"], len(keep) + i)) for i, c in enumerate(new)]
    print("mld cases:", [(c["name"], c["margin"]) for c in new], flush=True)
    subprocess.run([sys.executable, os.path.join(HERE, "refshim.py")], check=True)
    enc = [("%s_%s" % (c["name"], side), *B.make_pcm(c[side]), "master") for c in new for side in ("a", "b")]
    coded = {}
    with ProcessPoolExecutor(max(1, min(8, os.cpu_count() or 1))) as ex:
        for name, b in ex.map(reference_encode, enc):
            coded[name] = b
            with open(os.path.join(B.OUT, name + ".wak"), "wb") as f:
                f.write(b)
    for c in new:
        for side in ("a", "b"):
            fs, pcm = B.make_pcm(c[side])
            c[side] = dict(c[side], pcm_sha256=B.pcm_sha(pcm),
                           sha256=hashlib.sha256(coded["%s_%s" % (c["name"], side)]).hexdigest())
    man["cases"] = keep + new
    with open(B.MANIFEST, "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print("wrote", B.MANIFEST)


def main_cut15():
    """--cut15: add -15 dB cut cases (L/R-coded bands) to the manifest"""
    man = B.load_manifest()
    rng = np.random.default_rng(1515)
    jobs = []
    for src in SOURCES:
        fs, raw = B.source(src)
        if raw.shape[1] != 2:
            continue
        for off in rng.integers(0, raw.shape[0] - B.FRAMES, 4):
            jobs.append((src, int(off), "alloclr"))
    with ProcessPoolExecutor(max(1, min(8, os.cpu_count() or 1))) as ex:
        found = [c for res in ex.map(search_window, jobs) for c in res if c["kind"] == "cut" and c["cutoff"] == -15.0]
        print("cut -15 brackets:", len(found), flush=True)
        new = sorted([c for c in ex.map(refine2, found[:12]) if c is not None], key=lambda c: c["margin"])[:4]
    n0 = len(man["cases"])
    new = [dict(c, name="cut15_%02d" % (n0 + i)) for i, c in enumerate(new)]
    print("cut15 cases:", [(c["name"], c["margin"]) for c in new], flush=True)
    subprocess.run([sys.executable, os.path.join(HERE, "refshim.py")], check=True)
    enc = [("%s_%s" % (c["name"], side), *B.make_pcm(c[side]), "master") for c in new for side in ("a", "b")]
    coded = {}
    with ProcessPoolExecutor(max(1, min(8, os.cpu_count() or 1))) as ex:
        for name, b in ex.map(reference_encode, enc):
            coded[name] = b
            with open(os.path.join(B.OUT, name + ".wak"), "wb") as f:
                f.write(b)
    for c in new:
        for side in ("a", "b"):
            fs, pcm = B.make_pcm(c[side])
            c[side] = dict(c[side], pcm_sha256=B.pcm_sha(pcm),
                           sha256=hashlib.sha256(coded["%s_%s" % (c["name"], side)]).hexdigest())
    man["cases"] += new
    with open(B.MANIFEST, "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print("wrote", B.MANIFEST)


def main():
    if "--mld" in sys.argv:
        return main_mld()
    if "--cut15" in sys.argv:
        return main_cut15()
    jobs = []
    rng = np.random.default_rng(2026)
    for src in SOURCES:
        fs, raw = B.source(src)
        if raw.shape[1] != 2:
            continue
        for off in rng.integers(0, raw.shape[0] - B.FRAMES, 3):
            off = int(off) // 1024 * 1024 + int(rng.integers(0, 1024))
            off = min(off, raw.shape[0] - B.FRAMES)
            for mode in ("lrms", "alloc", "mld"):
                jobs.append((src, off, mode))
    found = {k: [] for k in WANT}
    with ProcessPoolExecutor(max(1, min(8, os.cpu_count() or 1))) as ex:
        for res in ex.map(search_window, jobs):
            for c in res:
                if c["kind"] in found:
                    found[c["kind"]].append(c)
        print({k: len(v) for k, v in found.items()}, flush=True)
        # every bracket refined toward its threshold, then the closest of each
        # kind (cut: half of them at the M/S cutoff -5 when found)
        cases = []
        for k, n in WANT.items():
            lst = found[k][:2 * n]
            if k != "budget":
                lst = [c for c in ex.map(refine2, lst) if c is not None]
                lst = sorted(lst, key=lambda c: c["margin"])
            if k == "cut":
                m5 = [c for c in lst if c["cutoff"] == -5.0][:n // 2]
                lst = m5 + [c for c in lst if c not in m5]
            cases += lst[:n]
    cases = [dict(c, name="%s_%02d" % (c["kind"], i)) for i, c in enumerate(cases)]
    print("cases:", len(cases), {k: sum(c["kind"] == k for c in cases) for k in WANT}, flush=True)

    subprocess.run([sys.executable, os.path.join(HERE, "refshim.py")], check=True)
    os.makedirs(B.OUT, exist_ok=True)
    enc = []
    for c in cases:
        for side in ("a", "b"):
            fs, pcm = B.make_pcm(c[side])
            enc.append(("%s_%s" % (c["name"], side), fs, pcm, "master"))
    for D, fs, prof in LSB_DENSE:
        enc.append(("lsbdense%d_%dk_%s" % (D, fs // 1000, prof), fs, B.lsb_dense_pcm(fs, D), prof))
    man = {"generated_by": "tests/golden/make_boundary_golden.py (CPU oracle search + reference shim)",
           "frames": B.FRAMES, "cases": [], "lsbdense": {}}
    coded = {}
    with ProcessPoolExecutor(max(1, min(8, os.cpu_count() or 1))) as ex:
        for name, b in ex.map(reference_encode, enc):
            coded[name] = b
            ext = "pac" if name.endswith("origin") else "wak"
            with open(os.path.join(B.OUT, name + "." + ext), "wb") as f:
                f.write(b)
    for c in cases:
        e = dict(c)
        for side in ("a", "b"):
            fs, pcm = B.make_pcm(c[side])
            e[side] = dict(c[side], pcm_sha256=B.pcm_sha(pcm),
                           sha256=hashlib.sha256(coded["%s_%s" % (c["name"], side)]).hexdigest())
        man["cases"].append(e)
    for D, fs, prof in LSB_DENSE:
        name = "lsbdense%d_%dk_%s" % (D, fs // 1000, prof)
        man["lsbdense"][name] = {"D": D, "fs": fs, "profile": prof, "pcm_sha256": B.pcm_sha(B.lsb_dense_pcm(fs, D)),
                                 "sha256": hashlib.sha256(coded[name]).hexdigest()}
    with open(B.MANIFEST, "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print("wrote", B.MANIFEST)


if __name__ == "__main__":
    main()
