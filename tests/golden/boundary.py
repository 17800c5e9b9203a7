"""Decision-boundary parity cases: shared by the generator
(tests/golden/make_boundary_golden.py), the CPU checks
(tests/test_boundary_oracle.py) and the GPU tests (tests/test_gpu_boundary.py).

TEST INFRASTRUCTURE (uses the CPU oracle, oracle/pyoracle.py, as the checker).

A case is a PAIR of short stereo streams (two hops: three blocks with the
Close() flush) that differ in ONE int16 sample by one LSB -- the finest step
real input has -- and across which the oracle's coder takes a different
decision:

  lrms    a band's L/R vs M/S flag, |sum(L^2 - R^2)| < 0.8 |sum(L^2 + R^2)|
          (codec.py:94-102), found by bisecting the right channel's gain;
  argmax  BitAlloc's first argmax over the valid bands of SMR - 6 bits
          (bitalloc.py:157-166), a common gain bisected;
  cut     BitAlloc's band invalidation max_all(SMR - 6 (bits - 1)) < -5 (M/S
          band) / -15 (L/R band) (bitalloc.py:167-173);
  budget  the allocation step's totalBits - nLines >= 0 (bitalloc.py:174-181);
  mld     a 64-line row of an MLD threshold going from "not needed" to
          "needed" because on its one deciding line min(BTHR_S, BTHR_S_MLD *
          mld) (psychoac.py:582-591) starts taking the MLD value -- the
          decision k_master_thr's lower-bound prune takes (pac_wave.h
          PAC_PRUNE_MARGIN); refined by more single-LSB changes toward
          MLD = BTHR_S (relative, as intensities);
  mldneed the same row transition because on its deciding line BTHR_S and
          BTHR_M change order (the line becomes able to need MLD_S at all) --
          the decision of k_master_thr's MLD-need pass (BTHR_M > BTHR_S).

Inputs are regenerated, not stored: a window of a stereo reference input
(tests/fixtures/inputs), each channel scaled by an exact gain (float.hex) and
rounded to int16, plus the listed single-sample changes.  The manifest keeps
the sha256 of every stream's PCM and of the reference's own encode of it
(tests/golden/boundary/, made by the reference coder through the refshim).
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)
import pyoracle as P  # noqa: E402

FRAMES = 2 * 1024
MANIFEST = os.path.join(HERE, "boundary_manifest.json")
OUT = os.path.join(HERE, "boundary")
INPUTS = os.path.join(ROOT, "tests", "fixtures", "inputs")
BIT_BUDGET = 2.27 * 1024 - 4 * (25 + 1) - 4 * 25 - 4        # codec.py:222-226, this op order
PRUNE_REL = 2.0 ** -30

_src = {}


def source(name):
    if name not in _src:
        fs, nch, n, pcm = P.read_wav(os.path.join(INPUTS, name))
        _src[name] = (fs, pcm)
    return _src[name]


def make_pcm(spec):
    """(sample rate, int16 [FRAMES, 2]) of a case stream"""
    fs, pcm = source(spec["src"])
    x = pcm[spec["off"]:spec["off"] + FRAMES].astype(np.float64)
    g = [float.fromhex(spec["gL"]), float.fromhex(spec["gR"])]
    y = np.stack([np.rint(x[:, 0] * g[0]), np.rint(x[:, 1] * g[1])], 1)
    for f, c, d in spec.get("pert", []):
        y[f, c] += d
    return fs, np.clip(y, -32768, 32767).astype(np.int16)


def pcm_sha(pcm):
    return hashlib.sha256(np.ascontiguousarray(pcm, dtype="<i2").tobytes()).hexdigest()


_lut = None


def to_float(pcm):
    """ReadDataBlock + vDequantizeUniform (the oracle's own conversion)"""
    global _lut
    if _lut is None:
        L = P.lib()
        _lut = np.array([L.pac_oracle_pcm_to_float(c) for c in range(-32768, 32768)])
    return _lut[pcm.astype(np.int32) + 32768]


def full_blocks(pcm):
    """the coder's 2048-sample blocks (priorBlock ++ hop; zero first prior,
    zero-padded last hop, the Close() flush block), [nb][2][2048]"""
    x = to_float(pcm)
    hops = -(-x.shape[0] // 1024)
    pad = np.zeros((hops * 1024, 2))
    pad[:x.shape[0]] = x
    seq = np.concatenate([np.zeros((1024, 2)), pad, np.zeros((1024, 2))])
    return [seq[1024 * t:1024 * t + 2048].T.copy() for t in range(hops + 1)]


def oracle_blocks(fs, pcm):
    """the oracle's per-block decisions (StBlock) of a stream, in order"""
    o = P.Oracle(fs, huffman=True)
    st = P.State()
    out = []
    for xb in full_blocks(pcm):
        out.append(o.block_master(xb[0], xb[1], st))
    return out


def key_alloc(blocks):
    return tuple((tuple(b.lrms), tuple(b.ba[0]), tuple(b.ba[1])) for b in blocks)


def key_lrms(blocks):
    return tuple(tuple(b.lrms) for b in blocks)


def band_layout(fs):
    nl = P.Oracle(fs, huffman=False).nlines()
    lo = np.concatenate([[0], np.cumsum(nl)[:-1]])
    return nl, lo


def mld_factor(fs):
    """MLD_F(MDCT freqs) (psychoac.py:349-372), as the oracle builds it"""
    f = (np.arange(1024) + 0.5) / 1024 * (fs / 2.0)
    v = np.power(10.0, 1.25 * (1 - np.cos(np.pi * (np.minimum(f, 3000.0) / 3000.0))) - 2.5)
    return v / v.max()


def mld_lines(b, fs):
    """per line: d_S = BTHR_S_MLD * mld - BTHR_S where BTHR_S > BTHR_M (the
    line needs MLD_S iff d_S < 0), d_M likewise; nan where the line cannot
    need it.  In dB (the reference's units)"""
    th = np.array([b.bthr[v][:] for v in range(6)])
    m = mld_factor(fs)
    dS = np.where(th[3] > th[2], th[5] * m - th[3], np.nan)
    dM = np.where(th[2] > th[3], th[4] * m - th[2], np.nan)
    return dM, dS


def ms_rows(b, fs):
    """64-line rows that M/S-coded bands use (k_master_lrms rowm >> 16)"""
    nl, lo = band_layout(fs)
    rows = 0
    for band in range(25):
        if b.lrms[band] and nl[band]:
            for r in range(lo[band] // 64, (lo[band] + nl[band] - 1) // 64 + 1):
                rows |= 1 << r
    return rows


def key_mld(blocks, fs):
    """per block: the MLD rows needed (bits 0-15 MLD_M, 16-31 MLD_S) among
    the rows M/S bands use"""
    out = []
    for b in blocks:
        dM, dS = mld_lines(b, fs)
        rows = ms_rows(b, fs)
        k = 0
        for r in range(16):
            if not (rows >> r) & 1:
                continue
            if np.any(dM[64 * r:64 * r + 64] < 0):
                k |= 1 << r
            if np.any(dS[64 * r:64 * r + 64] < 0):
                k |= 1 << (16 + r)
        out.append(k)
    return tuple(out)


def bitalloc_trace(smr, lrms, nlines, extra):
    """master BitAlloc (bitalloc.py:129-184) with every decision recorded:
    (bits, bitDifference, steps); a step = (im, gap to the runner-up, gmax,
    cutoff, cut, fits, the bits before the step)"""
    bits = [0] * 25
    valid = [True] * 25
    total = int(BIT_BUDGET + extra)
    steps = []
    while any(valid):
        im, best, second = -1, 0.0, -np.inf
        for b in range(25):
            if not valid[b]:
                continue
            v = smr[b] - bits[b] * 6.
            if im < 0 or v > best:
                if im >= 0:
                    second = max(second, best)
                im, best = b, v
            else:
                second = max(second, v)
        gmax = max(smr[b] - (bits[b] - 1) * 6. for b in range(25))
        cutoff = -5.0 if lrms[im] else -15.0
        cut = gmax < cutoff
        snap = tuple(bits)
        if cut:
            valid[im] = False
        fits = total - nlines[im] >= 0
        if fits:
            bits[im] += 1
            total -= nlines[im]
            if bits[im] >= 16:
                valid[im] = False
        else:
            valid[im] = False
        steps.append((im, best - second, gmax, cutoff, cut, fits, snap))
    for b in range(25):
        if bits[b] == 1:
            total += nlines[b]
            bits[b] = 0
    return bits, total - extra, steps


def lrms_ratio(xb, fs, band):
    """|sum(L^2 - R^2)| / |sum(L^2 + R^2)| of a band (numpy, as codec.py:94-102)"""
    nl, lo = band_layout(fs)
    L, R = np.fft.fft(xb[0]), np.fft.fft(xb[1])
    s = slice(lo[band], lo[band] + nl[band])
    return abs(np.sum(L[s] ** 2 - R[s] ** 2)) / abs(np.sum(L[s] ** 2 + R[s] ** 2))


def traces(fs, b):
    """both channels' BitAlloc traces of one block (the ch1 call sees ch0's
    bitDifference in extraBits, codec.py:257-260)"""
    nl, _ = band_layout(fs)
    out, ex = [], b.extra_in
    for ch in range(2):
        tr = bitalloc_trace(list(b.smr[ch]), list(b.lrms), nl, ex)
        assert tr[0] == list(b.ba[ch]), "BitAlloc trace != oracle"
        out.append(tr)
        ex += tr[1]
    return out


def classify(fs, pcm1, pcm2, b1, b2):
    """which decision differs first between the two streams' oracle runs:
    {"kind", "block", "detail", ...the fields signed_margin needs}"""
    for t, (x, y) in enumerate(zip(b1, b2)):
        if tuple(x.lrms) != tuple(y.lrms):
            band = next(b for b in range(25) if x.lrms[b] != y.lrms[b])
            return {"kind": "lrms", "block": t, "band": band, "detail": "band %d" % band}
        if x.extra_in != y.extra_in:
            return {"kind": "carry", "block": t, "detail": "reservoir"}
        tx, ty = traces(fs, x), traces(fs, y)
        for ch in range(2):
            for i, (sx, sy) in enumerate(zip(tx[ch][2], ty[ch][2])):
                if sx[0] != sy[0]:
                    return {"kind": "argmax", "block": t, "ch": ch, "step": i, "bands": [sx[0], sy[0]],
                            "detail": "ch %d step %d: band %d vs %d" % (ch, i, sx[0], sy[0])}
                if sx[4] != sy[4]:
                    return {"kind": "cut", "block": t, "ch": ch, "step": i, "cutoff": sx[3],
                            "detail": "ch %d step %d: cutoff %g" % (ch, i, sx[3])}
                if sx[5] != sy[5]:
                    return {"kind": "budget", "block": t, "ch": ch, "step": i, "detail": "ch %d step %d" % (ch, i)}
            if tx[ch][0] != ty[ch][0]:
                return {"kind": "other", "block": t, "detail": "ch %d" % ch}
    return None


def decision(case, fs, blocks):
    """the case's own decision in one stream's oracle run: the band's LRMS
    flag; the argmax band or the cut at (block, channel, step); the block's
    MLD row mask"""
    b = blocks[case["block"]]
    k = case["kind"]
    if k == "lrms":
        return b.lrms[case["band"]]
    if k in ("mld", "mldneed"):
        return key_mld(blocks, fs)[case["block"]]
    tr = traces(fs, b)[case["ch"]][2]
    if case["step"] >= len(tr):
        return None
    return tr[case["step"]][0] if k == "argmax" else (tr[case["step"]][4], tr[case["step"]][5])


def signed_margin(case, fs, pcm, blocks=None):
    """how far a stream sits from the case's decision threshold, signed (the
    sign is the decision): lrms -- ratio / 0.8 - 1 (numpy FFT); argmax -- the
    two bands' SMR - 6 bits difference at the step (dB); cut -- max_all(SMR -
    6 (bits - 1)) - cutoff (dB); mld -- MLD / M-S threshold - 1 as
    intensities; mldneed -- BTHR_S / BTHR_M - 1 (MLD_S; the reverse for
    MLD_M) as intensities.  None where the step no longer exists."""
    b = (blocks or oracle_blocks(fs, pcm))[case["block"]]
    k = case["kind"]
    if k == "lrms":
        return lrms_ratio(full_blocks(pcm)[case["block"]], fs, case["band"]) / 0.8 - 1.0
    if k in ("mld", "mldneed"):
        m = case["mld"]
        th = np.array([b.bthr[v][m["line"]] for v in range(6)])
        hi, lo = (th[3], th[2]) if m["var"] == "S" else (th[2], th[3])
        if k == "mldneed":            # the line's eligibility: BTHR_S > BTHR_M (MLD_S), or the reverse
            return float(np.expm1((hi - lo) * np.log(10) / 10))
        if not hi > lo:
            return None
        mld = th[5 if m["var"] == "S" else 4] * mld_factor(fs)[m["line"]]
        return float(np.expm1((mld - hi) * np.log(10) / 10))
    tr = traces(fs, b)[case["ch"]][2]
    if case["step"] >= len(tr):
        return None
    st = tr[case["step"]]
    if k == "argmax":
        b1, b2 = case["bands"]
        smr = list(b.smr[case["ch"]])
        return (smr[b1] - st[6][b1] * 6.) - (smr[b2] - st[6][b2] * 6.)
    if k == "cut":
        return st[2] - st[3]
    return None


def load_manifest():
    with open(MANIFEST) as f:
        return json.load(f)


LSB_FRAMES = 200 * 1024 - 317
LSB_SEED = 2026


def lsb_dense_pcm(fs, D):
    """Dense few-LSB M/S streams (the sparse "lsb" kind barely
    moves the allocation): L = B, the msx base (pink noise + tones), and
    R = B + d with d uniform in {-D .. D} on EVERY sample.  S = -d/2 is then
    white noise of a few LSB: at D = 8 the S channel gets bits in ~2 bands of
    most blocks (its SMR clears the -5 dB M/S cut of bitalloc.py:167-173),
    at D = 4 rarely -- its S SMRs sit just under that cut."""
    from pac_amd import synth
    base = synth.pink_tones_pcm(LSB_FRAMES, fs, LSB_SEED)
    b = base[:, 0].astype(np.int64)
    d = np.random.default_rng(LSB_SEED + D).integers(-D, D + 1, LSB_FRAMES)
    return np.clip(np.stack([b, b + d], 1), -32767, 32767).astype(np.int16)
