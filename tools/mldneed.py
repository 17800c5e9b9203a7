"""How many MLD rows the M/S combination needs (psychoac.py:582-591) on the
bench's device-synthesized pink noise + tones: per block, the M/S rows where
some line has BTHR_M > BTHR_S (MLD_M needed) or BTHR_S > BTHR_M (MLD_S
needed), by the oracle's calcBTHR.  Diagnostic for the threshold kernel's
mode 2; runs on a GPU box (the synthesizer is a HIP kernel)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import pac_amd  # noqa: E402,F401
from pac_amd import _lib  # noqa: E402
import pyoracle as P  # noqa: E402

nblk = int(sys.argv[1]) if len(sys.argv) > 1 else 300
ctx = _lib.Context(0)
nf = 1024 * (nblk + 1)
dev = ctx.alloc(nf * 4)
ctx.synth_pink_tones(dev, nf, 48000, 1234)
pcm = np.empty((nf, 2), dtype=np.int16)
ctx.to_host(pcm, dev)
o = P.Oracle(48000)
x = np.vectorize(o.L.pac_oracle_pcm_to_float)(pcm.reshape(-1)).reshape(pcm.shape)
N = 2048
n = np.arange(N)
sine = np.sin(np.pi * (n + 0.5) / N)
hann = 0.5 * (1 - np.cos(2 * np.pi * (n + 0.5) / N))
nl = o.nlines()
lower = np.concatenate([[0], np.cumsum(nl)[:-1]])
tot = {"ms_rows": 0, "need_mldM": 0, "need_mldS": 0, "blocks_without_mldS": 0, "blocks": 0}
for b in range(1, nblk):
    fL = x[(b - 1) * 1024:(b + 1) * 1024, 0]
    fR = x[(b - 1) * 1024:(b + 1) * 1024, 1]
    L, R = np.fft.fft(fL), np.fft.fft(fR)
    rows = set()
    for k in range(25):
        sl = slice(lower[k], lower[k] + nl[k] + 1)
        if nl[k] and abs(np.sum(L[sl] ** 2 - R[sl] ** 2)) < 0.8 * abs(np.sum(L[sl] ** 2 + R[sl] ** 2)):
            rows.update(range(lower[k] // 64, (lower[k] + nl[k] - 1) // 64 + 1))
    a, c = fL * sine * hann, fR * sine * hann
    bM = o.threshold((a + c) / 2)[0]
    bS = o.threshold((a - c) / 2)[0]
    nM = sum(1 for r in rows if np.any(bM[r * 64:r * 64 + 64] > bS[r * 64:r * 64 + 64]))
    nS = sum(1 for r in rows if np.any(bS[r * 64:r * 64 + 64] > bM[r * 64:r * 64 + 64]))
    tot["ms_rows"] += len(rows)
    tot["need_mldM"] += nM
    tot["need_mldS"] += nS
    tot["blocks_without_mldS"] += (nS == 0)
    tot["blocks"] += 1
print({k: (v / tot["blocks"] if k not in ("blocks",) else v) for k, v in tot.items()})
