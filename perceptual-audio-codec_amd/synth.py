"""Synthetic benchmark / test signals (BASELINE.json configs 2-3).

  white_pcm        48 kHz stereo white noise: N(0,1) * 0.25 * 32767, rint, clip
  pink_tones_pcm   pink noise + 440/1250/5300 Hz tones at 0.2/0.1/0.05,
                   R = 0.7 L_pink + 0.3 independent pink + 0.8 tones
  hash_white_pcm   host mirror of the device generator k_synth_white
                   (splitmix64 counter hash + Box-Muller), used by bench.py to
                   fill HBM without a PCIe upload
"""
import numpy as np


def _to_int16(x):
    return np.clip(np.rint(x), -32768, 32767).astype(np.int16)


def white_pcm(n_frames, n_ch=2, seed=1234, scale=0.25):
    rng = np.random.default_rng(seed)
    return _to_int16(rng.standard_normal((int(n_frames), n_ch)) * scale * 32767)


def _pink(rng, n):
    # Voss-McCartney-free spectral shaping: 1/sqrt(f) filter on white noise
    if n == 0:
        return np.zeros(0)
    w = rng.standard_normal(n)
    W = np.fft.rfft(w)
    f = np.arange(len(W), dtype=np.float64)
    f[0] = 1.0
    W /= np.sqrt(f)
    p = np.fft.irfft(W, n)
    return p / (np.std(p) + 1e-30)


def pink_tones_pcm(n_frames, fs=48000, seed=1234, pink_level=0.1):
    rng = np.random.default_rng(seed)
    n = int(n_frames)
    t = np.arange(n) / float(fs)
    tones = (0.2 * np.sin(2 * np.pi * 440 * t) + 0.1 * np.sin(2 * np.pi * 1250 * t)
             + 0.05 * np.sin(2 * np.pi * 5300 * t))
    pl = _pink(rng, n) * pink_level
    pi = _pink(rng, n) * pink_level
    L = pl + tones
    R = 0.7 * pl + 0.3 * pi + 0.8 * tones
    return _to_int16(np.stack([L, R], 1) * 32767)


MS_EXTREMES = ("dualmono", "antiphase", "rsilent", "lsilent", "lsb", "dcpair", "dcpure", "mixed")


def ms_extreme_pcm(kind, n_frames, fs=48000, seed=1234):
    """Stereo streams at the M/S decision's extremes (codec.py:94-102,
    psychoac.py:549-591): one of M = (L+R)/2, S = (L-R)/2 or a channel is
    identically zero, or nearly so.  B is the pink-noise + tones left channel
    kept within [-32767, 32767] so that -B is exact (no -32768 code).

      dualmono   L = R = B                          S == 0, LRMS = 1 in every non-silent band
      antiphase  L = B, R = -B                      M == 0
      rsilent    L = B, R = 0
      lsilent    L = 0, R = B
      lsb        L = B, R = B + sparse +-1 LSB      S tiny but not zero
      dcpair     L = B/2 + 10000, R = B/2 - 10000   S a pure DC offset
      dcpure     L = 10000, R = -3000               constant channels
      mixed      24-block segments cycling through the kinds above, plus
                 digital silence and the decorrelated pink + tones pair
    """
    n = int(n_frames)
    base = pink_tones_pcm(n, fs, seed)
    B = np.maximum(base[:, 0].astype(np.int32), -32767)
    z = np.zeros_like(B)
    if kind == "dualmono":
        L, R = B, B
    elif kind == "antiphase":
        L, R = B, -B
    elif kind == "rsilent":
        L, R = B, z
    elif kind == "lsilent":
        L, R = z, B
    elif kind == "lsb":
        rng = np.random.default_rng(seed + 1)
        d = rng.integers(-1, 2, n) * (rng.random(n) < 1.0 / 256)
        L, R = B, np.clip(B + d, -32767, 32767)
    elif kind == "dcpair":
        L, R = np.clip(B // 2 + 10000, -32767, 32767), np.clip(B // 2 - 10000, -32767, 32767)
    elif kind == "dcpure":
        L, R = z + 10000, z - 3000
    elif kind == "mixed":
        L, R = np.empty_like(B), np.empty_like(B)
        seg = 24 * 1024
        kinds = MS_EXTREMES[:-1] + ("silence", "pinktones")
        for k, s0 in enumerate(range(0, n, seg)):
            kk = kinds[k % len(kinds)]
            s1 = min(n, s0 + seg)
            if kk == "silence":
                L[s0:s1] = R[s0:s1] = 0
            elif kk == "pinktones":
                L[s0:s1], R[s0:s1] = base[s0:s1, 0], base[s0:s1, 1]
            else:
                p = ms_extreme_pcm(kk, n, fs, seed)
                L[s0:s1], R[s0:s1] = p[s0:s1, 0], p[s0:s1, 1]
    else:
        raise ValueError("unknown M/S extreme %r" % kind)
    return np.stack([L, R], 1).astype(np.int16)


_M64 = (1 << 64) - 1


def _splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def hash_white_pcm(n_samples, seed):
    """Host mirror of k_synth_white (pac_kernels.hip): int16[n_samples]."""
    i = np.arange(int(n_samples), dtype=np.uint64)
    s = np.uint64(seed)
    with np.errstate(over="ignore"):
        def sm(x):
            x = x + np.uint64(0x9E3779B97F4A7C15)
            x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            return x ^ (x >> np.uint64(31))
        h1 = sm(s ^ (np.uint64(2) * i))
        h2 = sm(s ^ (np.uint64(2) * i + np.uint64(1)))
    u1 = ((h1 >> np.uint64(11)).astype(np.float64) + 1.0) * 2.0 ** -53
    u2 = (h2 >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    z = np.sqrt(-2.0 * np.log(u1)) * np.cos(6.283185307179586 * u2)
    return _to_int16(z * 0.25 * 32767.0)
