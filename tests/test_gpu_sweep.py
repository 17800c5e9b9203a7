"""Wider GPU parity sweep: many blocks of varied material (noise at several
levels, pink noise + tones, chirps, decaying tone bursts, silence gaps,
clipped full-scale noise) at 32/44.1/48 kHz, both profiles, against the CPU
oracle.  Bars: bit-exact bytes; thresholds within 1e-11 dB
over every block (the GPU evaluates the masking sum in factored forms, see
csrc/pac_wave.h).  The oracle runs in a thread pool (ctypes releases the GIL).
"""
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import pac_amd  # noqa: F401
from pac_amd import pacfile, synth
from pac_amd.pcmfile import codes_to_float
import pyoracle as P

pytestmark = pytest.mark.gpu

POOL = 8


def _i16(x):
    return np.clip(np.rint(x), -32768, 32767).astype(np.int16)


def material(kind, n, fs, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / fs
    if kind.startswith("white"):
        lvl = {"white_loud": 0.25, "white_mid": 0.02, "white_soft": 0.0008}[kind]
        return synth.white_pcm(n, 2, seed=seed, scale=lvl)
    if kind == "pink_tones":
        return synth.pink_tones_pcm(n, fs, seed=seed)
    if kind == "chirp":
        f = 50.0 * (fs / 2 / 50.0) ** (t / t[-1])
        ph = 2 * np.pi * np.cumsum(f) / fs
        x = 0.5 * 32767 * np.sin(ph)
        return _i16(np.stack([x, np.roll(x, 37) * 0.7], 1))
    if kind == "bursts":
        x = np.zeros((n, 2))
        for _ in range(max(1, n // 3000)):
            on = rng.integers(0, n)
            f0 = rng.uniform(80, fs / 3)
            amp = rng.uniform(0.01, 0.6) * 32767
            d = np.arange(n - on) / fs
            env = np.exp(-d * rng.uniform(2, 30))
            for k in range(1, 6):
                if k * f0 < fs / 2:
                    x[on:, 0] += amp / k * env * np.sin(2 * np.pi * k * f0 * d)
                    x[on:, 1] += amp / k * env * np.sin(2 * np.pi * k * f0 * d + k)
        return _i16(x)
    if kind == "gaps":
        x = synth.white_pcm(n, 2, seed=seed, scale=0.1).astype(np.float64)
        mask = (np.arange(n) // 3000) % 2 == 0
        return _i16(x * mask[:, None])
    if kind == "clipped":
        return synth.white_pcm(n, 2, seed=seed, scale=1.5)
    raise ValueError(kind)


KINDS = ["white_loud", "white_mid", "white_soft", "pink_tones", "chirp", "bursts", "gaps", "clipped"]


def _streams(fs, seed0, blocks):
    rng = np.random.default_rng(seed0)
    out = []
    for i, k in enumerate(KINDS):
        n = int(blocks * 1024 + rng.integers(0, 1024))
        out.append(material(k, n, fs, seed0 + i))
    return out


def _oracle(profile, fs, streams, huffman):
    def one(s):
        return P.Oracle(fs, huffman=huffman).encode_data(profile, s)
    with ThreadPoolExecutor(POOL) as ex:
        return list(ex.map(one, streams))


@pytest.mark.parametrize("fs", [48000, 44100, 32000])
def test_origin_sweep_vs_oracle(ctx, fs):
    streams = _streams(fs, 100 + fs // 1000, 300)
    got = pacfile.encode_streams(streams, fs, pacfile.PROFILE_ORIGIN, context=ctx)
    exp = _oracle(P.ORIGIN, fs, streams, False)
    for k, g, e in zip(KINDS, got, exp):
        assert g == e, k


@pytest.mark.parametrize("fs", [48000, 44100])
def test_master_sweep_vs_oracle(ctx, fs):
    streams = _streams(fs, 200 + fs // 1000, 200)
    got = pacfile.encode_streams(streams, fs, pacfile.PROFILE_MASTER, context=ctx)
    exp = _oracle(P.MASTER, fs, streams, True)
    for k, g, e in zip(KINDS, got, exp):
        assert g == e, k


@pytest.mark.parametrize("fs", [48000, 44100])
def test_threshold_sweep(ctx, fs):
    """calcBTHR on 8 x 48 windowed blocks of every kind, both drop settings."""
    win = np.sin((np.arange(2048) + 0.5) * np.pi / 2048)
    blocks = []
    for i, k in enumerate(KINDS):
        pcm = material(k, 48 * 2048, fs, 900 + i)[:, 0]
        blocks.append(codes_to_float(pcm.astype(np.int64)).reshape(48, 2048) * win)
    data = np.concatenate(blocks)
    tl = threading.local()

    def oracle():
        if not hasattr(tl, "o"):
            tl.o = P.Oracle(fs, huffman=False)
        return tl.o
    for no_drop in (False, True):
        thr, npk = ctx.debug_threshold(fs, data, no_drop)

        def one(i):
            ref, peaks, _ = oracle().threshold(data[i], no_drop)
            return len(peaks), float(np.max(np.abs(thr[i] - ref)))
        with ThreadPoolExecutor(POOL) as ex:
            res = list(ex.map(one, range(data.shape[0])))
        assert [r[0] for r in res] == list(npk)
        worst = max(r[1] for r in res)
        assert worst < 1e-11, worst
