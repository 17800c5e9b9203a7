"""Block-switching extension (BASELINE configs[4]).  No
reference coder switches blocks (pacfile.py:23,48), so parity is UNPINNED
against the reference: the HIP path (csrc/pac_bs.h, k_bs_attack / k_bs_flags /
k_master_thr_short and the short branches of k_master_front / k_master_pack /
k_dec_synth) is checked byte for byte against the oracle's restatement of the
same design (oracle/pac_oracle.c, block switching section), whose filterbank
is itself checked for perfect reconstruction and pre-echo reduction on the
CPU (tests/test_oracle.py::test_block_switch_*).  Bar: bit-exact bytes,
reservoir state and decoded samples; the short frames really occur."""
import numpy as np
import pytest

import pac_amd  # noqa: F401
from pac_amd import pacfile, synth, _lib
import pyoracle as P

pytestmark = pytest.mark.gpu
MASTER = pacfile.PROFILE_MASTER


def bursts(n, fs, seed, nch=2, every=7000):
    """pink noise + tones with decaying noise bursts every ~`every` frames"""
    rng = np.random.default_rng(seed)
    x = synth.pink_tones_pcm(n, fs, seed=seed).astype(np.int32)[:, :nch] // 4
    for t0 in range(int(rng.integers(300, 3000)), n, every):
        L = min(2500, n - t0)
        env = np.exp(-np.arange(L) / 500.0)
        for c in range(nch):
            x[t0:t0 + L, c] += (rng.standard_normal(L) * (14000 - 3000 * c) * env).astype(np.int32)
    return np.ascontiguousarray(np.clip(x, -32768, 32767).astype(np.int16))


@pytest.mark.parametrize("fs,window", [(48000, _lib.WINDOW_SINE), (44100, _lib.WINDOW_SINE),
                                       (48000, _lib.WINDOW_KBD)])
def test_bs_streams_vs_oracle(ctx, fs, window):
    lens = [0, 1, 1023, 1024, 5000, 20 * 1024, 33 * 1024 + 17, 60 * 1024]
    streams = [bursts(n, fs, i) for i, n in enumerate(lens)]
    states = [_lib.StreamState() for _ in lens]
    got = pacfile.encode_streams(streams, fs, MASTER, context=ctx, states=states, window=window,
                                 block_switch=True)
    plain = pacfile.encode_streams(streams, fs, MASTER, context=ctx, window=window)
    o = P.Oracle(fs, huffman=True, window=window, block_switch=True)
    nshort = 0
    for i, s in enumerate(streams):
        st = P.State()
        assert got[i] == o.encode_data(P.MASTER, s, state=st), "stream %d differs" % i
        assert (states[i].extra_bits, states[i].bit_deposit) == (st.extraBits, st.deposit)
        nshort += int((o.bs_plan(s) & 1).sum())
        if len(s) >= 20 * 1024:
            assert got[i] != plain[i]
    assert nshort >= 10          # the short path is exercised


def test_bs_decode_vs_oracle(ctx):
    fs = 48000
    streams = [bursts(n, fs, 10 + n) for n in (3000, 17 * 1024 + 3, 40 * 1024)]
    got = pacfile.encode_streams(streams, fs, MASTER, context=ctx, block_switch=True)
    dec = pacfile.decode_streams(got, fs, 2, MASTER, context=ctx, block_switch=True)
    o = P.Oracle(fs, huffman=True, block_switch=True)
    for s, g, d in zip(streams, got, dec):
        ref = o.decode_data(P.MASTER, g, 2)
        assert d.shape == ref.shape
        assert np.array_equal(d, ref)


def test_bs_mono(ctx):
    fs = 44100
    streams = [bursts(n, fs, 20 + i, nch=1) for i, n in enumerate((9000, 30 * 1024 + 5))]
    got = pacfile.encode_streams(streams, fs, MASTER, context=ctx, block_switch=True)
    o = P.Oracle(fs, huffman=True, block_switch=True)
    for s, g in zip(streams, got):
        assert g == o.encode_data(P.MASTER, s)
        assert np.array_equal(pacfile.decode_streams([g], fs, 1, MASTER, context=ctx, block_switch=True)[0],
                              o.decode_data(P.MASTER, g, 1))


def test_bs_chunking_invariance(ctx):
    """Chunked pass 1 (reservoir and short frames across chunk boundaries)."""
    import ctypes as C
    fs = 48000
    streams = [bursts(37 * 1024 + 11, fs, 5), bursts(20 * 1024, fs, 6)]
    full = pacfile.encode_streams(streams, fs, MASTER, context=ctx, block_switch=True)
    small = _lib.Context(0)
    try:
        f = small.L.pac_set_chunk_blocks
        f.argtypes = [C.c_void_p, C.c_int64]
        f(small.h, 7)
        assert pacfile.encode_streams(streams, fs, MASTER, context=small, block_switch=True) == full
    finally:
        small.close()


def test_bs_rejections(ctx):
    fs = 48000
    x = bursts(5000, fs, 1)
    with pytest.raises(_lib.PacError):
        pacfile.encode_streams([x], fs, pacfile.PROFILE_ORIGIN, context=ctx, block_switch=True)
    st = _lib.StreamState()
    st.flags = _lib.STREAM_NO_FLUSH
    with pytest.raises(_lib.PacError):
        pacfile.encode_streams([x], fs, MASTER, context=ctx, states=[st], block_switch=True)
