"""GPU parity of the master path at the geometry the bench measures, and of
the master profile on every reference input (BASELINE configs[3]'s file
batch), against the CPU oracle.  Bar: bit-exact bytes and reservoir states.

Headline geometry (`pac_abi.hip` `run_master`, no env overrides): 6 000
streams in one call, so every chunk of the default 32 768 blocks holds more
than PAC_WIDE_MAX = 4 096 streams until the ragged ones end -- the one-lane
`k_master_tail` over ~94 tail waves, the `i % 3` / `i & 1` buffer rotation
over >= 5 chunks, the `s_setprio` co-running of the tail and `k_master_emit`
beside the thresholds, the emission's per-wave bump allocation over thousands
of waves -- and then the wide tail over the long streams' last chunks.  The
streams are sampled across the batch in the library's length order (the tail
lane of a stream is its position in that order): the first and last streams,
the tail-wave boundaries 63/64 and 4 095/4 096, the first and last running
stream of every chunk, plus a stride; 24 of the sampled streams carry
M/S-extreme signals (pac_amd.synth.ms_extreme_pcm: dual-mono, anti-phase, a
silent channel, +-1 LSB differences, DC pairs) instead of pink noise + tones.

Reference: `codec/codec.py:83-129,222-260`, `codec/Huffman.py:353-371`,
`codec/pacfile.py:273-366,388-503`.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from conftest import fixture

import pac_amd  # noqa: F401
from pac_amd import _lib, pacfile, synth
import pyoracle as P

pytestmark = pytest.mark.gpu
MASTER = pacfile.PROFILE_MASTER
POOL = max(1, min(16, os.cpu_count() or 1))
CHUNK = 32768          # run_master's default chunk (no block switching)
WIDE_MAX = 4096        # PAC_WIDE_MAX: chunks of more streams take the one-lane tail


def _chunk_geometry(blocks):
    """run_master's chunks of one group: (t0, S, running streams), streams
    ordered by length, longest first (std::stable_sort)"""
    order = np.argsort(-blocks, kind="stable")
    srt = blocks[order]
    gmax = max(1, int(srt[0]))
    n_act, t0, out = len(srt), 0, []
    while t0 < gmax:
        while n_act > 1 and srt[n_act - 1] <= t0:
            n_act -= 1
        S = max(1, min(CHUNK // n_act, gmax - t0))
        out.append((t0, S, n_act))
        t0 += S
    return order, out


def _sample_positions(ns, chunks, stride):
    pos = {0, 1, 62, 63, 64, 65, 127, 128, 4094, 4095, 4096, 4097, ns - 2, ns - 1}
    for _, _, n_act in chunks:
        pos.update({n_act - 1, n_act - 64, max(0, n_act - 65)})
    pos.update(range(0, ns, stride))
    return sorted(p for p in pos if 0 <= p < ns)


def test_master_headline_geometry_vs_oracle(ctx):
    fs, ns = 48000, 6000
    rng = np.random.default_rng(4242)
    hops = np.full(ns, 23, dtype=np.int64)                       # 24 blocks with the Close() flush
    ragged = rng.choice(ns, 1000, replace=False)
    hops[ragged] = rng.integers(5, 48, ragged.size)              # 6 .. 48 blocks
    frames = hops * 1024 - rng.integers(0, 1024, ns)             # zero-padded last hops
    fo = np.zeros(ns + 1, dtype=np.int64)
    fo[1:] = np.cumsum(frames)
    blocks = (frames + 1023) // 1024 + 1
    order, chunks = _chunk_geometry(blocks)
    one_lane = [c for c in chunks if c[2] > WIDE_MAX]
    assert len(chunks) >= 6 and len(one_lane) >= 4, chunks     # the geometry this test is for
    assert one_lane[0][2] // 64 >= 93

    st0 = [_lib.StreamState() for _ in range(ns)]
    ex0 = rng.integers(-40, 40, ns)
    dp0 = rng.integers(-300, 3000, ns)
    for s, e, d in zip(st0, ex0, dp0):
        s.extra_bits, s.bit_deposit = int(e), int(d)

    nframes = int(fo[-1])
    pcm_dev = ctx.alloc(nframes * 4)
    cap = int(blocks.sum()) * 2 * 1024
    out_dev = ctx.alloc(cap)
    try:
        ctx.synth_pink_tones(pcm_dev, nframes, fs, seed=777)
        # M/S extremes (dual-mono, anti-phase, a silent channel, +-1 LSB, DC
        # pairs, mixed) over sampled streams of the call, in the one-lane tail
        # and the wide tail alike: codec.py:94-102, psychoac.py:549-591
        sample = [int(order[k]) for k in _sample_positions(ns, chunks, 97)]
        sample = sorted(set(sample) | {0, ns - 1})
        extreme = {i: synth.MS_EXTREMES[k % len(synth.MS_EXTREMES)]
                   for k, i in enumerate(sample[::max(1, len(sample) // 24)])}
        for i, kind in extreme.items():
            ctx.to_device(pcm_dev + int(fo[i]) * 4, synth.ms_extreme_pcm(kind, int(frames[i]), fs, seed=1000 + i))
        p = _lib.params(fs, 2, MASTER)
        _, so = ctx.encode_streams(p, pcm_dev, fo, out=out_dev, out_capacity=cap, pcm_is_device=True,
                                   out_is_device=True, states=st0)
        body = np.empty(int(so[-1]), dtype=np.uint8)
        ctx.to_host(body, out_dev)
        # every stream's data section: 2 x blocks channel-blocks of <L nBytes> + payload
        for i in range(ns):
            pos, end, n = int(so[i]), int(so[i + 1]), 0
            while pos < end:
                pos += 4 + int.from_bytes(body[pos:pos + 4].tobytes(), "little")
                n += 1
            assert pos == end and n == 2 * blocks[i], "stream %d: framing" % i
        assert len(sample) >= 64 and len(extreme) >= 24
        pcms = {}
        for i in sample:
            a = np.empty((int(frames[i]), 2), dtype=np.int16)
            ctx.to_host(a, pcm_dev + int(fo[i]) * 4)
            pcms[i] = a
    finally:
        ctx.free(out_dev)
        ctx.free(pcm_dev)

    def one(i):
        st = P.State(int(ex0[i]), int(dp0[i]))
        data = P.Oracle(fs, huffman=True).encode_data(P.MASTER, pcms[i], state=st)
        return data, (st.extraBits, st.deposit)

    with ThreadPoolExecutor(POOL) as ex:
        ref = dict(zip(sample, ex.map(one, sample)))
    rank = np.empty(ns, dtype=np.int64)
    rank[order] = np.arange(ns)
    bad = [(i, int(rank[i])) for i in sample if body[so[i]:so[i + 1]].tobytes() != ref[i][0]]
    assert not bad, "streams (index, length rank) differ from the oracle: %s" % bad[:10]
    bad = [i for i in sample if (st0[i].extra_bits, st0[i].bit_deposit) != ref[i][1]]
    assert not bad, "reservoir states differ: %s" % bad[:10]


INPUTS = sorted(f for f in os.listdir(os.path.dirname(fixture("harpsichord.wav"))) if f.endswith(".wav"))


def test_master_all_reference_inputs_vs_oracle(ctx):
    """The 22 reference inputs (all 44.1 kHz stereo: configs[3]'s file batch)
    as independent streams of one pac_encode_wav call, whole files, against
    the oracle -- castanets, daft, german, trumpet, piano1, piano_test1,
    pop_test3, rock_test3 and speech_test1 have no master .wak in the
    reference; the other 13 are also pinned by its files."""
    assert len(INPUTS) == 22
    paths = [fixture(n) for n in INPUTS]
    got = pacfile.encode_wav_files(paths, profile=MASTER, context=ctx)

    def one(path):
        return P.encode_file(path, P.MASTER)

    with ThreadPoolExecutor(POOL) as ex:
        ref = list(ex.map(one, paths))
    bad = [n for n, g, r in zip(INPUTS, got, ref) if g != r]
    assert not bad, bad


def test_front_mdct_paths_agree_on_reference_inputs(ctx):
    """The default front takes its MDCT lines from the LRMS spectra
    (mdct_from_dft); PAC_FRONT_FAST=0 transforms in the front.
    Both give the same bytes on every reference input."""
    paths = [fixture(n) for n in INPUTS]
    fast = pacfile.encode_wav_files(paths, profile=MASTER, context=ctx)
    old = os.environ.get("PAC_FRONT_FAST")
    os.environ["PAC_FRONT_FAST"] = "0"
    try:
        c2 = _lib.Context(0)
    finally:
        if old is None:
            del os.environ["PAC_FRONT_FAST"]
        else:
            os.environ["PAC_FRONT_FAST"] = old
    try:
        slow = pacfile.encode_wav_files(paths, profile=MASTER, context=c2)
    finally:
        c2.close()
    bad = [n for n, a, b in zip(INPUTS, fast, slow) if a != b]
    assert not bad, bad


@pytest.mark.parametrize("env", [{"PAC_MLD_SKIP": "0"},          # every MLD row, the pairs in one launch (mode 0)
                                 {"PAC_TAIL_MODE": "serial"},    # every kernel on one stream, in order
                                 {"PAC_SIDE_FUSED": "0"},        # LRMS and spectra as two kernels
                                 {"PAC_FRONT_LATE": "1"},        # front(i) beside thr(i+1), thresholds double-buffered
                                 {"PAC_SIDE_EARLY": "1"},        # side(i+2) beside thr(i+1), spectra double-buffered
                                 {"PAC_TAIL_EARLY": "1"},        # tail(i) right after front(i)
                                 {"PAC_SIDE_CODED": "0"}])       # coded lines formed by the front, not the side kernel
def test_schedules_agree_on_reference_inputs(ctx, env):
    """The pipelined default (the MLD skip with its row mask, four streams, the
    fused side kernel) and the alternative schedules give the same bytes on
    every reference input (the default is pinned to the oracle above)."""
    paths = [fixture(n) for n in INPUTS]
    base = pacfile.encode_wav_files(paths, profile=MASTER, context=ctx)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        c2 = _lib.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    try:
        alt = pacfile.encode_wav_files(paths, profile=MASTER, context=c2)
    finally:
        c2.close()
    bad = [n for n, a, b in zip(INPUTS, base, alt) if a != b]
    assert not bad, bad
