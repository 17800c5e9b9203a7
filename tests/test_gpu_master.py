"""GPU parity of the master profile (codec/: M/S, Huffman, bit reservoir)
against the committed .wak fixture, the reference-generated goldens and the CPU
oracle.  Bar: bit-exact bytes and reservoir state."""
import os

import numpy as np
import pytest

from conftest import GOLD, fixture

import pac_amd  # noqa: F401
from pac_amd import pacfile, _lib, synth
import pyoracle as P

pytestmark = pytest.mark.gpu
MASTER = pacfile.PROFILE_MASTER


def test_piano_test2_wak_bit_exact(ctx):
    """coded/piano_test2.wak (reference fixture) byte for byte."""
    got = pacfile.encode_file(fixture("piano_test2.wav"), profile=MASTER, context=ctx)
    with open(fixture("piano_test2.wak"), "rb") as f:
        ref = f.read()
    assert len(got) == len(ref)
    assert got == ref


@pytest.mark.parametrize("name", ["master_pinktones48k", "master_zero48k", "master_square44k",
                                  "master_white48k"])
def test_golden_reference_streams(ctx, name):
    pcm = np.load(os.path.join(GOLD, name + ".in.npy"))
    with open(os.path.join(GOLD, name + ".wak"), "rb") as f:
        ref = f.read()
    fs = {"48k": 48000, "44k": 44100}[name[-3:]]
    body = pacfile.encode_streams([pcm], fs, MASTER, context=ctx)[0]
    assert pacfile.header_bytes(fs, 2, pcm.shape[0]) + body == ref


def test_harpsichord_master_vs_oracle(ctx):
    """harpsichord.wav through the master coder (no committed golden for it;
    the oracle is pinned on 13 master fixtures)."""
    fs, nch, n, pcm = P.read_wav(fixture("harpsichord.wav"))
    got = pacfile.encode_streams([pcm], fs, MASTER, context=ctx)[0]
    o = P.Oracle(fs, huffman=True)
    assert got == o.encode_data(P.MASTER, pcm)


@pytest.mark.parametrize("fs", [48000, 44100])
def test_multi_stream_vs_oracle_and_state(ctx, fs):
    """Independent streams in one call (each with its own reservoir), ragged
    lengths, plus the returned reservoir state (extraBits, bitDeposit)."""
    lens = [0, 1023, 1024, 3000, 15 * 1024 + 5, 40 * 1024]
    streams = [synth.pink_tones_pcm(n, fs, seed=i + 3) if i % 2 else synth.white_pcm(n, 2, seed=i)
               for i, n in enumerate(lens)]
    states = [_lib.StreamState() for _ in lens]
    got = pacfile.encode_streams(streams, fs, MASTER, context=ctx, states=states)
    o = P.Oracle(fs, huffman=True)
    for i, s in enumerate(streams):
        st = P.State()
        exp = o.encode_data(P.MASTER, s, state=st)
        assert got[i] == exp, "stream %d differs" % i
        assert (states[i].extra_bits, states[i].bit_deposit) == (st.extraBits, st.deposit)


def test_chunking_invariance(ctx):
    """Chunked processing (reservoir carried across chunk boundaries in the
    middle of a stream) gives the same bytes."""
    fs = 48000
    streams = [synth.pink_tones_pcm(37 * 1024 + 11, fs, seed=5), synth.white_pcm(20 * 1024, 2, seed=6)]
    full = pacfile.encode_streams(streams, fs, MASTER, context=ctx)
    lib = ctx.L
    import ctypes as C
    small = _lib.Context(0)
    try:
        small_set = getattr(lib, "pac_set_chunk_blocks")
        small_set.argtypes = [C.c_void_p, C.c_int64]
        small_set(small.h, 7)
        chunked = pacfile.encode_streams(streams, fs, MASTER, context=small)
    finally:
        small.close()
    assert chunked == full


def test_chunk_blocks_bound(ctx):
    """chunks above PAC_CHUNK_MAX (131071 blocks) would wrap the
    tail's 32-bit buffer offsets into zeros -- refused (pac_set_chunk_blocks
    and PAC_CHUNK_BLOCKS alike); the bound itself encodes the same bytes."""
    import ctypes as C
    fs = 48000
    streams = [synth.pink_tones_pcm(9 * 1024 + 5, fs, seed=8), synth.white_pcm(6 * 1024, 2, seed=9)]
    full = pacfile.encode_streams(streams, fs, MASTER, context=ctx)
    c2 = _lib.Context(0)
    try:
        assert ctx.L.pac_set_chunk_blocks(c2.h, C.c_int64(131072)) == _lib.PAC_E_ARG
        assert ctx.L.pac_set_chunk_blocks(c2.h, C.c_int64(131071)) == 0
        assert pacfile.encode_streams(streams, fs, MASTER, context=c2) == full
    finally:
        c2.close()
    c3 = _ctx_with_env(PAC_CHUNK_BLOCKS=131072)
    try:
        with pytest.raises(_lib.PacError):
            pacfile.encode_streams(streams, fs, MASTER, context=c3)
    finally:
        c3.close()


def _ctx_with_env(**env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return _lib.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("env", [{"PAC_DEBUG_STG_BIAS": 5 * 2 ** 30},   # staging offsets past 4 GiB
                                 {"PAC_DEBUG_STG_CAP": 3000}])           # staging overflow -> the pack path
def test_tail_emission_staging(ctx, env):
    """The tail emits each channel-block into a staging buffer (bump-allocated
    per wave) that k_master_place copies to the file offsets: offsets past
    4 GiB, and a staging overflow (the call re-runs through k_master_pack
    from the initial reservoir states), give the same bytes and states."""
    fs = 48000
    lens = [0, 5 * 1024 + 3, 20 * 1024, 33 * 1024 + 700]
    streams = [synth.pink_tones_pcm(n, fs, seed=i + 11) for i, n in enumerate(lens)]
    st0 = [_lib.StreamState() for _ in lens]
    for i, st in enumerate(st0):
        st.extra_bits, st.bit_deposit = 17 * i, 250 * i - 40
    ref_states = [_lib.StreamState() for _ in lens]
    for a, b in zip(ref_states, st0):
        a.extra_bits, a.bit_deposit = b.extra_bits, b.bit_deposit
    ref = pacfile.encode_streams(streams, fs, MASTER, context=ctx, states=ref_states)
    c2 = _ctx_with_env(**env)
    try:
        got = pacfile.encode_streams(streams, fs, MASTER, context=c2, states=st0)
    finally:
        c2.close()
    assert got == ref
    assert [(s.extra_bits, s.bit_deposit) for s in st0] == [(s.extra_bits, s.bit_deposit) for s in ref_states]
    o = P.Oracle(fs, huffman=True)
    for i in (1, 3):                                   # and the oracle from the same initial states
        st = P.State(17 * i, 250 * i - 40)
        assert got[i] == o.encode_data(P.MASTER, streams[i], state=st)
        assert (st.extraBits, st.deposit) == (st0[i].extra_bits, st0[i].bit_deposit)


@pytest.mark.parametrize("wide", [0, 1])
def test_tail_variants_vs_oracle(ctx, wide):
    """Both reservoir tails -- one lane per stream (many streams) and one wave
    per stream (few streams, the default below PAC_WIDE_MAX) -- give the
    oracle's bytes and reservoir states on ragged streams."""
    fs = 44100
    lens = [0, 700, 1024, 9 * 1024 + 77, 22 * 1024, 31 * 1024 + 5]
    streams = [synth.pink_tones_pcm(n, fs, seed=40 + i) if i % 2 else synth.white_pcm(n, 2, seed=50 + i)
               for i, n in enumerate(lens)]
    states = [_lib.StreamState() for _ in lens]
    for i, st in enumerate(states):
        st.extra_bits, st.bit_deposit = 5 * i, 300 * i - 7
    c2 = _ctx_with_env(PAC_TAIL_WIDE=wide)
    try:
        got = pacfile.encode_streams(streams, fs, MASTER, context=c2, states=states)
    finally:
        c2.close()
    o = P.Oracle(fs, huffman=True)
    for i, pcm in enumerate(streams):
        st = P.State(5 * i, 300 * i - 7)
        assert got[i] == o.encode_data(P.MASTER, pcm, state=st), "stream %d" % i
        assert (states[i].extra_bits, states[i].bit_deposit) == (st.extraBits, st.deposit)


def test_plugin_surface_per_block_matches(ctx, tmp_path):
    """PACFile.WriteDataBlock per hop with the Huffman reservoir object, as the
    reference driver runs it (pacfile.py:474-499), equals the fixture prefix."""
    from pac_amd.pcmfile import PCMFile
    from pac_amd.huffman import Huffman
    huffman = Huffman()
    out = tmp_path / "p.wak"
    inFile = PCMFile(fixture("piano_test2.wav"))
    outFile = pacfile.PACFile(str(out), profile=MASTER, context=ctx)
    cp = inFile.OpenForReading()
    cp.nMDCTLines, cp.nScaleBits, cp.nMantSizeBits = 1024, 4, 4
    cp.targetBitsPerSample, cp.nTableIDBits = 2.27, 4
    cp.nSamplesPerBlock = cp.nMDCTLines
    outFile.OpenForWriting(cp)
    for _ in range(30):
        data = inFile.ReadDataBlock(cp)
        if not data:
            break
        outFile.WriteDataBlock(data, cp, huffman)
    outFile.fp.close()
    got = out.read_bytes()
    with open(fixture("piano_test2.wak"), "rb") as f:
        ref = f.read()
    assert got == ref[:len(got)]


def test_codec_encode_tuple_master(ctx):
    """codec.Encode (codec.py:83-129) tuple fields vs the oracle for a block."""
    from pac_amd import codec
    from pac_amd.audiofile import CodingParams
    from pac_amd.huffman import Huffman
    from pac_amd.psychoac import ScaleFactorBands, AssignMDCTLinesFromFreqLimits
    from pac_amd.pcmfile import codes_to_float
    fs = 48000
    pcm = synth.pink_tones_pcm(4 * 1024, fs, seed=9)
    x = [codes_to_float(pcm[1024:3072, c]) for c in range(2)]
    cp = CodingParams()
    cp.sampleRate, cp.nChannels, cp.nMDCTLines = fs, 2, 1024
    cp.nScaleBits, cp.nMantSizeBits, cp.targetBitsPerSample, cp.nTableIDBits = 4, 4, 2.27, 4
    cp.sfBands = ScaleFactorBands(AssignMDCTLinesFromFreqLimits(1024, fs))
    cp.extraBits = 17
    h = Huffman()
    h.bitDeposit = 1234
    sf, ba, signs, codes, tid, overall, lrms = codec.Encode(x, cp, h, profile=codec.PROFILE_MASTER,
                                                            context=ctx)
    o = P.Oracle(fs, huffman=True)
    st = P.State()
    st.extraBits, st.deposit = 17, 1234
    ob = o.block_master(x[0], x[1], st)
    assert list(lrms) == list(ob.lrms)
    assert (cp.extraBits, h.bitDeposit) == (st.extraBits, st.deposit)
    for c in range(2):
        assert overall[c] == ob.overall[c]
        assert tid[c] == ob.table_id[c]
        assert list(ba[c]) == list(ob.ba[c])
        assert list(sf[c]) == list(ob.sf[c])
        nl = cp.sfBands.nLines
        bal = np.repeat(np.array(ob.ba[c][:]), nl)
        om = np.array(ob.mant[c][:])[:len(bal)]
        keep = bal > 0
        assert signs[c] == [int(m >> (b - 1)) & 1 for m, b in zip(om[keep], bal[keep])]
        assert len(codes[c]) == int(keep.sum()) and all(isinstance(s, str) and s for s in codes[c])


class _Bits:
    """MSB-first bit writer with PackedBits.WriteBits semantics (bitpack.py:36-101)."""

    def __init__(self, nbytes):
        self.b = bytearray(nbytes)
        self.pos = 0

    def write(self, value, n):
        for i in range(n - 1, -1, -1):
            if (value >> i) & 1:
                self.b[self.pos >> 3] |= 0x80 >> (self.pos & 7)
            self.pos += 1


def _write_data_block_ref(tup, cp):
    """Restatement of the reference's PACFile.WriteDataBlock packing loop
    (codec/pacfile.py:288-351) consuming the codec.Encode 7-tuple exactly as
    the reference does: len() and int(s, 2) of the Huffman code strings."""
    import struct
    scaleFactor, bitAlloc, signBits, mantissa, tableID, overallScaleFactor, LRMS = tup
    out = b""
    nl = cp.sfBands.nLines
    for iCh in range(cp.nChannels):
        nBits = cp.nScaleBits + cp.nTableIDBits
        iMant = 0
        for iBand in range(cp.sfBands.nBands):
            nBits += cp.nMantSizeBits + cp.nScaleBits
            if bitAlloc[iCh][iBand]:
                nBits += nl[iBand]
                for j in range(nl[iBand]):
                    nBits += len(mantissa[iCh][iMant + j])
                iMant += nl[iBand]
        nBits += len(LRMS)
        nBytes = nBits // 8 + (1 if nBits % 8 else 0)
        out += struct.pack("<L", nBytes)
        pb = _Bits(nBytes)
        pb.write(overallScaleFactor[iCh], cp.nScaleBits)
        pb.write(tableID[iCh], cp.nTableIDBits)
        iMant = 0
        for iBand in range(cp.sfBands.nBands):
            ba = bitAlloc[iCh][iBand]
            pb.write(ba - 1 if ba else 0, cp.nMantSizeBits)
            pb.write(int(scaleFactor[iCh][iBand]), cp.nScaleBits)
            if bitAlloc[iCh][iBand]:
                for j in range(nl[iBand]):
                    pb.write(signBits[iCh][iMant + j], 1)
                for j in range(nl[iBand]):
                    s = mantissa[iCh][iMant + j]
                    pb.write(int(s, 2), len(s))
                iMant += nl[iBand]
        for iBand in range(cp.sfBands.nBands):
            pb.write(int(LRMS[iBand]), 1)
        out += bytes(pb.b)
    return out


def test_codec_encode_tuple_feeds_reference_writer(ctx):
    """The master codec.Encode tuple (signBits, Huffman code strings, tableID,
    ...) consumed by a restatement of the reference's WriteDataBlock packing
    loop reproduces coded/piano_test2.wak block by block (first 40 blocks)."""
    from pac_amd import codec
    from pac_amd.huffman import Huffman
    from pac_amd.pcmfile import PCMFile
    from pac_amd.psychoac import ScaleFactorBands, AssignMDCTLinesFromFreqLimits
    with open(fixture("piano_test2.wak"), "rb") as f:
        ref = f.read()
    fs, nch, ns, nlines, off = P.parse_pac_header(ref)
    inFile = PCMFile(fixture("piano_test2.wav"))
    cp = inFile.OpenForReading()
    cp.nMDCTLines = cp.nSamplesPerBlock = 1024
    cp.nScaleBits, cp.nMantSizeBits, cp.targetBitsPerSample, cp.nTableIDBits = 4, 4, 2.27, 4
    cp.sfBands = ScaleFactorBands(AssignMDCTLinesFromFreqLimits(1024, cp.sampleRate))
    cp.extraBits = 0
    h = Huffman()
    prior = [np.zeros(1024) for _ in range(nch)]
    pos = off
    for blk in range(40):
        data = inFile.ReadDataBlock(cp)
        if data is None:
            break
        full = [np.concatenate((prior[c], data[c])) for c in range(nch)]
        prior = data
        tup = codec.Encode(full, cp, h, profile=codec.PROFILE_MASTER, context=ctx)
        assert all(isinstance(s, str) for s in tup[3][0])
        got = _write_data_block_ref(tup, cp)
        assert got == ref[pos:pos + len(got)], "block %d differs" % blk
        pos += len(got)
    inFile.Close(cp)
