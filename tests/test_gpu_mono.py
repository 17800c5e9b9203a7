"""Mono master extension.  The reference's master
coder is stereo only (codec.py:46-47, 98), so parity is UNPINNED against the
reference: one channel coded by the master pipeline with LRMS all 0 (the 25
flag bits still written), BTHR_L alone, one BitAlloc + Huffman + deposit per
block.  The HIP path is checked byte for byte against the oracle's restatement
(oracle/pac_oracle.c pac_oracle_block_master with xR == NULL), which
tests/test_oracle.py::test_mono_master_first_block_is_stereo_left ties to the
stereo coder.  Bar: bit-exact bytes, reservoir state and decoded samples."""
import numpy as np
import pytest

import pac_amd  # noqa: F401
from pac_amd import pacfile, synth, _lib, codec
import pyoracle as P

pytestmark = pytest.mark.gpu
MASTER = pacfile.PROFILE_MASTER


def _mono(n, fs, seed):
    return np.ascontiguousarray(synth.pink_tones_pcm(n, fs, seed=seed)[:, :1])


@pytest.mark.parametrize("fs", [44100, 48000])
def test_mono_master_streams_vs_oracle(ctx, fs):
    lens = [0, 1, 1023, 1024, 5000, 20 * 1024, 33 * 1024 + 17]
    streams = [_mono(n, fs, i) if i % 2 else np.ascontiguousarray(synth.white_pcm(n, 1, seed=i))
               for i, n in enumerate(lens)]
    states = [_lib.StreamState() for _ in lens]
    got = pacfile.encode_streams(streams, fs, MASTER, context=ctx, states=states)
    o = P.Oracle(fs, huffman=True)
    for i, s in enumerate(streams):
        st = P.State()
        assert got[i] == o.encode_data(P.MASTER, s, state=st), "stream %d differs" % i
        assert (states[i].extra_bits, states[i].bit_deposit) == (st.extraBits, st.deposit)


def test_mono_master_decode_vs_oracle(ctx):
    fs = 48000
    streams = [_mono(n, fs, n) for n in (3000, 17 * 1024 + 3)]
    got = pacfile.encode_streams(streams, fs, MASTER, context=ctx)
    dec = pacfile.decode_streams(got, fs, 1, MASTER, context=ctx)
    o = P.Oracle(fs, huffman=True)
    for g, d in zip(got, dec):
        assert np.array_equal(d, o.decode_data(P.MASTER, g, 1))


def test_mono_master_block_fields(ctx):
    """codec.Encode on one mono block: the tuple's fields and the reservoir
    state equal the oracle's."""
    from pac_amd.audiofile import CodingParams
    from pac_amd.huffman import Huffman
    from pac_amd.psychoac import ScaleFactorBands, AssignMDCTLinesFromFreqLimits
    from pac_amd.pcmfile import codes_to_float
    fs = 48000
    x = [codes_to_float(_mono(4 * 1024, fs, 9)[1024:3072, 0])]
    cp = CodingParams()
    cp.sampleRate, cp.nChannels, cp.nMDCTLines = fs, 1, 1024
    cp.nScaleBits, cp.nMantSizeBits, cp.targetBitsPerSample, cp.nTableIDBits = 4, 4, 2.27, 4
    cp.sfBands = ScaleFactorBands(AssignMDCTLinesFromFreqLimits(1024, fs))
    cp.extraBits = -40
    h = Huffman()
    h.bitDeposit = 900
    sf, ba, signs, codes, tid, overall, lrms = codec.Encode(x, cp, h, profile=codec.PROFILE_MASTER,
                                                            context=ctx)
    o = P.Oracle(fs, huffman=True)
    st = P.State()
    st.extraBits, st.deposit = -40, 900
    ob = o.block_master(x[0], None, st)
    assert list(lrms) == [0] * 25
    assert (cp.extraBits, h.bitDeposit) == (st.extraBits, st.deposit)
    assert len(ba) == 1 and overall[0] == ob.overall[0] and tid[0] == ob.table_id[0]
    assert list(ba[0]) == list(ob.ba[0])
    assert list(sf[0]) == list(ob.sf[0])


def test_mono_master_wav_file(ctx, tmp_path):
    """A mono WAV through the device ingest (pac_encode_wav) and egress
    (pac_decode_wav) against the oracle's encode and decode drivers."""
    fs = 44100
    x = _mono(9 * 1024 + 100, fs, 21)
    path = tmp_path / "mono.wav"
    path.write_bytes(P.wav_bytes(fs, 1, x.shape[0], x))
    got = pacfile.encode_wav_files([str(path)], MASTER, context=ctx)[0]
    assert got == P.encode_file(str(path), P.MASTER)
    cpath = tmp_path / "mono.wak"
    cpath.write_bytes(got)
    assert pacfile.decode_to_wav([got], MASTER, context=ctx)[0] == P.decode_file(str(cpath), P.MASTER)
