"""GPU parity of the origin profile (PerceptualAudioCodec_Origin/codec) against
the committed golden bitstream and the CPU oracle.  Bar: bit-exact bytes."""
import numpy as np
import pytest

from conftest import fixture

import pac_amd  # noqa: F401  (registers the package)
from pac_amd import pacfile, _lib, synth
import pyoracle as P

pytestmark = pytest.mark.gpu

ORIGIN = pacfile.PROFILE_ORIGIN


def test_harpsichord_pac_bit_exact(ctx):
    """coded/harpsichord.pac (reference fixture, 387 blocks) byte for byte."""
    got = pacfile.encode_file(fixture("harpsichord.wav"), profile=ORIGIN, context=ctx)
    with open(fixture("harpsichord.pac"), "rb") as f:
        ref = f.read()
    assert len(got) == len(ref)
    assert got == ref


def _oracle_streams(streams, fs):
    o = P.Oracle(fs, huffman=False)
    return [o.encode_data(P.ORIGIN, s) for s in streams]


@pytest.mark.parametrize("fs", [48000, 44100, 32000])
def test_white_noise_streams_vs_oracle(ctx, fs):
    """Multi-stream batch (config 2 style: white noise) vs the CPU oracle."""
    rng = np.random.default_rng(fs)
    lens = [0, 1, 1023, 1024, 1025, 5000, 20 * 1024, 33 * 1024 + 7]
    streams = [synth.white_pcm(n, 2, seed=fs + i) for i, n in enumerate(lens)]
    got = pacfile.encode_streams(streams, fs, ORIGIN, context=ctx)
    exp = _oracle_streams(streams, fs)
    for i, (g, e) in enumerate(zip(got, exp)):
        assert g == e, "stream %d (len %d) differs" % (i, lens[i])


@pytest.mark.parametrize("nch", [1, 3])
def test_channel_counts_vs_oracle(ctx, nch):
    fs = 44100
    streams = [synth.white_pcm(8 * 1024 + 100, nch, seed=7 + nch, scale=0.1)]
    got = pacfile.encode_streams(streams, fs, ORIGIN, context=ctx)
    exp = _oracle_streams(streams, fs)
    assert got == exp


@pytest.mark.parametrize("name", ["origin_white48k", "origin_zero48k", "origin_square44k",
                                  "origin_mono44k"])
def test_golden_reference_streams(ctx, name):
    """Bitstreams the reference itself produced (tests/golden/make_golden.py):
    white noise @48 kHz, digital silence (signed-zero MDCT lines), full-scale
    square wave (-32768 -> +0.0, quantizer clip) with an impulse train, mono."""
    import os
    from conftest import GOLD
    pcm = np.load(os.path.join(GOLD, name + ".in.npy"))
    with open(os.path.join(GOLD, name + ".pac"), "rb") as f:
        ref = f.read()
    fs = {"48k": 48000, "44k": 44100}[name[-3:]]
    body = pacfile.encode_streams([pcm], fs, ORIGIN, context=ctx)[0]
    assert pacfile.header_bytes(fs, pcm.shape[1], pcm.shape[0]) + body == ref


def test_plugin_surface_matches_batch(ctx, tmp_path):
    """PACFile.WriteDataBlock hop by hop (the reference's own driver loop,
    pacfile.py:474-499) gives the same bytes as the batched GPU call."""
    from pac_amd.pcmfile import PCMFile
    src = fixture("harpsichord.wav")
    out = tmp_path / "h.pac"
    inFile = PCMFile(src)
    outFile = pacfile.PACFile(str(out), profile=ORIGIN, context=ctx)
    cp = inFile.OpenForReading()
    cp.nMDCTLines = 1024
    cp.nScaleBits = 4
    cp.nMantSizeBits = 4
    cp.targetBitsPerSample = 2.27
    cp.nSamplesPerBlock = cp.nMDCTLines
    outFile.OpenForWriting(cp)
    nblk = 0
    while nblk < 40:
        data = inFile.ReadDataBlock(cp)
        if not data:
            break
        outFile.WriteDataBlock(data, cp)
        nblk += 1
    outFile.fp.close()
    got = out.read_bytes()
    with open(fixture("harpsichord.pac"), "rb") as f:
        ref = f.read()
    assert got == ref[:len(got)]


def test_codec_encode_tuple_matches_oracle(ctx):
    """codec.Encode (Origin codec.py:52-67) fields for one block vs the oracle's
    per-stage values: overall scale, SMR (1e-9 abs), bit allocation, scale
    factors, mantissas."""
    from pac_amd import codec
    from pac_amd.audiofile import CodingParams
    from pac_amd.psychoac import ScaleFactorBands, AssignMDCTLinesFromFreqLimits
    fs, nch = 48000, 2
    pcm = synth.white_pcm(3 * 1024, nch, seed=11)
    x = np.stack([synth_float(pcm[:2048, c]) for c in range(nch)])
    cp = CodingParams()
    cp.sampleRate, cp.nChannels, cp.nMDCTLines = fs, nch, 1024
    cp.nScaleBits, cp.nMantSizeBits, cp.targetBitsPerSample = 4, 4, 2.27
    cp.sfBands = ScaleFactorBands(AssignMDCTLinesFromFreqLimits(1024, fs))
    sf, ba, mant, overall = codec.Encode([x[0], x[1]], cp, profile=codec.PROFILE_ORIGIN,
                                         context=ctx)
    o = P.Oracle(fs, huffman=False)
    for c in range(nch):
        ob = o.block_origin(x[c])
        assert overall[c] == ob.overall
        assert list(ba[c]) == list(ob.ba)
        assert list(sf[c]) == list(ob.sf)
        keep = np.repeat(np.array(ob.ba[:]) > 0, cp.sfBands.nLines)
        assert np.array_equal(mant[c], np.array(ob.mant[:])[keep])


def synth_float(codes):
    from pac_amd.pcmfile import codes_to_float
    return codes_to_float(codes)
