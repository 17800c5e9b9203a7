"""GPU decoder (pac_decode_streams: PACFile.ReadDataBlock + codec.Decode + the
decode driver) against the reference's own decodes and
the CPU oracle.  Bars: output WAV files byte-exact; float samples before the
int16 conversion within 1e-12 of the oracle's (IMDCT rounding order differs)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLD, ROOT, fixture

import pac_amd  # noqa: F401
from pac_amd import pacfile, synth
import pyoracle as P

pytestmark = pytest.mark.gpu

MAN = json.load(open(os.path.join(GOLD, "decode_manifest.json")))


def sha(b):
    return hashlib.sha256(b).hexdigest()


def _path(name):
    return fixture(name[len("fixtures/"):]) if name.startswith("fixtures/") else os.path.join(GOLD, name)


@pytest.mark.parametrize("name", sorted(MAN["shim"]))
def test_decode_file_equals_reference_shim(ctx, name):
    prof = pacfile.PROFILE_ORIGIN if name.endswith(".pac") else pacfile.PROFILE_MASTER
    got = pacfile.decode_file(_path(name), profile=prof, context=ctx)
    assert sha(got) == MAN["shim"][name]["sha256"]


def test_piano_test2_equals_reference_output(ctx):
    got = pacfile.decode_file(fixture("piano_test2.wak"), profile=pacfile.PROFILE_MASTER, context=ctx)
    assert sha(got) == MAN["reference_outputs"]["piano_test2"]


@pytest.mark.parametrize("name", ["fixtures/harpsichord.pac", "fixtures/piano_test2.wak", "master_white48k.wak",
                                  "origin_square44k.pac"])
def test_float_samples_vs_oracle(ctx, name):
    prof = pacfile.PROFILE_ORIGIN if name.endswith(".pac") else pacfile.PROFILE_MASTER
    with open(_path(name), "rb") as f:
        b = f.read()
    fs, nch, ns, _, off = pacfile.parse_header(b)
    from pac_amd import _lib
    pcm, fo, fl = ctx.decode_streams(_lib.params(fs, nch, prof), b[off:], [0, len(b) - off], want_float=True)
    o = P.Oracle(fs, huffman=(prof == pacfile.PROFILE_MASTER))
    rp, rf = o.decode_data(prof, b[off:], nch, want_float=True)
    assert pcm.shape == rp.shape
    assert np.max(np.abs(fl - rf)) < 1e-12
    assert np.array_equal(pcm, rp)


@pytest.mark.parametrize("prof", [pacfile.PROFILE_ORIGIN, pacfile.PROFILE_MASTER])
def test_multi_stream_round_trip_vs_oracle(ctx, prof):
    """encode_streams -> decode_streams on ragged streams (0, 1, 1023, 1024,
    1025, 40 blocks + 7 frames) equals the oracle's decode of the same bytes"""
    fs = 44100
    lens = [0, 1, 1023, 1024, 1025, 40 * 1024 + 7]
    streams = [synth.pink_tones_pcm(n, fs, seed=i) if n else np.zeros((0, 2), np.int16)
               for i, n in enumerate(lens)]
    secs = pacfile.encode_streams(streams, fs, prof, context=ctx)
    got = pacfile.decode_streams(secs, fs, 2, prof, context=ctx)
    o = P.Oracle(fs, huffman=(prof == pacfile.PROFILE_MASTER))
    for n, sec, g in zip(lens, secs, got):
        ref = o.decode_data(prof, sec, 2)
        assert g.shape == ref.shape, n
        assert np.array_equal(g, ref), n
        # the coded delay: decoded frames = blocks x 1024 >= input frames
        assert g.shape[0] >= n


@pytest.mark.parametrize("prof", [pacfile.PROFILE_ORIGIN, pacfile.PROFILE_MASTER])
def test_parse_and_synthesis_boundaries(ctx, prof):
    """Channel-block counts across the parse's 512-lane workgroups and 64-lane
    code tiles (lanes past the last channel-block stay in the wave-uniform line
    loops) and streams across the synthesis' 64-block segments: 3 streams of
    130, 66 and 65 hops (+ the flush block) = 528 stereo channel-blocks"""
    fs = 48000
    lens = [130 * 1024, 66 * 1024 - 5, 65 * 1024]
    streams = [synth.pink_tones_pcm(n, fs, seed=10 + i) for i, n in enumerate(lens)]
    secs = pacfile.encode_streams(streams, fs, prof, context=ctx)
    got = pacfile.decode_streams(secs, fs, 2, prof, context=ctx)
    o = P.Oracle(fs, huffman=(prof == pacfile.PROFILE_MASTER))
    for n, sec, g in zip(lens, secs, got):
        assert np.array_equal(g, o.decode_data(prof, sec, 2)), n


def test_read_data_block_surface(ctx, tmp_path):
    """PACFile.ReadDataBlock hop by hop (the reference's decode driver loop,
    skipping the first result) written through PCMFile gives decode_file's bytes"""
    from pac_amd.pcmfile import PCMFile
    src = fixture("piano_test2.wak")
    inFile = pacfile.PACFile(src, profile=pacfile.PROFILE_MASTER, context=ctx)
    cp = inFile.OpenForReading()
    cp.bitsPerSample = 16
    out = tmp_path / "o.wav"
    outFile = PCMFile(str(out))
    outFile.OpenForWriting(cp)
    first = True
    nblk = 0
    while True:
        data = inFile.ReadDataBlock(cp)
        if not data:
            break
        nblk += 1
        if first:
            first = False
            continue
        outFile.WriteDataBlock(data, cp)
    inFile.Close(cp)
    outFile.Close(cp)
    assert sha(out.read_bytes()) == MAN["reference_outputs"]["piano_test2"]
    assert nblk > 2


def test_mono_and_three_channel_origin(ctx):
    for nch in (1, 3):
        pcm = synth.white_pcm(9 * 1024 + 11, nch, seed=nch, scale=0.05)
        sec = pacfile.encode_streams([pcm], 32000, pacfile.PROFILE_ORIGIN, context=ctx)[0]
        got = pacfile.decode_streams([sec], 32000, nch, pacfile.PROFILE_ORIGIN, context=ctx)[0]
        ref = P.Oracle(32000, huffman=False).decode_data(P.ORIGIN, sec, nch)
        assert np.array_equal(got, ref)


@pytest.mark.parametrize("name,prof", [("piano_test2.wak", pacfile.PROFILE_MASTER),
                                       ("harpsichord.pac", pacfile.PROFILE_ORIGIN)])
def test_corrupt_nbytes_is_refused(ctx, name, prof):
    """A channel-block whose '<L nBytes' is cut short (its fields run past it)
    makes the decoder raise PAC_E_ARG -- the reference's PackedBits raises --
    and never read outside the data."""
    from pac_amd import _lib
    with open(fixture(name), "rb") as f:
        b = bytearray(f.read())
    fs, nch, ns, _, off = pacfile.parse_header(bytes(b))
    # the largest channel-block: shrink its nBytes by 40 and drop the last 40
    # bytes of its payload (the channel-blocks after it stay intact)
    pos, big, bign = off, off, -1
    while pos + 4 <= len(b):
        n = int.from_bytes(b[pos:pos + 4], "little")
        if n > bign:
            big, bign = pos, n
        pos += 4 + n
    b[big:big + 4] = (bign - 40).to_bytes(4, "little")
    del b[big + 4 + bign - 40:big + 4 + bign]
    with pytest.raises(_lib.PacError) as e:
        ctx.decode_streams(_lib.params(fs, nch, prof), bytes(b[off:]), [0, len(b) - off])
    assert e.value.code == -1
