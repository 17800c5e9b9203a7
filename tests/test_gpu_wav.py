"""WAV ingest and egress on the device: the reference's
PCMFile header scan, frame reads and padding, the exact-multiple extra hop
(pcmfile.py:32-100, pacfile.py:240-242) and the decode driver's WAV output
(pcmfile.py:103-147), checked against the host mirror (pac_amd.pcmfile, itself
byte-identical to the reference), the reference's coded files and the
reference's decodes outputs/*.wav (sha256)."""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

from conftest import GOLD, fixture
from test_oracle import REF_FIXTURES

import pac_amd  # noqa: F401
from pac_amd import pacfile, _lib, synth
from pac_amd.pcmfile import read_for_encode
import pyoracle as P

pytestmark = pytest.mark.gpu
PROF = {P.ORIGIN: pacfile.PROFILE_ORIGIN, P.MASTER: pacfile.PROFILE_MASTER}


def test_scan_matches_host_parser(ctx):
    names = sorted(os.listdir(os.path.dirname(fixture("harpsichord.wav"))))
    blobs = [open(fixture(n), "rb").read() for n in names]
    fo = np.zeros(len(blobs) + 1, dtype=np.int64)
    fo[1:] = np.cumsum([len(b) for b in blobs])
    info = ctx.wav_scan(b"".join(blobs), fo)
    for n, w in zip(names, info):
        cp, fr = read_for_encode(fixture(n))
        assert w.status == 0
        assert (w.sample_rate, w.n_channels, w.num_samples, w.frames) == \
            (cp.sampleRate, cp.nChannels, cp.numSamples, fr.shape[0]), n


@pytest.mark.parametrize("prof", [P.ORIGIN, P.MASTER])
def test_encode_wav_files_reference_bitstreams(ctx, prof):
    items = [(i, c) for i, c, p in REF_FIXTURES if p == prof]
    got = pacfile.encode_wav_files([fixture(i) for i, _ in items], PROF[prof], context=ctx)
    for (i, c), g in zip(items, got):
        with open(fixture(c), "rb") as f:
            assert g == f.read(), c


def _wav(frames, fs=44100, tail=b""):
    nch = frames.shape[1]
    data = np.ascontiguousarray(frames, dtype="<i2").tobytes()
    h = struct.pack("<4sL4s4sLHHLLHH4sL", b"RIFF", 36 + len(data) + len(tail), b"WAVE", b"fmt ", 16, 1, nch, fs,
                    fs * nch * 2, nch * 2, 16, b"data", len(data))
    return h + data + tail


@pytest.mark.parametrize("tail", [b"", b"LIST\x04\x00\x00\x00abcd", b"\x01\x02\x03", bytes(range(256)) * 20])
@pytest.mark.parametrize("prof", [pacfile.PROFILE_ORIGIN, pacfile.PROFILE_MASTER])
def test_exact_multiple_quirk(ctx, tmp_path, tail, prof):
    """numSamples an exact multiple of 1024: the driver reads one more hop from
    the bytes after the data chunk (byte granular, zero padded) -- the device
    scan + gather must equal the host mirror + the oracle"""
    pcm = synth.pink_tones_pcm(7 * 1024, 44100, seed=len(tail))
    w = _wav(pcm, tail=tail)
    path = tmp_path / "q.wav"
    path.write_bytes(w)
    got = pacfile.encode_wav_files([w], prof, context=ctx)[0]
    assert got == pacfile.encode_file(str(path), profile=prof, context=ctx)
    cp, fr = read_for_encode(str(path))
    o = P.Oracle(44100, huffman=(prof == pacfile.PROFILE_MASTER))
    exp = o.encode_data(P.MASTER if prof == pacfile.PROFILE_MASTER else P.ORIGIN, fr)
    assert got[len(pacfile.header_bytes(44100, 2, cp.numSamples)):] == exp


@pytest.mark.parametrize("claimed,cut", [(3 * 1024 + 5, 2 * 4096 + 6), (4 * 1024, 3 * 4096 + 1),
                                         (0xFFFFFFFF // 4, 5 * 4096 + 40), (4 * 1024, 0)])
@pytest.mark.parametrize("prof", [pacfile.PROFILE_ORIGIN, pacfile.PROFILE_MASTER])
def test_truncated_wav(ctx, tmp_path, claimed, cut, prof):
    """data chunk shorter than its header (cut short, or a streaming header):
    the device scan codes the bytes present, as the reference's reads
    (pcmfile.py:69-80) -- equal to the host mirror and the oracle"""
    pcm = synth.pink_tones_pcm(6 * 1024, 44100, seed=cut)
    d = np.ascontiguousarray(pcm, dtype="<i2").tobytes()[:cut]
    w = struct.pack("<4sL4s4sLHHLLHH4sL", b"RIFF", 36 + len(d), b"WAVE", b"fmt ", 16, 1, 2, 44100, 44100 * 4, 4,
                    16, b"data", min(claimed * 4, 0xFFFFFFFF)) + d
    path = tmp_path / "t.wav"
    path.write_bytes(w)
    info = ctx.wav_scan(w, [0, len(w)])[0]
    cp, fr = read_for_encode(str(path))
    assert info.frames == fr.shape[0] == (cut + 3) // 4
    got = pacfile.encode_wav_files([w], prof, context=ctx)[0]
    assert got == pacfile.encode_file(str(path), profile=prof, context=ctx)
    o = P.Oracle(44100, huffman=(prof == pacfile.PROFILE_MASTER))
    exp = o.encode_data(P.MASTER if prof == pacfile.PROFILE_MASTER else P.ORIGIN, fr)
    assert got[len(pacfile.header_bytes(44100, 2, cp.numSamples)):] == exp


def test_bad_first_wav_raises_its_wav_error(ctx):
    """sample rate and channels taken from the first file: a malformed first
    file raises the reference's PCMFile error, not a parameter error"""
    with pytest.raises(_lib.PacError) as e:
        pacfile.encode_wav_files([b"RIFF0000WAVEjunkjunk"], pacfile.PROFILE_MASTER, context=ctx)
    assert "'fmt '" in str(e.value)


def test_bad_wav_raises(ctx):
    with pytest.raises(_lib.PacError) as e:
        pacfile.encode_wav_files([b"RIFX0000WAVEfmt "], pacfile.PROFILE_ORIGIN, context=ctx, n_channels=2,
                                 sample_rate=44100)
    assert "RIFF" in str(e.value)


MAN = json.load(open(os.path.join(GOLD, "decode_manifest.json")))


def test_decode_to_wav_reference_outputs(ctx):
    """the 12 master files decoded to WAV bytes in one device call == the
    reference's outputs/*.wav"""
    names = sorted(MAN["reference_outputs"])
    coded = [open(fixture(n + ".wak"), "rb").read() for n in names]
    wavs = pacfile.decode_to_wav(coded, pacfile.PROFILE_MASTER, context=ctx)
    for n, w in zip(names, wavs):
        assert hashlib.sha256(w).hexdigest() == MAN["reference_outputs"][n], n
