"""GPU parity at the M/S decision's extremes (tests/msx.py): dual-mono
(S == 0: every S threshold is the threshold in quiet, every S line on the SPL
floor), anti-phase (M == 0), one silent channel, sparse +-1 LSB differences
(S tiny, not zero), DC pairs, and a stream cycling through them -- 201 blocks
each, master and Origin coders, 44.1 and 48 kHz, all eight streams of a
profile and rate as independent streams of one call, through the C-ABI.

Bar: the reference's own bytes (tests/golden/msx/, made by the reference's
coders), whole files -- except the Origin coder's constant-channel streams,
whose zero-magnitude mantissa signs are the sign of FFT rounding noise
(tests/msx.py: the reference's own two MDCTs disagree on them); there every
other field must be equal.  The master profile is also checked from random
initial reservoir states against the oracle (bytes and final states).

Reference: codec/codec.py:94-102 (LRMS), psychoac.py:549-591 (M/S lines, six
calcBTHR, MLD), :662-682 (band selection), bitalloc.py:157-184, the SPL
floor psychoac.py:15-42.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import msx

import pac_amd  # noqa: F401
from pac_amd import _lib, pacfile
import pyoracle as P

pytestmark = pytest.mark.gpu
PROF = {"master": pacfile.PROFILE_MASTER, "origin": pacfile.PROFILE_ORIGIN}
POOL = max(1, min(16, os.cpu_count() or 1))


def _group(fs, prof):
    return [n for n in msx.CASES if msx.case(n)["fs"] == fs and msx.case(n)["profile"] == prof]


@pytest.mark.parametrize("fs", [44100, 48000])
@pytest.mark.parametrize("prof", ["master", "origin"])
def test_msx_one_call_vs_reference(ctx, fs, prof):
    names = _group(fs, prof)
    assert len(names) == 8
    bodies = pacfile.encode_streams([msx.pcm(n) for n in names], fs, PROF[prof], context=ctx)
    nl = msx.nlines(fs)
    bad = []
    for n, body in zip(names, bodies):
        ref = msx.reference(n)
        got = pacfile.header_bytes(fs, 2, msx.FRAMES) + body
        if n in msx.NOISE_SIGN:
            assert got[:26 + 50] == ref[:26 + 50]
            ok, _ = msx.origin_equal_up_to_noise_signs(body, msx.data_section(ref), nl)
            if not ok:
                bad.append(n)
        elif got != ref:
            bad.append(n)
    assert not bad, bad


@pytest.mark.parametrize("fs", [44100, 48000])
def test_msx_master_reservoir_states_vs_oracle(ctx, fs):
    """from random initial reservoir states (codingParams.extraBits,
    huffman.bitDeposit): bytes and final states equal the oracle's"""
    names = _group(fs, "master")
    rng = np.random.default_rng(fs)
    ex0 = rng.integers(-40, 40, len(names))
    dp0 = rng.integers(-300, 3000, len(names))
    st = [_lib.StreamState() for _ in names]
    for s, e, d in zip(st, ex0, dp0):
        s.extra_bits, s.bit_deposit = int(e), int(d)
    bodies = pacfile.encode_streams([msx.pcm(n) for n in names], fs, PROF["master"], context=ctx, states=st)

    def one(k):
        s = P.State(int(ex0[k]), int(dp0[k]))
        data = P.Oracle(fs, huffman=True).encode_data(P.MASTER, msx.pcm(names[k]), state=s)
        return data, (s.extraBits, s.deposit)

    with ThreadPoolExecutor(POOL) as ex:
        ref = list(ex.map(one, range(len(names))))
    bad = [names[k] for k in range(len(names)) if bodies[k] != ref[k][0]]
    assert not bad, bad
    bad = [names[k] for k in range(len(names)) if (st[k].extra_bits, st[k].bit_deposit) != ref[k][1]]
    assert not bad, bad


@pytest.mark.parametrize("fs", [44100, 48000])
def test_msx_plugin_surface_per_block(ctx, fs, tmp_path):
    """PACFile.WriteDataBlock hop by hop with the Huffman reservoir object (the
    per-block path, pac_encode_block), as the reference driver runs it
    (pacfile.py:474-499), on the dual-mono, anti-phase and silent-channel
    streams: the first 24 hops equal the reference file's prefix"""
    from pac_amd.huffman import Huffman
    from pac_amd.pcmfile import PCMFile
    for kind in ("dualmono", "antiphase", "rsilent"):
        name = "%s_%dk_master.wak" % (kind, fs // 1000)
        wav, out = tmp_path / (kind + ".wav"), tmp_path / (kind + ".wak")
        x = msx.pcm(name)
        wav.write_bytes(P.wav_bytes(fs, 2, x.shape[0], x))
        huffman = Huffman()
        inFile = PCMFile(str(wav))
        outFile = pacfile.PACFile(str(out), profile=PROF["master"], context=ctx)
        cp = inFile.OpenForReading()
        cp.nMDCTLines, cp.nScaleBits, cp.nMantSizeBits = 1024, 4, 4
        cp.targetBitsPerSample, cp.nTableIDBits = 2.27, 4
        cp.nSamplesPerBlock = cp.nMDCTLines
        outFile.OpenForWriting(cp)
        for _ in range(24):
            outFile.WriteDataBlock(inFile.ReadDataBlock(cp), cp, huffman)
        outFile.fp.close()
        got = out.read_bytes()
        ref = msx.reference(name)
        assert len(got) > 26 + 50 + 24 * 8 and got == ref[:len(got)], name
