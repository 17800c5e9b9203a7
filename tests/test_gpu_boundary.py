"""GPU parity AT the coder's decision boundaries: pairs of
streams one LSB apart across which the reference flips an LRMS flag, a
BitAlloc argmax, the -5 / -15 dB band cut or the budget test, or across which
an MLD row goes from "not needed" to "needed" with the crossing line within
2^-30 of the M/S threshold (tests/golden/boundary.py); and the dense few-LSB
M/S streams whose S channel gets bits.

Bar: the reference coder's own bytes (tests/golden/boundary/), whole files;
from random initial reservoir states, the oracle's bytes and final states;
the MLD cases also with the MLD skip and its prune off (PAC_MLD_SKIP=0):
the same bytes, so the prune's margin never decides a threshold.  All
streams of a sample rate in ONE pac_encode_streams call, through the C-ABI.

Reference: codec/codec.py:94-102, bitalloc.py:129-184, psychoac.py:570-591.
"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from conftest import GOLD

sys.path.insert(0, GOLD)
import boundary as B  # noqa: E402
import pyoracle as P  # noqa: E402

import pac_amd  # noqa: E402,F401
from pac_amd import _lib, pacfile  # noqa: E402

pytestmark = pytest.mark.gpu
MAN = B.load_manifest()
CASES = MAN["cases"]
POOL = max(1, min(16, os.cpu_count() or 1))


def ref_file(name, prof="master"):
    with open(os.path.join(B.OUT, name + (".wak" if prof == "master" else ".pac")), "rb") as f:
        return f.read()


def streams(kinds=None):
    """{fs: [(name, pcm)]} of the case streams (both sides)"""
    out = {}
    for c in CASES:
        if kinds and c["kind"] not in kinds:
            continue
        for side in ("a", "b"):
            fs, pcm = B.make_pcm(c[side])
            assert B.pcm_sha(pcm) == c[side]["pcm_sha256"]
            out.setdefault(fs, []).append(("%s_%s" % (c["name"], side), pcm))
    return out


def test_boundary_pairs_vs_reference(ctx):
    bad = []
    for fs, lst in sorted(streams().items()):
        bodies = pacfile.encode_streams([x for _, x in lst], fs, pacfile.PROFILE_MASTER, context=ctx)
        for (name, pcm), body in zip(lst, bodies):
            if pacfile.header_bytes(fs, 2, pcm.shape[0]) + body != ref_file(name):
                bad.append(name)
    assert not bad, bad


def test_boundary_pairs_reservoir_states_vs_oracle(ctx):
    """from random initial reservoir states the budget moves, so other
    decisions sit near these inputs' thresholds too: bytes and final states
    equal the oracle's"""
    for fs, lst in sorted(streams().items()):
        rng = np.random.default_rng(fs + 1)
        ex0 = rng.integers(-40, 40, len(lst))
        dp0 = rng.integers(-300, 3000, len(lst))
        st = [_lib.StreamState() for _ in lst]
        for s, e, d in zip(st, ex0, dp0):
            s.extra_bits, s.bit_deposit = int(e), int(d)
        bodies = pacfile.encode_streams([x for _, x in lst], fs, pacfile.PROFILE_MASTER, context=ctx, states=st)

        def one(k):
            s = P.State(int(ex0[k]), int(dp0[k]))
            return P.Oracle(fs, huffman=True).encode_data(P.MASTER, lst[k][1], state=s), (s.extraBits, s.deposit)

        with ThreadPoolExecutor(POOL) as ex:
            ref = list(ex.map(one, range(len(lst))))
        bad = [lst[k][0] for k in range(len(lst))
               if bodies[k] != ref[k][0] or (st[k].extra_bits, st[k].bit_deposit) != ref[k][1]]
        assert not bad, (fs, bad)


def test_mld_prune_boundary_skip_on_off(ctx, monkeypatch):
    """the MLD-crossing streams with the MLD skip and prune on (default) and
    off: the same bytes, and the reference's"""
    lst = streams({"mld"})
    assert lst
    monkeypatch.setenv("PAC_MLD_SKIP", "0")
    off = _lib.Context(0)
    monkeypatch.delenv("PAC_MLD_SKIP")
    try:
        for fs, items in sorted(lst.items()):
            pcms = [x for _, x in items]
            a = pacfile.encode_streams(pcms, fs, pacfile.PROFILE_MASTER, context=ctx)
            b = pacfile.encode_streams(pcms, fs, pacfile.PROFILE_MASTER, context=off)
            assert a == b
            for (name, pcm), body in zip(items, a):
                assert pacfile.header_bytes(fs, 2, pcm.shape[0]) + body == ref_file(name), name
    finally:
        off.close()


@pytest.mark.parametrize("prof", ["master", "origin"])
def test_lsbdense_vs_reference(ctx, prof):
    """the dense few-LSB M/S streams (S gets bits), both rates, vs the
    reference coder's files"""
    items = [(n, e) for n, e in sorted(MAN["lsbdense"].items()) if e["profile"] == prof]
    assert len(items) == 4
    P_ = pacfile.PROFILE_MASTER if prof == "master" else pacfile.PROFILE_ORIGIN
    bad = []
    for fs in (44100, 48000):
        grp = [(n, B.lsb_dense_pcm(fs, e["D"])) for n, e in items if e["fs"] == fs]
        bodies = pacfile.encode_streams([x for _, x in grp], fs, P_, context=ctx)
        for (n, pcm), body in zip(grp, bodies):
            if pacfile.header_bytes(fs, 2, pcm.shape[0]) + body != ref_file(n, prof):
                bad.append(n)
    assert not bad, bad
