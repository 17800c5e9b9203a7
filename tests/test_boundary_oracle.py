"""The decision-boundary cases (tests/golden/boundary.py) on the CPU: every
pair still brackets its decision in the oracle, at the recorded distance, and
the oracle's bytes equal the reference coder's own encodes of both streams
(tests/golden/boundary/, made by tests/golden/make_boundary_golden.py).  So
the oracle the GPU tests compare with is pinned by the reference at exactly
these boundaries.

Reference: codec/codec.py:94-102 (LRMS), bitalloc.py:129-184 (argmax, the
-5 / -15 dB cut, the budget test), psychoac.py:570-591 (MLD combination).
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
from pac_amd import pacfile  # noqa: E402

MAN = B.load_manifest()
CASES = MAN["cases"]
POOL = max(1, min(8, os.cpu_count() or 1))


def ref_file(name, prof="master"):
    with open(os.path.join(B.OUT, name + (".wak" if prof == "master" else ".pac")), "rb") as f:
        return f.read()


def test_manifest_covers_every_decision():
    kinds = {}
    for c in CASES:
        kinds[c["kind"]] = kinds.get(c["kind"], 0) + 1
    assert {"lrms", "argmax", "cut", "mld", "mldneed"} <= set(kinds), kinds
    assert kinds["lrms"] >= 6 and kinds["argmax"] >= 6 and kinds["cut"] >= 4 and kinds["mld"] >= 3, kinds
    assert any(c["kind"] == "cut" and c["cutoff"] == -5.0 for c in CASES)
    assert any(c["kind"] == "cut" and c["cutoff"] == -15.0 for c in CASES)
    # the MLD prune's boundary: at least three rows whose deciding line sits
    # within 2^-30 of the M/S threshold (relative, as intensities) on both sides
    assert sum(c["kind"] == "mld" and c["margin"] < B.PRUNE_REL for c in CASES) >= 3
    # the LRMS flags within 1e-8 (relative) of the 0.8 ratio, the cuts within 1e-4 dB
    assert all(c["margin"] < 1e-8 for c in CASES if c["kind"] == "lrms")
    assert all(c["margin"] < 1e-4 for c in CASES if c["kind"] == "cut")


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_case_brackets_its_decision(case):
    """the two streams are the recorded PCM, a few LSB apart; the oracle takes
    the named decision differently on them, each within the recorded distance
    of the threshold and on opposite sides"""
    fs, pa = B.make_pcm(case["a"])
    _, pb = B.make_pcm(case["b"])
    assert B.pcm_sha(pa) == case["a"]["pcm_sha256"] and B.pcm_sha(pb) == case["b"]["pcm_sha256"]
    assert 1 <= np.count_nonzero(pa != pb) <= 9 and np.max(np.abs(pa.astype(int) - pb.astype(int))) <= 2
    ba, bb = B.oracle_blocks(fs, pa), B.oracle_blocks(fs, pb)
    assert B.decision(case, fs, ba) != B.decision(case, fs, bb)
    if case["kind"] != "budget":
        ma, mb = B.signed_margin(case, fs, pa, ba), B.signed_margin(case, fs, pb, bb)
        assert (ma > 0) != (mb > 0) or case["kind"] == "argmax", (ma, mb)
        assert max(abs(ma), abs(mb)) <= case["margin"] * (1 + 1e-6) + 1e-15


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_equals_reference_at_the_boundary(case):
    """the oracle's whole file (header + data) of both streams equals the
    reference coder's"""
    for side in ("a", "b"):
        fs, pcm = B.make_pcm(case[side])
        body = P.Oracle(fs, huffman=True).encode_data(P.MASTER, pcm)
        got = pacfile.header_bytes(fs, 2, pcm.shape[0]) + body
        assert got == ref_file("%s_%s" % (case["name"], side)), (case["name"], side)


def test_lsbdense_oracle_equals_reference():
    """the dense few-LSB M/S streams, master and Origin coders, both rates"""
    items = sorted(MAN["lsbdense"].items())

    def one(it):
        name, e = it
        pcm = B.lsb_dense_pcm(e["fs"], e["D"])
        assert B.pcm_sha(pcm) == e["pcm_sha256"]
        prof = P.MASTER if e["profile"] == "master" else P.ORIGIN
        body = P.Oracle(e["fs"], huffman=prof == P.MASTER).encode_data(prof, pcm)
        return name, pacfile.header_bytes(e["fs"], 2, pcm.shape[0]) + body == ref_file(name, e["profile"])

    with ThreadPoolExecutor(POOL) as ex:
        bad = [n for n, ok in ex.map(one, items) if not ok]
    assert not bad, bad


@pytest.mark.parametrize("fs", [44100, 48000])
def test_lsbdense_moves_the_s_allocation(fs):
    """unlike the sparse "lsb" kind, the dense +-8 LSB differences give the S
    channel bits in most blocks (at +-4 rarely: its S SMRs sit just under the
    -5 dB cut), where dual-mono gives none"""
    for D, lo, hi in ((8, 0.5, 1.0), (4, -1.0, 0.5)):
        pcm = B.lsb_dense_pcm(fs, D)[:40 * 1024]
        bl = B.oracle_blocks(fs, pcm)
        frac = np.mean([any(b.lrms[k] and b.ba[1][k] for k in range(25)) for b in bl])
        assert lo < frac <= hi, (D, frac)
        mono = pcm.copy()
        mono[:, 1] = mono[:, 0]
        assert all(not any(b.ba[1][k] for k in range(25) if b.lrms[k]) for b in B.oracle_blocks(fs, mono))
