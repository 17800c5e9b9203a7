"""The CPU oracle's decoder (oracle/pac_oracle.c pac_oracle_decode: PACFile.
ReadDataBlock + codec.Decode + the decode driver + PCMFile.WriteDataBlock) is
pinned byte for byte against:
  * the reference's own committed decodes outputs/*.wav (12 master files,
    SURVEY.md 8(c)) -- piano_test2 always (its .wak is a fixture, the
    output's sha256 is in tests/golden/decode_manifest.json), all 12 when
    /root/reference is present;
  * the reference decoder run through the semantics shim
    (tests/golden/make_decode_golden.py) on every encode golden and on
    harpsichord.pac (origin: the reference committed no matching decode).
"""
import hashlib
import json
import os

import pytest

from conftest import fixture, GOLD, REF, ROOT

import pyoracle as P

MAN = json.load(open(os.path.join(GOLD, "decode_manifest.json")))


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.mark.parametrize("name", sorted(MAN["shim"]))
def test_decode_equals_reference_shim(name):
    path = fixture(name[len("fixtures/"):]) if name.startswith("fixtures/") else os.path.join(GOLD, name)
    prof = P.ORIGIN if name.endswith(".pac") else P.MASTER
    assert sha(P.decode_file(path, prof)) == MAN["shim"][name]["sha256"]


def test_piano_test2_decode_equals_reference_output():
    got = P.decode_file(fixture("piano_test2.wak"), P.MASTER)
    assert sha(got) == MAN["reference_outputs"]["piano_test2"]


@pytest.mark.parametrize("name", sorted(MAN["reference_outputs"]))
def test_decode_equals_reference_outputs(name):
    """the reference's own decodes outputs/<name>.wav (sha256) of the committed .wak"""
    got = P.decode_file(fixture(name + ".wak"), P.MASTER)
    assert sha(got) == MAN["reference_outputs"][name]
    with open(os.path.join(REF, "outputs", name + ".wav"), "rb") as f:
        assert got == f.read()
