"""GPU parity against every reference-held bitstream,
committed under tests/fixtures/ (MANIFEST.json): the whole files, encoded by
the HIP path through the C-ABI, byte for byte -- 3 origin .pac and 13 master
.wak -- and the reference's own decodes (outputs/*.wav, by sha256) of the 12
master files, decoded on the GPU.  All 16 streams are also encoded together
in one call per profile (independent streams sharing a launch)."""
import hashlib
import json
import os

import pytest

from conftest import GOLD, fixture

import pac_amd  # noqa: F401
from pac_amd import pacfile
from pac_amd.pcmfile import read_for_encode
from test_oracle import REF_FIXTURES
import pyoracle as P

pytestmark = pytest.mark.gpu
PROF = {P.ORIGIN: pacfile.PROFILE_ORIGIN, P.MASTER: pacfile.PROFILE_MASTER}


def _ref(coded):
    with open(fixture(coded), "rb") as f:
        return f.read()


@pytest.mark.parametrize("inp,coded,prof", REF_FIXTURES, ids=[c for _, c, _ in REF_FIXTURES])
def test_reference_bitstream_whole_file(ctx, inp, coded, prof):
    got = pacfile.encode_file(fixture(inp), profile=PROF[prof], context=ctx)
    ref = _ref(coded)
    assert len(got) == len(ref)
    assert got == ref


@pytest.mark.parametrize("prof", [P.ORIGIN, P.MASTER])
def test_reference_bitstreams_one_call(ctx, prof):
    """every input of the profile as independent streams of ONE encode call"""
    items = [(i, c) for i, c, p in REF_FIXTURES if p == prof]
    reads = [read_for_encode(fixture(i)) for i, _ in items]
    bodies = pacfile.encode_streams([fr for _, fr in reads], reads[0][0].sampleRate, PROF[prof], context=ctx)
    for (i, c), (cp, _), body in zip(items, reads, bodies):
        assert pacfile.header_bytes(cp.sampleRate, cp.nChannels, cp.numSamples) + body == _ref(c), c


MAN = json.load(open(os.path.join(GOLD, "decode_manifest.json")))


@pytest.mark.parametrize("name", sorted(MAN["reference_outputs"]))
def test_reference_decodes(ctx, name):
    """GPU decode of coded/<name>.wak == the reference's outputs/<name>.wav"""
    got = pacfile.decode_file(fixture(name + ".wak"), profile=pacfile.PROFILE_MASTER, context=ctx)
    assert hashlib.sha256(got).hexdigest() == MAN["reference_outputs"][name]
