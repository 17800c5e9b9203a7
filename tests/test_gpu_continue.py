"""Stream continuation across calls (pac_stream_state flags, SURVEY.md 5 and
8(e)): a stream encoded in several calls -- each later call carrying its
priorBlock, all but the last without the Close() flush block, the master
reservoir handed from call to call -- gives exactly the one-call bytes, and
so the reference's file for the fixtures.  For the origin profile this is
also the block-range split of one stream over GPUs with a one-hop halo."""
import pytest

from conftest import fixture

import pac_amd  # noqa: F401
from pac_amd import pacfile, synth, _lib
from pac_amd.pcmfile import read_for_encode

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("parts", [2, 3, 5, 16])
@pytest.mark.parametrize("name,prof", [("harpsichord", pacfile.PROFILE_ORIGIN),
                                       ("piano_test2", pacfile.PROFILE_MASTER)])
def test_reference_file_in_parts(ctx, name, prof, parts):
    cp, fr = read_for_encode(fixture(name + ".wav"))
    body = pacfile.encode_stream_parts(fr, cp.sampleRate, parts, prof, context=ctx)
    got = pacfile.header_bytes(cp.sampleRate, cp.nChannels, cp.numSamples) + body
    with open(fixture(name + (".pac" if prof == pacfile.PROFILE_ORIGIN else ".wak")), "rb") as f:
        assert got == f.read()


@pytest.mark.parametrize("n", [1, 1024, 1025, 9 * 1024, 9 * 1024 + 700])
@pytest.mark.parametrize("prof", [pacfile.PROFILE_ORIGIN, pacfile.PROFILE_MASTER])
def test_synthetic_in_parts(ctx, n, prof):
    pcm = synth.pink_tones_pcm(n, 48000, seed=n)
    one = pacfile.encode_streams([pcm], 48000, prof, context=ctx)[0]
    for parts in (2, 4, 9):
        assert pacfile.encode_stream_parts(pcm, 48000, parts, prof, context=ctx) == one, parts


def test_origin_parts_independent_calls_in_one_batch(ctx):
    """origin parts need no state: all parts of a stream as independent streams
    of ONE call (what a rank would do with its block range), concatenated"""
    from pac_amd import shard
    cp, fr = read_for_encode(fixture("harpsichord.wav"))
    sp = shard.split_stream(fr.shape[0], 6)
    states = [_lib.StreamState() for _ in sp]
    for st, (_, _, fl) in zip(states, sp):
        st.flags = fl
    bodies = pacfile.encode_streams([fr[lo:hi] for lo, hi, _ in sp], cp.sampleRate, pacfile.PROFILE_ORIGIN,
                                    context=ctx, states=states)
    with open(fixture("harpsichord.pac"), "rb") as f:
        ref = f.read()
    assert pacfile.header_bytes(cp.sampleRate, cp.nChannels, cp.numSamples) + b"".join(bodies) == ref


def test_no_new_hop_is_empty(ctx):
    st = _lib.StreamState()
    st.flags = _lib.STREAM_HAS_PRIOR | _lib.STREAM_NO_FLUSH
    out = pacfile.encode_streams([synth.white_pcm(1024, 2, seed=1)], 48000, pacfile.PROFILE_ORIGIN, context=ctx,
                                 states=[st])
    assert out == [b""]
