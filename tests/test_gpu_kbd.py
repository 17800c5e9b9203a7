"""KBD window extension (window.py:56-78, alpha 4, as the
MDCT window of encoder and decoder).  No reference coder uses it, so parity is
UNPINNED against the reference: the HIP path is checked byte for byte against
the oracle restated with the same window (oracle/pac_oracle.c
pac_oracle_set_window, itself within 1.4e-15 of a numpy restatement of
window.py:56-78 -- tests/test_oracle.py::test_kbd_window_matches_window_py),
and the decode of a KBD stream against the oracle's."""
import numpy as np
import pytest

import pac_amd  # noqa: F401
from pac_amd import pacfile, synth, _lib
import pyoracle as P

pytestmark = pytest.mark.gpu
KBD = _lib.WINDOW_KBD


@pytest.mark.parametrize("prof", [pacfile.PROFILE_ORIGIN, pacfile.PROFILE_MASTER])
@pytest.mark.parametrize("fs", [44100, 48000])
def test_kbd_encode_decode_vs_oracle(ctx, prof, fs):
    streams = [synth.pink_tones_pcm(n, fs, seed=n) for n in (5000, 20 * 1024, 33 * 1024 + 17)]
    got = pacfile.encode_streams(streams, fs, prof, context=ctx, window=KBD)
    sine = pacfile.encode_streams(streams, fs, prof, context=ctx)
    o = P.Oracle(fs, huffman=(prof == pacfile.PROFILE_MASTER), window=1)
    op = P.MASTER if prof == pacfile.PROFILE_MASTER else P.ORIGIN
    for s, g, sn in zip(streams, got, sine):
        assert g == o.encode_data(op, s)
        assert g != sn                       # the window is really in use
        dec = pacfile.decode_streams([g], fs, 2, prof, context=ctx, window=KBD)[0]
        assert np.array_equal(dec, o.decode_data(op, g, 2))
