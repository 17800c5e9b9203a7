"""The CPU oracle against the reference's own encodes of the M/S-extreme
streams (tests/msx.py): dual-mono (S == 0), anti-phase (M == 0), one silent
channel, sparse +-1 LSB differences, DC pairs and a stream cycling through
them, 201 blocks each, master and Origin coders, 44.1 and 48 kHz.  Bar:
byte-exact whole files, except the Origin coder on a constant channel, where
the sign of zero-magnitude mantissas is the sign of FFT rounding noise
(tests/msx.py docstring) and everything else must be equal.

Reference: codec/codec.py:94-102, psychoac.py:549-591,662-682,
bitalloc.py:157-184; Origin codec.py:52-67, bitalloc.py:129-202.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import pytest

import msx
import pyoracle as P

POOL = max(1, min(8, os.cpu_count() or 1))


def _oracle_file(name):
    c = msx.case(name)
    prof = P.MASTER if c["profile"] == "master" else P.ORIGIN
    x = msx.pcm(name)
    o = P.Oracle(c["fs"], huffman=(prof == P.MASTER))
    return P.pac_header(c["fs"], 2, x.shape[0], o.nlines()) + o.encode_data(prof, x)


@pytest.fixture(scope="module")
def oracle_files():
    for n in msx.CASES:           # regenerate (and hash-check) the inputs once, serially
        msx.pcm(n)
    with ThreadPoolExecutor(POOL) as ex:
        return dict(zip(msx.CASES, ex.map(_oracle_file, msx.CASES)))


def test_msx_inputs_are_the_extremes():
    """the generated streams are what their names say"""
    for fs in (44100, 48000):
        d = msx.pcm("dualmono_%dk_master.wak" % (fs // 1000))
        assert (d[:, 0] == d[:, 1]).all() and d.min() >= -32767 and (d != 0).mean() > 0.99
        a = msx.pcm("antiphase_%dk_master.wak" % (fs // 1000))
        assert (a[:, 0].astype(int) == -a[:, 1].astype(int)).all()
        r = msx.pcm("rsilent_%dk_master.wak" % (fs // 1000))
        assert (r[:, 1] == 0).all() and (r[:, 0] != 0).mean() > 0.99
        s = msx.pcm("lsb_%dk_master.wak" % (fs // 1000))
        diff = s[:, 0].astype(int) - s[:, 1].astype(int)
        assert set(diff.tolist()) <= {-1, 0, 1} and 0.001 < (diff != 0).mean() < 0.01
        c = msx.pcm("dcpure_%dk_master.wak" % (fs // 1000))
        assert (c[:, 0] == 10000).all() and (c[:, 1] == -3000).all()


@pytest.mark.parametrize("name", msx.CASES)
def test_oracle_vs_reference_msx(oracle_files, name):
    ref = msx.reference(name)
    got = oracle_files[name]
    if name not in msx.NOISE_SIGN:
        assert got == ref
        return
    assert got[:26] == ref[:26]
    ok, flips = msx.origin_equal_up_to_noise_signs(msx.data_section(got), msx.data_section(ref),
                                                   msx.nlines(msx.case(name)["fs"]))
    assert ok and flips > 0


def test_reference_mdct_signs_of_a_constant_are_noise():
    """The root cause of the NOISE_SIGN limit, on the oracle's own MDCT: the
    sine-windowed constant's 1 023 non-DC lines are rounding noise (< 1e-15
    of the DC line), so their signs carry no information the reference
    defines."""
    import numpy as np
    o = P.Oracle(44100, huffman=False)
    n = np.arange(2048)
    x = np.full(2048, 2 * 10000 / 65535.0) * np.sin(np.pi * (n + 0.5) / 2048)
    X = o.mdct(x)
    assert abs(X[0]) > 0.1
    assert np.abs(X[1:]).max() < 1e-15 * abs(X[0])
