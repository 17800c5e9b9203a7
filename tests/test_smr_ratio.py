"""The SMR-as-intensity-ratio identity the master and origin kernels use
(pac_common.h pac_spl_ratio / pac_ratio_db), checked on the
host against a restatement of the reference's SPL() (psychoac.py:15-33, whose
Python-2 minval Intensity(-30) is 10**-13 and whose result is clamped at
-30 dB):

    SPL(P) - SPL(I) = 10 log10(max(P, 10^-12.6) / I)   for I above the floor,

and the band maximum of SMR terms is 10 log10 of the band maximum of the
ratios (SPL is monotone).  The MLD thresholds enter the M/S combination
max(BTHR_M, min(BTHR_S, MLD_S)) as intensities 10^((mld SPL(I) - 96)/10)
(pac_mld_intensity): the combination commutes with that monotone map.
Tolerance: 1e-11 dB (the GPU threshold probes' bar)."""
import numpy as np

IMIN = 2.51188643150958e-13          # PAC_SPL_IMIN


def ref_spl(x):
    """psychoac.py SPL(): minval 10**-13 (Python 2 integer division), -30 dB clamp"""
    x = np.maximum(np.asarray(x, dtype=np.float64), 1e-13)
    s = 96.0 + 10.0 * np.log10(x)
    return np.maximum(s, -30.0)


def ratio_db(P, I):
    return 10.0 * np.log10(np.maximum(P, IMIN) / I)


def test_floor_constant_is_minus_30_db():
    assert abs(96.0 + 10.0 * np.log10(IMIN) + 30.0) < 1e-12
    assert ref_spl(IMIN * 0.999) == -30.0


def test_spl_difference_is_log_ratio():
    rng = np.random.default_rng(7)
    # MDCT intensities from exactly zero through the floor to full scale; threshold
    # intensities over the range the threshold in quiet and the maskers give
    P = np.concatenate([np.zeros(64), 10.0 ** rng.uniform(-16, 0.7, 200000)])
    I = 10.0 ** rng.uniform(-10.5, 8.0, P.size)
    d = (ref_spl(P) - ref_spl(I)) - ratio_db(P, I)
    assert np.max(np.abs(d)) < 1e-11


def test_band_maximum_commutes():
    rng = np.random.default_rng(11)
    for _ in range(200):
        n = int(rng.integers(1, 120))
        P = 10.0 ** rng.uniform(-15, 0.5, n)
        P[rng.random(n) < 0.1] = 0.0
        I = 10.0 ** rng.uniform(-10, 6, n)
        off = 6.02 * int(rng.integers(0, 16))
        ref = np.max((ref_spl(P) - off) - ref_spl(I))          # calcStereoSMR's band max
        got = 10.0 * np.log10(np.max(np.maximum(P, IMIN) / I)) - off
        assert abs(ref - got) < 1e-11


def test_mld_combination_on_intensities():
    rng = np.random.default_rng(13)
    n = 100000
    bM, bS, bSm = (10.0 ** rng.uniform(-10, 6, n) for _ in range(3))
    mld = rng.uniform(0.05, 1.0, n)
    # reference: dB domain, MLD_S = BTHR_S_MLD * mld
    thr_db = np.maximum(ref_spl(bM), np.minimum(ref_spl(bS), ref_spl(bSm) * mld))
    # kernels: intensities, MLD_S as 10^((mld SPL - 96)/10)
    mld_i = 10.0 ** ((ref_spl(bSm) * mld - 96.0) / 10.0)
    thr_i = np.maximum(bM, np.minimum(bS, mld_i))
    assert np.max(np.abs(ref_spl(thr_i) - thr_db)) < 1e-11
