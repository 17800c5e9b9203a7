"""Scale-factor band layout (host side of psychoac.py used by the file format).

Only the pieces the PACFile header needs live on the host:
``AssignMDCTLinesFromFreqLimits`` (psychoac.py:124-156) and
``ScaleFactorBands`` (psychoac.py:193-213).  The masking model itself runs in
the HIP kernels (csrc/pac_wave.h).
"""
import numpy as np

cbFreqLimits = (100.0, 200.0, 300.0, 400.0, 510.0, 630.0, 770.0, 920.0, 1080.0, 1270.0,
                1480.0, 1720.0, 2000.0, 2320.0, 2700.0, 3150.0, 3700.0, 4400.0, 5300.0,
                6400.0, 7700.0, 9500.0, 12000.0, 15500.0, 24000.0)


def AssignMDCTLinesFromFreqLimits(nMDCTLines, sampleRate, flimit=cbFreqLimits):
    """Lines per band; ``sampleRate / 2`` is Python-2 integer division there."""
    mdct_lines = (np.arange(nMDCTLines) + 0.5) / nMDCTLines * (int(sampleRate) // 2)
    lower = 0
    out = []
    for limit in flimit:
        upper = sampleRate / 2.0 if limit >= sampleRate / 2.0 else limit
        band = mdct_lines[mdct_lines <= upper]
        band = band[band > lower]
        out.append(len(band))
        lower = upper
    return out


class ScaleFactorBands:
    """Bands sharing a scale factor and a bit allocation (psychoac.py:193-213)."""

    def __init__(self, nLines):
        self.nBands = len(nLines)
        self.nLines = np.array(nLines)
        self.lowerLine = np.append(0, np.cumsum(nLines)[:-1])
        self.upperLine = np.add(self.nLines, np.subtract(self.lowerLine, 1))
