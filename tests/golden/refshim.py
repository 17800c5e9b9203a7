"""Build a Python-3 runnable copy of the reference codec in /tmp (never in the repo).

TEST-FIXTURE GENERATION ONLY.  Nothing in the product, the tests or bench.py
imports this; it is run by hand in the build container (where /root/reference
exists) by ``make_golden.py`` to produce the small vectors under tests/golden/.

The reference (wisamreid/Perceptual-Audio-Codec) is Python 2 + numpy 1.x.  The
copy applies only syntax and Py2/numpy-1 *semantics* edits (integer division,
builtin ``max``, value-based uint64 shifts, bytes literals) -- no algorithm
change -- following the recipe recorded in SURVEY.md section 8(c).  The Huffman
tables are read from our neutral export (``export_huffman_tables.py``), never
unpickled.

    python tests/golden/refshim.py      # (re)builds /tmp/pac_refshim/{master,origin}
"""
import os
import re
import shutil
import subprocess
import sys

REF = "/root/reference"
SHIM = "/tmp/pac_refshim"
HUFF_BIN = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..",
                                        "perceptual-audio-codec_amd", "data",
                                        "huffman_tables.bin"))

MODULES_MASTER = ["audiofile", "bitalloc", "bitpack", "codec", "mdct", "pacfile",
                  "pcmfile", "psychoac", "quantize", "window", "Huffman"]
MODULES_ORIGIN = ["audiofile", "bitalloc", "bitpack", "codec", "mdct", "pacfile",
                  "pcmfile", "psychoac", "quantize", "window"]

HUFF_INIT = '''
    def __init__(self):
        import struct as _st
        self.huffmanTables = {}
        with open(%r, "rb") as _f:
            _d = _f.read()
        assert _d[:8] == b"PACHUF01"
        _n = _st.unpack_from("<I", _d, 8)[0]; _o = 12
        for _t in range(_n):
            _tid, _ne, _el, _eb = _st.unpack_from("<IIII", _d, _o); _o += 16
            _enc = {-1: format(_eb, "0%%db" %% _el)}
            for _i in range(_ne):
                _s, _l, _b = _st.unpack_from("<iII", _d, _o); _o += 12
                _enc[_s] = format(_b, "0%%db" %% _l)
            self.huffmanTables[_tid] = HuffmanTable(_enc)
        self.histograms = {}
        self.ESCAPE_CODE = -1
        self.bitDeposit = 0
''' % HUFF_BIN


def _truncate_main(src):
    lines = src.splitlines()
    for i, ln in enumerate(lines):
        if re.match(r"^if\s+__name__\s*==", ln):
            lines = lines[:i]
            break
    return "\n".join(lines).expandtabs(4) + "\n"


def _sub(src, old, new, count=1, regex=False):
    n = len(re.findall(old, src)) if regex else src.count(old)
    if n < count:
        raise RuntimeError("shim edit failed: %r (found %d)" % (old, n))
    return re.sub(old, new, src) if regex else src.replace(old, new)


def edit(mod, src, profile):
    src = src.lstrip("﻿")
    if mod == "mdct":
        src = _sub(src, "N/2", "N//2")
    if mod == "psychoac":
        src = re.sub(r"(?m)^import solution\.psychoac_ as sol\n", "", src)
        src = "import builtins as _bi\n" + src
        src = _sub(src, "p = (1/2)*(a-r)/(a+r-2*b)", "p = 0*(a-r)/(a+r-2*b)")
        src = _sub(src, "Xwdb[freqs[idx]-1]", "Xwdb[int(freqs[idx])-1]")
        src = _sub(src, "Xwdb[freqs[idx]]", "Xwdb[int(freqs[idx])]")
        src = _sub(src, "Xwdb[freqs[idx]+1]", "Xwdb[int(freqs[idx])+1]")
        if profile == "master":
            src = _sub(src, "(freqs[idx]+p)*(sampleRate/N)", "(freqs[idx]+p)*(sampleRate//N)")
        else:
            src = _sub(src, "(freqs[idx]+p)*(fs/N)", "(freqs[idx]+p)*(fs//N)")
        src = _sub(src, "[0:N/2]", "[0:N//2]")
        src = _sub(src, "intensity=10**((spl-96)/10)",
                   "intensity=10**((spl-96)//10) if isinstance(spl, int) else 10**((spl-96)/10)")
        src = _sub(src, "max(self.SPL - 40.0, 0)", "_bi.max(self.SPL - 40.0, 0)", count=2)
    if mod == "quantize":
        src = _sub(src, "bool = np.bool\n", "bool = np.bool_\n")
        src = _sub(src, "aQuantizedNumVec[sign] += signBitMask",
                   "aQuantizedNumVec[sign] += np.uint64(signBitMask)")
        src = _sub(src, "mantissaVec = vQuantizeUniform(inputVals, R) << (scale + 1)",
                   "mantissaVec = vQuantizeUniform(inputVals, R) << np.uint64(scale + 1)")
        src = _sub(src, "mantissaVec >>= R - nMantBits + 1",
                   "mantissaVec >>= np.uint64(R - nMantBits + 1)")
        src = _sub(src, "mantissaVec[sign] += signBitMask",
                   "mantissaVec[sign] += np.uint64(signBitMask)")
    if mod == "bitpack":
        src = _sub(src, "self.data.tostring()", "self.data.tobytes()")
        src = _sub(src, "np.fromstring(data,dtype=np.uint8)",
                   "np.frombuffer(data,dtype=np.uint8).copy()")
        src = src.replace("&= self.data[self.iByte]", "&= int(self.data[self.iByte])")
        src = src.replace("dataMask = self.data[self.iByte]", "dataMask = int(self.data[self.iByte])")
        src = _sub(src, "        return info\n", "        return int(info)\n")
    if mod == "pcmfile":
        src = _sub(src, 'tag[0:4] != "RIFF" or tag[8:12]!= "WAVE"',
                   'tag[0:4] != b"RIFF" or tag[8:12]!= b"WAVE"')
        src = src.replace('raise "ERROR: File opened for PCMFile is not a RIFF file!"',
                          'raise Exception("not RIFF")')
        src = src.replace("raise \"ERROR: Didn't find WAV file 'fmt ' chunk following RIFF file header\"",
                          "raise Exception('no fmt')")
        src = _sub(src, 'tag[0:4] == "fmt "', 'tag[0:4] == b"fmt "')
        src = _sub(src, 'tag[0:4] == "data"', 'tag[0:4] == b"data"')
        src = _sub(src, "numSamples /= nChannels", "numSamples //= nChannels")
        src = src.replace("(codingParams.bitsPerSample/BYTESIZE)", "(codingParams.bitsPerSample//BYTESIZE)")
        src = _sub(src, '*"\\0"', '*b"\\0"')
        src = src.replace('"RIFF", chunkSize, "WAVE", "fmt "', 'b"RIFF", chunkSize, b"WAVE", b"fmt "')
        src = src.replace('codingParams.bitsPerSample, "data", dataBytes',
                          'codingParams.bitsPerSample, b"data", dataBytes')
        src = src.replace("dataBlock.tostring()", "dataBlock.tobytes()")
    if mod == "pacfile":
        src = _sub(src, "tag='PAC '", "tag=b'PAC '")
        src = src.replace('raise "Tried to read a non-PAC file into a PACFile object"',
                          'raise Exception("non-PAC")')
        src = src.replace('raise "Only read a partial block of coded PACFile data"',
                          'raise Exception("partial")')
        src = _sub(src, "nBytes /= BYTESIZE", "nBytes //= BYTESIZE")
        src = _sub(src, "nBytes = nBytes/BYTESIZE + 1", "nBytes = nBytes//BYTESIZE + 1")
        src = src.replace("dtype=np.float)", "dtype=float)")
    if mod == "Huffman":
        src = _sub(src, "import cPickle as pickle", "import pickle as _unused_pickle")
        src = re.sub(r"\n    def __init__\(self\):\n        with open\('huffmanTables.pickle'.*?self\.bitDeposit = 0\n",
                     HUFF_INIT, src, count=1, flags=re.S)
        assert "PACHUF01" in src
        src = _sub(src, "extraBit = self.bitDeposit/100", "extraBit = self.bitDeposit//100")
    if mod == "bitalloc":
        src = src.replace("print('*')", "pass")
    if mod == "codec" and profile == "master":
        src = _sub(src, "sum(len(huff) for huff in m)", "__import__('builtins').sum(len(huff) for huff in m)")
    return src


def build(profile):
    srcdir = os.path.join(REF, "codec" if profile == "master" else
                          "PerceptualAudioCodec_Origin/codec")
    dst = os.path.join(SHIM, profile)
    if os.path.exists(dst):
        shutil.rmtree(dst)
    os.makedirs(dst)
    mods = MODULES_MASTER if profile == "master" else MODULES_ORIGIN
    for m in mods:
        with open(os.path.join(srcdir, m + ".py"), encoding="utf-8") as f:
            src = _truncate_main(f.read())
        with open(os.path.join(dst, m + ".py"), "w") as f:
            f.write(src)
    subprocess.run([sys.executable, "-m", "lib2to3", "-w", "-n", "-f", "print", "-f",
                    "xrange", dst], check=True, capture_output=True)
    for m in mods:
        p = os.path.join(dst, m + ".py")
        with open(p) as f:
            src = f.read()
        with open(p, "w") as f:
            f.write(edit(m, src, profile))
    return dst


DRIVER = '''
import os, sys, numpy as np
from pcmfile import PCMFile
from pacfile import PACFile

def encode(inp, out, profile):
    """Mirror of the reference driver (pacfile.py __main__ encode half)."""
    huffman = None
    if profile == "master":
        from Huffman import Huffman
        huffman = Huffman()
    inFile = PCMFile(inp); outFile = PACFile(out)
    cp = inFile.OpenForReading()
    cp.nMDCTLines = 1024; cp.nScaleBits = 4; cp.nMantSizeBits = 4
    cp.targetBitsPerSample = 2.27
    if profile == "master": cp.nTableIDBits = 4
    cp.nSamplesPerBlock = cp.nMDCTLines
    outFile.OpenForWriting(cp)
    while True:
        data = inFile.ReadDataBlock(cp)
        if not data: break
        if huffman is None: outFile.WriteDataBlock(data, cp)
        else: outFile.WriteDataBlock(data, cp, huffman)
    inFile.Close(cp)
    z = [np.zeros(cp.nMDCTLines), np.zeros(cp.nMDCTLines)]
    if huffman is None: outFile.WriteDataBlock(z, cp)
    else: outFile.WriteDataBlock(z, cp, huffman)
    outFile.fp.close()
    return cp, huffman


def decode(inp, out, profile):
    """Mirror of the reference driver (pacfile.py __main__ decode half)."""
    huffman = None
    if profile == "master":
        from Huffman import Huffman
        huffman = Huffman()
    inFile = PACFile(inp); outFile = PCMFile(out)
    cp = inFile.OpenForReading()
    cp.bitsPerSample = 16
    if profile == "master": cp.nTableIDBits = 4
    outFile.OpenForWriting(cp)
    first = True
    while True:
        data = inFile.ReadDataBlock(cp, huffman) if huffman is not None else inFile.ReadDataBlock(cp)
        if not data: break
        if first:
            first = False
            continue
        outFile.WriteDataBlock(data, cp)
    inFile.Close(cp)
    outFile.Close(cp)
'''


def main():
    for prof in ("master", "origin"):
        d = build(prof)
        with open(os.path.join(d, "refdriver.py"), "w") as f:
            f.write(DRIVER)
        print("built", d)


if __name__ == "__main__":
    main()
