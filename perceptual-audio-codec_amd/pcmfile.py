"""16-bit PCM WAV file -- mirror of the reference's pcmfile.py:29-147.

``PCMFile`` keeps the reference's protocol and quirks (4-byte chunk-tag scan,
zero-padded final hop, -32768 read as +0.0).  ``read_for_encode`` returns the
whole stream as int16 frames exactly as the reference's hop-by-hop reads
would hand them to the encoder, for the batched GPU path.
"""
import struct

import numpy as np

from .audiofile import AudioFile, CodingParams

BYTESIZE = 8


def codes_to_float(codes):
    """int16 codes -> signed fractions (pcmfile.py:89-98 + quantize.py:120-145):
    +-2|c|/65535, with -32768 -> +0.0 (the sign-bit mask drops it)."""
    c = np.asarray(codes).astype(np.int64)
    a = np.abs(c)
    v = 2.0 * np.where(a == 32768, 0, a) / 65535.0
    return np.where((c < 0) & (c != -32768), -v, v)


def float_to_codes(x):
    """signed fractions -> int16 codes (pcmfile.py:127-134): magnitude through
    vQuantizeUniform(|x|, 16), cast to int16, then the sign re-applied."""
    x = np.asarray(x, dtype=np.float64)
    neg = np.signbit(x)
    a = np.abs(x)
    code = np.where(a < 1, np.floor((a * 65535.0 + 1.0) / 2.0), 32767).astype(np.int64)
    t = code.astype(np.int16)
    return np.where(neg, -t, t).astype(np.int16)


def _scan_header(fp):
    tag = fp.read(12)
    if tag[0:4] != b"RIFF" or tag[8:12] != b"WAVE":
        raise ValueError("ERROR: File opened for PCMFile is not a RIFF file!")
    while True:
        tag = fp.read(4)
        if len(tag) < 4:
            raise ValueError("ERROR: Didn't find WAV file 'fmt ' chunk following RIFF file header")
        if tag[0:4] == b"fmt ":
            break
    (formatSize, formatTag, nChannels, sampleRate, bytesPerSec, blockAlign,
     bitsPerSample) = struct.unpack("<LHHLLHH", fp.read(20))
    if formatTag != 1:
        raise ValueError("Opened a non-PCM WAV file as a PCMFile")
    if bitsPerSample != 16:
        raise ValueError("PCMFile was not 16-bits per sample")
    while True:
        tag = fp.read(4)
        if len(tag) < 4:
            raise ValueError("Didn't find WAV file 'data' chunk following 'fmt ' chunk")
        if tag[0:4] == b"data":
            break
    numSamples = struct.unpack("<L", fp.read(4))[0]
    numSamples //= nChannels * (bitsPerSample // BYTESIZE)
    return nChannels, sampleRate, bitsPerSample, numSamples


class PCMFile(AudioFile):
    """Handlers for a PCM file containing audio data in 16-bit PCM WAV format."""

    def ReadFileHeader(self):
        nCh, fs, bits, ns = _scan_header(self.fp)
        p = CodingParams()
        p.nChannels = nCh
        p.bitsPerSample = bits
        p.sampleRate = fs
        p.numSamples = ns
        p.bytesReadSoFar = 0
        return p

    def ReadDataBlock(self, codingParams):
        """Next nSamplesPerBlock frames as signed fractions per channel, or None."""
        bps = codingParams.bitsPerSample // BYTESIZE
        bytesToRead = codingParams.nSamplesPerBlock * codingParams.nChannels * bps
        left = codingParams.nChannels * codingParams.numSamples * bps - codingParams.bytesReadSoFar
        if left <= 0:
            block = None
        elif left < bytesToRead:
            block = self.fp.read(left)
        else:
            block = self.fp.read(bytesToRead)
        codingParams.bytesReadSoFar += bytesToRead
        if block and len(block) < bytesToRead:
            block += b"\0" * (bytesToRead - len(block))
        elif not block:
            return None
        codes = np.frombuffer(block, dtype="<i2").reshape(-1, codingParams.nChannels)
        return [codes_to_float(codes[:, c]) for c in range(codingParams.nChannels)]

    def WriteFileHeader(self, codingParams):
        bps = codingParams.bitsPerSample // BYTESIZE
        dataBytes = codingParams.numSamples * codingParams.nChannels * bps
        self.fp.write(struct.pack("<4sL4s4sLHHLLHH4sL", b"RIFF", 36 + dataBytes, b"WAVE", b"fmt ",
                                  16, 1, codingParams.nChannels, codingParams.sampleRate,
                                  codingParams.sampleRate * codingParams.nChannels * bps,
                                  codingParams.nChannels * bps, codingParams.bitsPerSample,
                                  b"data", dataBytes))

    def WriteDataBlock(self, data, codingParams):
        nCh = len(data)
        if nCh != codingParams.nChannels:
            raise ValueError("Data block to PCMFile did not have expected number of channels")
        n = min(len(d) for d in data)
        codes = np.stack([float_to_codes(np.asarray(d)[:n]) for d in data], axis=1)
        self.fp.write(codes.astype("<i2").tobytes())


def read_for_encode(path, nMDCTLines=1024):
    """(codingParams, frames int16 [n, nCh]) exactly as the reference driver's
    PCMFile.ReadDataBlock loop feeds PACFile.WriteDataBlock (pacfile.py:474-494).

    Mirrors the interaction with PACFile.WriteFileHeader's inverted padding
    quirk (pacfile.py:240-242): when numSamples is an exact multiple of
    nMDCTLines the header count is bumped by nMDCTLines, and the reader then
    tries one more hop, which picks up whatever bytes follow the data chunk.
    A file holding fewer data bytes than its header claims is read up to its
    last byte (the partial frame zero-padded, as ReadDataBlock pads a short
    read, pcmfile.py:73-78) and gets no extra hop: the next read comes back
    empty and the driver stops (pacfile.py:482).
    """
    with open(path, "rb") as fp:
        nCh, fs, bits, ns = _scan_header(fp)
        nbytes = ns * nCh * 2
        raw = fp.read(nbytes)
        extra = b""
        if len(raw) < nbytes:
            raw += b"\0" * (-len(raw) % (nCh * 2))
        elif ns % nMDCTLines == 0:
            extra = fp.read(nMDCTLines * nCh * 2)
    frames = np.frombuffer(raw, dtype="<i2").reshape(-1, nCh)
    if extra:
        pad = extra + b"\0" * (nMDCTLines * nCh * 2 - len(extra))
        frames = np.concatenate([frames, np.frombuffer(pad, dtype="<i2").reshape(-1, nCh)])
    p = CodingParams()
    p.nChannels = nCh
    p.bitsPerSample = bits
    p.sampleRate = fs
    p.numSamples = ns
    p.bytesReadSoFar = 0
    return p, np.ascontiguousarray(frames)
