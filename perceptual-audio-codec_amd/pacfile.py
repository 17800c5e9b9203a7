"""PAC/WAK coded-file plugin -- mirror of the reference's pacfile.py:115-383.

``PACFile`` keeps the reference surface (ReadFileHeader / WriteFileHeader /
WriteDataBlock / Close / Encode) and file layout:

    'PAC ' <LHLLHH sampleRate nChannels numSamples nMDCTLines nScaleBits
    nMantSizeBits> <L nBands> <nBands H nLines>   then per block, per channel:
    <L nBytes> + nBytes of MSB-first packed bits.

Every block is encoded by the HIP kernels (``codec.Encode`` ->
``pac_encode_block``).  For throughput use the batch entry points
``encode_file`` / ``encode_streams`` which run whole streams in one GPU call
(``pac_encode_streams``); the bytes are identical.  Decoding
(``ReadDataBlock``, ``decode_file``, ``decode_streams``) runs on the GPU
through ``pac_decode_streams``: the file's data section is decoded in one call
when it is opened and ReadDataBlock hands out the reference's per-block
results (overlap-added signed fractions, then the final overlap half).
"""
import struct

import numpy as np

from . import _lib
from . import codec
from .audiofile import AudioFile, CodingParams
from .pcmfile import read_for_encode
from .psychoac import AssignMDCTLinesFromFreqLimits, ScaleFactorBands

PROFILE_ORIGIN = 0
PROFILE_MASTER = 1


def header_bytes(sampleRate, nChannels, numSamples, nMDCTLines=1024, nScaleBits=4,
                 nMantSizeBits=4):
    """File header as PACFile.WriteFileHeader writes it (pacfile.py:231-262),
    including the inverted zero-padding quirk (pacfile.py:240-242): only an
    exact multiple of nMDCTLines is bumped by one half-block."""
    ns = numSamples
    if not ns % nMDCTLines:
        ns += nMDCTLines - ns % nMDCTLines
    nLines = AssignMDCTLinesFromFreqLimits(nMDCTLines, sampleRate)
    h = b"PAC " + struct.pack("<LHLLHH", sampleRate, nChannels, ns, nMDCTLines, nScaleBits,
                              nMantSizeBits)
    h += struct.pack("<L", len(nLines)) + struct.pack("<%dH" % len(nLines), *nLines)
    return h


class PACFile(AudioFile):
    """Handlers for a perceptually coded audio file I am encoding/decoding."""

    tag = b"PAC "

    def __init__(self, filename, profile=PROFILE_MASTER, context=None, window=_lib.WINDOW_SINE):
        super().__init__(filename)
        self.profile = profile
        self.context = context
        self.window = window       # _lib.WINDOW_KBD: extension (parity unpinned), not in the file header

    def ReadFileHeader(self):
        tag = self.fp.read(4)
        if tag != self.tag:
            raise ValueError("Tried to read a non-PAC file into a PACFile object")
        (sampleRate, nChannels, numSamples, nMDCTLines, nScaleBits,
         nMantSizeBits) = struct.unpack("<LHLLHH", self.fp.read(struct.calcsize("<LHLLHH")))
        nBands = struct.unpack("<L", self.fp.read(4))[0]
        nLines = struct.unpack("<%dH" % nBands, self.fp.read(2 * nBands))
        p = CodingParams()
        p.sampleRate = sampleRate
        p.nChannels = nChannels
        p.numSamples = numSamples
        p.nMDCTLines = p.nSamplesPerBlock = nMDCTLines
        p.nScaleBits = nScaleBits
        p.nMantSizeBits = nMantSizeBits
        p.sfBands = ScaleFactorBands(nLines)
        p.overlapAndAdd = [np.zeros(nMDCTLines, dtype=np.float64) for _ in range(nChannels)]
        return p

    def ReadDataBlock(self, codingParams, huffman=None):
        """pacfile.py:153-229: the next block of reconstituted signed-fraction
        samples per channel (1024 each), the final overlap-and-add half at the
        end of the file, then None."""
        if getattr(self, "_dec", None) is None:
            data = self.fp.read()
            ctx = self.context or codec.default_context()
            # the header's values (the library rejects what the kernels do not
            # support); Huffman-coded (.wak) iff a Huffman object is passed, as
            # the master ReadDataBlock(codingParams, huffman) vs Origin's
            # ReadDataBlock(codingParams)
            prof = PROFILE_MASTER if huffman is not None else self.profile
            p = _lib.params(codingParams.sampleRate, codingParams.nChannels, prof, window=self.window)
            p.n_mdct_lines = int(codingParams.nMDCTLines)
            p.n_scale_bits = int(codingParams.nScaleBits)
            p.n_mant_size_bits = int(codingParams.nMantSizeBits)
            _, fo, fl = ctx.decode_streams(p, data, [0, len(data)], preroll=True, want_float=True)
            self._dec = fl
            self._pos = 0
        if self._pos >= self._dec.shape[0]:
            return None
        blk = self._dec[self._pos:self._pos + codingParams.nMDCTLines]
        self._pos += codingParams.nMDCTLines
        return [blk[:, c].copy() for c in range(codingParams.nChannels)]

    def WriteFileHeader(self, codingParams):
        self.fp.write(header_bytes(codingParams.sampleRate, codingParams.nChannels,
                                   codingParams.numSamples, codingParams.nMDCTLines,
                                   codingParams.nScaleBits, codingParams.nMantSizeBits))
        if not codingParams.numSamples % codingParams.nMDCTLines:
            codingParams.numSamples += (codingParams.nMDCTLines
                                        - codingParams.numSamples % codingParams.nMDCTLines)
        codingParams.sfBands = ScaleFactorBands(
            AssignMDCTLinesFromFreqLimits(codingParams.nMDCTLines, codingParams.sampleRate))
        codingParams.priorBlock = [np.zeros(codingParams.nMDCTLines, dtype=np.float64)
                                   for _ in range(codingParams.nChannels)]
        codingParams.extraBits = 0
        codingParams.curBlock = 0

    def WriteDataBlock(self, data, codingParams, huffman=None):
        full = [np.concatenate((codingParams.priorBlock[c], data[c]))
                for c in range(codingParams.nChannels)]
        codingParams.priorBlock = data
        raw = codec.encode_block_bytes(full, codingParams, huffman, self.profile, self.context)
        self.fp.write(raw)

    def Close(self, codingParams, huffman=None):
        if self.fp.mode == "wb":
            data = [np.zeros(codingParams.nMDCTLines) for _ in range(codingParams.nChannels)]
            self.WriteDataBlock(data, codingParams, huffman)
        self.fp.close()

    def Encode(self, data, codingParams, huffman=None):
        return codec.Encode(data, codingParams, huffman, profile=self.profile,
                            context=self.context)


# ---------------------------------------------------------------------------
# batch entry points (one GPU call for whole streams)
# ---------------------------------------------------------------------------

def encode_streams(streams, sample_rate, profile=PROFILE_MASTER, context=None, states=None,
                   window=_lib.WINDOW_SINE, block_switch=False):
    """Encode independent streams (list of int16 [frames, nCh] arrays sharing
    sample rate and channel count).  Returns a list of data-section bytes."""
    ctx = context or codec.default_context()
    nch = streams[0].shape[1]
    fo = np.zeros(len(streams) + 1, dtype=np.int64)
    fo[1:] = np.cumsum([s.shape[0] for s in streams])
    pcm = np.concatenate([np.ascontiguousarray(s, dtype=np.int16) for s in streams]) \
        if len(streams) > 1 else np.ascontiguousarray(streams[0], dtype=np.int16)
    p = _lib.params(sample_rate, nch, profile, window=window, block_switch=block_switch)
    out, so = ctx.encode_streams(p, pcm, fo, states=states)
    return [out[so[i]:so[i + 1]].tobytes() for i in range(len(streams))]


def encode_stream_parts(frames, sample_rate, parts, profile=PROFILE_MASTER, context=None,
                        window=_lib.WINDOW_SINE):
    """One stream encoded in `parts` calls (pac_amd.shard.split_stream): each
    call carries its priorBlock and, for the master profile, the reservoir
    state of the previous call (codingParams.extraBits, huffman.bitDeposit).
    Returns the data section -- identical to one call's.  Origin parts could
    run on different GPUs; here they run in order on one context."""
    from .shard import split_stream
    st = _lib.StreamState()
    body = b""
    for lo, hi, flags in split_stream(frames.shape[0], parts):
        st.flags = flags
        states = [st]
        body += encode_streams([frames[lo:hi]], sample_rate, profile, context, states=states, window=window)[0]
        st = states[0]
    return body


def encode_file(in_path, out_path=None, profile=PROFILE_MASTER, context=None, window=_lib.WINDOW_SINE, block_switch=False):
    """The reference driver's encode half (pacfile.py:430-499) for one file,
    as a single GPU call.  Returns the coded file bytes (and writes them)."""
    cp, frames = read_for_encode(in_path)
    body = encode_streams([frames], cp.sampleRate, profile, context, window=window, block_switch=block_switch)[0]
    data = header_bytes(cp.sampleRate, cp.nChannels, cp.numSamples) + body
    if out_path:
        with open(out_path, "wb") as f:
            f.write(data)
    return data


def encode_wav_files(wav_files, profile=PROFILE_MASTER, context=None, n_channels=None, sample_rate=None,
                     window=_lib.WINDOW_SINE, block_switch=False):
    """The encode driver (pacfile.py:430-499) for many WAV files (paths or
    bytes) sharing sample rate and channel count, with the WAV parsing on the
    device (pac_encode_wav).  Returns the coded files' bytes."""
    ctx = context or codec.default_context()
    blobs = []
    for w in wav_files:
        if isinstance(w, (bytes, bytearray)):
            blobs.append(bytes(w))
        else:
            with open(w, "rb") as f:
                blobs.append(f.read())
    fo = np.zeros(len(blobs) + 1, dtype=np.int64)
    fo[1:] = np.cumsum([len(b) for b in blobs])
    blob = b"".join(blobs)
    if sample_rate is None or n_channels is None:
        first = ctx.wav_scan(blobs[0], [0, len(blobs[0])])[0]
        if first.status:      # the reference's PCMFile raise for this file, not a parameter error
            raise _lib.PacError(_lib.PAC_E_ARG, "file 0: " + _lib.wav_status_message(first.status))
        sample_rate = sample_rate or first.sample_rate
        n_channels = n_channels or first.n_channels
    p = _lib.params(sample_rate, n_channels, profile, window=window, block_switch=block_switch)
    out, so, info = ctx.encode_wav(p, blob, fo)
    return [header_bytes(w.sample_rate, w.n_channels, w.num_samples) + out[so[i]:so[i + 1]].tobytes()
            for i, w in enumerate(info)]


# ---------------------------------------------------------------------------
# decoding (pacfile.py:153-229, codec.py:25-65, the driver pacfile.py:478-499)
# ---------------------------------------------------------------------------

def parse_header(b):
    """PACFile.ReadFileHeader on bytes: (sampleRate, nChannels, numSamples,
    nLines, offset of the data section)"""
    if b[:4] != PACFile.tag:
        raise ValueError("Tried to read a non-PAC file into a PACFile object")
    fs, nch, ns, nmdct, nsb, nmb = struct.unpack("<LHLLHH", b[4:22])
    nb = struct.unpack("<L", b[22:26])[0]
    nl = struct.unpack("<%dH" % nb, b[26:26 + 2 * nb])
    return fs, nch, ns, list(nl), 26 + 2 * nb


def decode_streams(sections, sample_rate, n_channels, profile=PROFILE_MASTER, context=None, preroll=False,
                   window=_lib.WINDOW_SINE, block_switch=False):
    """Decode independent data sections (bytes) sharing sample rate and channel
    count in one GPU call.  Returns a list of int16 [frames, nCh] arrays: the
    frames the reference's decode driver writes (or, with preroll, every
    ReadDataBlock result)."""
    ctx = context or codec.default_context()
    so = np.zeros(len(sections) + 1, dtype=np.int64)
    so[1:] = np.cumsum([len(x) for x in sections])
    p = _lib.params(sample_rate, n_channels, profile, window=window, block_switch=block_switch)
    pcm, fo, _ = ctx.decode_streams(p, b"".join(sections), so, preroll=preroll)
    return [pcm[fo[i]:fo[i + 1]] for i in range(len(sections))]


def wav_bytes(sampleRate, nChannels, numSamples, frames):
    """PCMFile.WriteFileHeader (sizes from numSamples, pcmfile.py:103-116)
    followed by the frames, as the reference decode driver writes them"""
    data_bytes = numSamples * nChannels * 2
    h = struct.pack("<4sL4s4sLHHLLHH4sL", b"RIFF", 36 + data_bytes, b"WAVE", b"fmt ", 16, 1, nChannels,
                    sampleRate, sampleRate * nChannels * 2, nChannels * 2, 16, b"data", data_bytes)
    return h + np.ascontiguousarray(frames, dtype="<i2").tobytes()


def decode_file(in_path, out_path=None, profile=PROFILE_MASTER, context=None, window=_lib.WINDOW_SINE, block_switch=False):
    """The reference driver's decode half (pacfile.py:430-499) for one coded
    file, as one GPU call.  Returns the output WAV bytes (and writes them)."""
    with open(in_path, "rb") as f:
        b = f.read()
    fs, nch, ns, _, off = parse_header(b)
    pcm = decode_streams([b[off:]], fs, nch, profile, context, window=window, block_switch=block_switch)[0]
    out = wav_bytes(fs, nch, ns, pcm)
    if out_path:
        with open(out_path, "wb") as f:
            f.write(out)
    return out


def decode_to_wav(coded_files, profile=PROFILE_MASTER, context=None, window=_lib.WINDOW_SINE, block_switch=False):
    """The decode driver (pacfile.py:430-499) for many coded files (bytes)
    sharing sample rate and channel count: the output WAV files' bytes, the
    WAV header and sample conversion written on the device (pac_decode_wav)."""
    ctx = context or codec.default_context()
    heads = [parse_header(b) for b in coded_files]
    fs, nch = heads[0][0], heads[0][1]
    secs = [b[h[4]:] for b, h in zip(coded_files, heads)]
    so = np.zeros(len(secs) + 1, dtype=np.int64)
    so[1:] = np.cumsum([len(x) for x in secs])
    p = _lib.params(fs, nch, profile, window=window, block_switch=block_switch)
    out, wo = ctx.decode_wav(p, b"".join(secs), so, [h[2] for h in heads])
    return [out[wo[i]:wo[i + 1]].tobytes() for i in range(len(secs))]
