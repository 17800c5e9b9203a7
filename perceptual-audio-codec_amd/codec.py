"""Per-block encode entry -- mirror of the reference's codec.Encode
(codec.py:83-129, master) and Origin codec.Encode (Origin codec.py:52-67).

The computation runs in the HIP kernels through ``pac_encode_block``; this
module only marshals the reference's argument conventions (lists of float64
channel blocks, the mutable ``codingParams`` / ``huffman`` state) and returns
the reference's tuples:

  origin: (scaleFactor, bitAlloc, mantissa, overallScaleFactor)
  master: (scaleFactor, bitAlloc, signBits, huffmanCodedMantissa, tableID,
           overallScaleFactor, LRMS)
"""
import numpy as np

from . import _lib

PROFILE_ORIGIN = 0
PROFILE_MASTER = 1

_default_ctx = None


def default_context():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = _lib.Context(0)
    return _default_ctx


def _params_from(codingParams, profile):
    p = _lib.params(codingParams.sampleRate, codingParams.nChannels, profile,
                    getattr(codingParams, "targetBitsPerSample", 2.27),
                    window=getattr(codingParams, "window", _lib.WINDOW_SINE))   # KBD: extension
    p.n_mdct_lines = int(codingParams.nMDCTLines)
    p.n_scale_bits = int(codingParams.nScaleBits)
    p.n_mant_size_bits = int(codingParams.nMantSizeBits)
    p.n_table_id_bits = int(getattr(codingParams, "nTableIDBits", 4))
    return p


def _run(data, codingParams, huffman, profile, context):
    ctx = context or default_context()
    p = _params_from(codingParams, profile)
    full = np.stack([np.asarray(d, dtype=np.float64) for d in data])
    if full.shape[1] != 2 * codingParams.nMDCTLines:
        raise ValueError("expected priorBlock ++ data blocks of %d samples"
                         % (2 * codingParams.nMDCTLines))
    st = _lib.StreamState()
    if profile == PROFILE_MASTER:
        st.extra_bits = int(getattr(codingParams, "extraBits", 0))
        st.bit_deposit = int(huffman.bitDeposit) if huffman is not None else 0
    raw, fields, st = ctx.encode_block(p, full, st)
    if profile == PROFILE_MASTER:
        codingParams.extraBits = int(st.extra_bits)
        if huffman is not None:
            huffman.bitDeposit = int(st.bit_deposit)
    return raw, fields


def encode_block_bytes(data, codingParams, huffman=None, profile=PROFILE_MASTER, context=None):
    """Bytes PACFile.WriteDataBlock writes for one block (all channels)."""
    return _run(data, codingParams, huffman, profile, context)[0]


def Encode(data, codingParams, huffman=None, profile=PROFILE_MASTER, context=None):
    """codec.Encode: the block's coded fields, as the reference returns them."""
    raw, f = _run(data, codingParams, huffman, profile, context)
    nch = codingParams.nChannels
    nl = np.asarray(codingParams.sfBands.nLines if hasattr(codingParams, "sfBands")
                    else _lib.band_layout(codingParams.sampleRate), dtype=np.int64)
    scaleFactor = [np.array(f.sf[c][:], dtype=np.int32) for c in range(nch)]
    bitAlloc = [np.array(f.ba[c][:], dtype=np.int64) for c in range(nch)]
    overall = [int(f.overall[c]) for c in range(nch)]
    mant = []
    for c in range(nch):
        m = np.array(f.mant[c][:], dtype=np.int32)
        mant.append(m[:nl.sum()][np.repeat(bitAlloc[c] > 0, nl)])
    if profile == PROFILE_ORIGIN:
        return scaleFactor, bitAlloc, mant, overall
    # StripSignBits (codec.py:67-81) and huffman.encodeData's code strings
    # (Huffman.py:274-309) as the GPU pack kernel emitted them, one per coded
    # line in band order -- what PACFile.WriteDataBlock consumes (pacfile.py:296-336)
    signBits, huffCoded = [], []
    for c in range(nch):
        keep = np.repeat(bitAlloc[c] > 0, nl)
        ba = np.repeat(bitAlloc[c], nl)[keep]
        signBits.append([int(v >> (b - 1)) & 1 for v, b in zip(mant[c], ba)])
        codes = np.array(f.huff_code[c][:], dtype=np.uint64)[:nl.sum()][keep]
        lens = np.array(f.huff_len[c][:], dtype=np.int64)[:nl.sum()][keep]
        huffCoded.append([format(int(v), "0%db" % n) for v, n in zip(codes, lens)])
    tableID = [int(f.table_id[c]) for c in range(nch)]
    LRMS = np.array(f.lrms[:], dtype=np.int64)
    return scaleFactor, bitAlloc, signBits, huffCoded, tableID, overall, LRMS
