"""ctypes binding of libpacgpu.so (include/pac_gpu.h).

The HIP library is the only compute path: if it is missing or cannot load,
every encode raises -- there is no CPU fallback.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PAC_LIB") or os.path.join(HERE, "libpacgpu.so")   # PAC_LIB: A/B builds
HUFF_PATH = os.path.join(HERE, "data", "huffman_tables.bin")

PAC_OK = 0
ERRORS = {-1: "PAC_E_ARG", -2: "PAC_E_HIP", -3: "PAC_E_NOMEM", -4: "PAC_E_UNSUPPORTED",
          -5: "PAC_E_TABLES", -6: "PAC_E_CAPACITY"}


PAC_E_ARG = -1
# pac_wav_info.status -> the reference's PCMFile raise (pcmfile.py:36-51), as
# wav_status_msg in csrc/pac_abi.hip
WAV_STATUS = {-1: "File opened for PCMFile is not a RIFF file!",
              -2: "Didn't find WAV file 'fmt ' chunk following RIFF file header",
              -3: "Opened a non-PCM WAV file as a PCMFile",
              -4: "PCMFile was not 16-bits per sample",
              -5: "Didn't find WAV file 'data' chunk following 'fmt ' chunk"}


def wav_status_message(status):
    return WAV_STATUS.get(status, "malformed WAV file")


class PacError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s: %s" % (ERRORS.get(code, code), msg))
        self.code = code


class Params(C.Structure):
    _fields_ = [("sample_rate", C.c_int32), ("n_channels", C.c_int32),
                ("n_mdct_lines", C.c_int32), ("n_scale_bits", C.c_int32),
                ("n_mant_size_bits", C.c_int32), ("n_table_id_bits", C.c_int32),
                ("target_bits_per_sample", C.c_double), ("profile", C.c_int32),
                ("window", C.c_int32), ("block_switch", C.c_int32)]


WINDOW_SINE = 0      # SineWindow (window.py:27-39): the reference coders
WINDOW_KBD = 1       # KBDWindow alpha 4 (window.py:56-78): extension, parity unpinned


STREAM_HAS_PRIOR = 1     # include/pac_gpu.h: first 1024 frames are the priorBlock
STREAM_NO_FLUSH = 2      # no Close() flush block: the stream continues in a later call


class StreamState(C.Structure):
    _fields_ = [("extra_bits", C.c_int64), ("bit_deposit", C.c_int64), ("flags", C.c_int32),
                ("reserved", C.c_int32)]


class WavInfo(C.Structure):       # pac_wav_info
    _fields_ = [("sample_rate", C.c_int32), ("n_channels", C.c_int32), ("bits_per_sample", C.c_int32),
                ("status", C.c_int32), ("num_samples", C.c_int64), ("data_offset", C.c_int64),
                ("frames", C.c_int64), ("extra_bytes", C.c_int64)]


class Timing(C.Structure):
    _fields_ = [("front_ms", C.c_float), ("alloc_ms", C.c_float), ("scan_ms", C.c_float),
                ("pack_ms", C.c_float), ("total_ms", C.c_float),
                ("n_channel_blocks", C.c_int64), ("out_bytes", C.c_int64),
                ("thr_ms", C.c_float), ("lrms_ms", C.c_float), ("thr_short_ms", C.c_float),
                ("spec_ms", C.c_float), ("emit_ms", C.c_float), ("chunks", C.c_int32), ("repacked", C.c_int32)]


class BlockFields(C.Structure):
    _fields_ = [("n_channels", C.c_int32), ("overall", C.c_int32 * 8),
                ("ba", (C.c_int32 * 25) * 8), ("sf", (C.c_int32 * 25) * 8),
                ("mant", (C.c_int32 * 1024) * 8), ("table_id", C.c_int32 * 8),
                ("lrms", C.c_int32 * 25), ("nbytes", C.c_int32 * 8),
                ("smr", (C.c_double * 25) * 8),
                ("huff_code", (C.c_uint64 * 1024) * 8), ("huff_len", (C.c_int32 * 1024) * 8)]


_lib = None


def lib():
    """Load libpacgpu.so (building it first if the sources are newer)."""
    global _lib
    if _lib is not None:
        return _lib
    from . import build as _build
    if not _build.up_to_date():
        if os.path.exists(_build.HIPCC):
            _build.build()
    if not os.path.exists(LIB_PATH):
        raise PacError(-2, "libpacgpu.so missing at %s (run python -m pac_amd.build); "
                           "there is no CPU fallback" % LIB_PATH)
    L = C.CDLL(LIB_PATH)
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    sig = {
        "pac_ctx_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "pac_ctx_destroy": (None, [vp]),
        "pac_last_error": (C.c_char_p, []),
        "pac_version": (C.c_int, []),
        "pac_huffman_load": (C.c_int, [vp, C.c_char_p, i64]),
        "pac_band_layout": (C.c_int, [i32, C.POINTER(i32)]),
        "pac_encode_streams": (C.c_int, [vp, C.POINTER(Params), i32, vp, C.POINTER(i64), i32, vp,
                                         i64, i32, C.POINTER(i64), C.POINTER(StreamState)]),
        "pac_encode_bound": (i64, [C.POINTER(Params), i32, C.POINTER(i64)]),
        "pac_decode_streams": (C.c_int, [vp, C.POINTER(Params), i32, vp, C.POINTER(i64), i32, i32, vp, i64,
                                         i32, vp, C.POINTER(i64)]),
        "pac_decode_layout": (C.c_int, [C.POINTER(Params), i32, vp, C.POINTER(i64), i32, C.POINTER(i64)]),
        "pac_wav_scan": (C.c_int, [vp, i32, vp, C.POINTER(i64), i32, C.POINTER(WavInfo)]),
        "pac_encode_wav": (C.c_int, [vp, C.POINTER(Params), i32, vp, C.POINTER(i64), i32, vp, i64, i32,
                                     C.POINTER(i64), C.POINTER(StreamState), C.POINTER(WavInfo)]),
        "pac_decode_wav": (C.c_int, [vp, C.POINTER(Params), i32, vp, C.POINTER(i64), i32, C.POINTER(i64), vp, i64,
                                     i32, C.POINTER(i64)]),
        "pac_encode_block": (C.c_int, [vp, C.POINTER(Params), vp, C.POINTER(StreamState), vp, i64,
                                       C.POINTER(i64), C.POINTER(BlockFields)]),
        "pac_device_alloc": (C.c_int, [vp, i64, C.POINTER(vp)]),
        "pac_device_free": (C.c_int, [vp, vp]),
        "pac_copy_to_device": (C.c_int, [vp, vp, vp, i64]),
        "pac_copy_to_host": (C.c_int, [vp, vp, vp, i64]),
        "pac_synth_white": (C.c_int, [vp, vp, i64, C.c_uint64]),
        "pac_synth_pink_tones": (C.c_int, [vp, vp, i64, C.c_int32, C.c_uint64]),
        "pac_synth_bursts": (C.c_int, [vp, vp, i64, i64, C.c_uint64]),
        "pac_sync": (C.c_int, [vp]),
        "pac_set_timing": (C.c_int, [vp, i32]),
        "pac_set_chunk_blocks": (C.c_int, [vp, i64]),
        "pac_last_timing": (C.c_int, [vp, C.POINTER(Timing)]),
        "pac_debug_threshold": (C.c_int, [vp, i32, i32, vp, i32, vp, vp]),
        "pac_debug_mdct": (C.c_int, [vp, i32, vp, vp]),
        "pac_debug_mdct_dft": (C.c_int, [vp, i32, vp, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(rc):
    if rc != PAC_OK:
        msg = lib().pac_last_error()
        raise PacError(rc, msg.decode() if msg else "")
    return rc


def band_layout(sample_rate):
    out = (C.c_int32 * 25)()
    check(lib().pac_band_layout(int(sample_rate), out))
    return np.array(out[:], dtype=np.int64)


class Context:
    """One device context (pac_ctx): stream, tables, work buffers."""

    def __init__(self, device=0, huffman=True):
        L = lib()
        h = C.c_void_p()
        check(L.pac_ctx_create(int(device), C.byref(h)))
        self.h = h
        self.L = L
        self.device = device
        if huffman and os.path.exists(HUFF_PATH):
            with open(HUFF_PATH, "rb") as f:
                img = f.read()
            check(L.pac_huffman_load(self.h, img, len(img)))

    def close(self):
        if getattr(self, "h", None):
            self.L.pac_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- encode ---------------------------------------------------------
    def encode_streams(self, params, pcm, frame_offsets, out=None, out_capacity=None,
                       pcm_is_device=False, out_is_device=False, states=None):
        """pcm: host int16 array (frames x channels, streams back to back) or a
        device pointer (int) when pcm_is_device.  Returns (out, stream_offsets)."""
        fo = np.ascontiguousarray(frame_offsets, dtype=np.int64)
        ns = len(fo) - 1
        fo_p = fo.ctypes.data_as(C.POINTER(C.c_int64))
        if out is None:
            cap = int(self.L.pac_encode_bound(C.byref(params), ns, fo_p))
            out = np.empty(max(cap, 1), dtype=np.uint8)
        if isinstance(out, np.ndarray):
            out_ptr = out.ctypes.data
            cap = out.nbytes if out_capacity is None else out_capacity
        else:
            out_ptr = out
            cap = out_capacity
        if pcm_is_device:
            pcm_ptr = pcm
        else:
            pcm = np.ascontiguousarray(pcm, dtype=np.int16)
            pcm_ptr = pcm.ctypes.data
        so = np.zeros(ns + 1, dtype=np.int64)
        st = None
        if states is not None:
            st = (StreamState * ns)(*states)
        check(self.L.pac_encode_streams(self.h, C.byref(params), ns, pcm_ptr, fo_p,
                                        int(bool(pcm_is_device)), out_ptr, int(cap),
                                        int(bool(out_is_device)),
                                        so.ctypes.data_as(C.POINTER(C.c_int64)),
                                        st if st is not None else None))
        if states is not None:
            for i in range(ns):
                states[i] = st[i]
        return out, so

    def decode_streams(self, params, data, stream_offsets, preroll=False, want_float=False,
                       data_is_device=False, out=None, out_capacity_frames=None, out_is_device=False):
        """Decode data sections (bytes / uint8 array, or a device pointer when
        data_is_device) delimited by stream_offsets.  Returns (pcm, frame
        offsets, float samples or None); pcm is int16 [frames, nCh] unless
        out_is_device (then `out` is returned)."""
        so = np.ascontiguousarray(stream_offsets, dtype=np.int64)
        ns = len(so) - 1
        fo = np.zeros(ns + 1, dtype=np.int64)
        if data_is_device:
            dptr = data
        else:
            buf = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
            buf = np.ascontiguousarray(buf, dtype=np.uint8)
            dptr = buf.ctypes.data
        nch = params.n_channels
        args = [self.h, C.byref(params), ns, dptr, so.ctypes.data_as(C.POINTER(C.c_int64)),
                int(bool(data_is_device)), int(bool(preroll))]
        fo_p = fo.ctypes.data_as(C.POINTER(C.c_int64))
        if out is None:      # output size: host-side layout walk (host data) or a size query (device data)
            if data_is_device:
                rc = self.L.pac_decode_streams(*args, None, 0, 0, None, fo_p)
                if rc not in (PAC_OK, -6):
                    check(rc)
            else:
                check(self.L.pac_decode_layout(C.byref(params), ns, dptr, so.ctypes.data_as(C.POINTER(C.c_int64)),
                                               int(bool(preroll)), fo_p))
            frames = int(fo[-1])
            if out_is_device:
                raise ValueError("out_is_device needs an out pointer")
            out = np.zeros((max(frames, 1), nch), dtype=np.int16)
            cap = frames
        else:
            cap = out_capacity_frames if out_capacity_frames is not None else out.shape[0]
        fl = np.zeros((max(int(fo[-1]) if fo[-1] else cap, 1), nch)) if want_float else None
        optr = out if out_is_device else out.ctypes.data
        check(self.L.pac_decode_streams(*args, optr, int(cap), int(bool(out_is_device)),
                                        fl.ctypes.data if want_float else None, fo_p))
        frames = int(fo[-1])
        if out_is_device:
            return out, fo, (fl[:frames] if want_float else None)
        return out[:frames], fo, (fl[:frames] if want_float else None)

    # --- WAV ingest / egress on the device --------------------------------
    def wav_scan(self, blob, file_offsets, blob_is_device=False):
        fo = np.ascontiguousarray(file_offsets, dtype=np.int64)
        n = len(fo) - 1
        info = (WavInfo * n)()
        ptr = blob if blob_is_device else np.ascontiguousarray(np.frombuffer(blob, dtype=np.uint8)).ctypes.data
        keep = blob
        check(self.L.pac_wav_scan(self.h, n, ptr, fo.ctypes.data_as(C.POINTER(C.c_int64)), int(bool(blob_is_device)),
                                  info))
        del keep
        return list(info)

    def encode_wav(self, params, blob, file_offsets, blob_is_device=False, out=None, out_capacity=None,
                   out_is_device=False, states=None):
        """pac_encode_wav: WAV files back to back in blob (bytes, or a device
        pointer).  Returns (out, stream byte offsets, [WavInfo])."""
        fo = np.ascontiguousarray(file_offsets, dtype=np.int64)
        n = len(fo) - 1
        info = (WavInfo * n)()
        if blob_is_device:
            ptr = blob
        else:
            arr = np.frombuffer(blob, dtype=np.uint8)
            ptr = arr.ctypes.data
        if out is None:
            # pac_encode_bound over the frames the device scan finds (a bad file
            # counts 0: the encode call reports it)
            scan = self.wav_scan(blob, fo, blob_is_device=blob_is_device)
            ffo = np.zeros(n + 1, dtype=np.int64)
            ffo[1:] = np.cumsum([w.frames if w.status == 0 else 0 for w in scan])
            cap = int(self.L.pac_encode_bound(C.byref(params), n, ffo.ctypes.data_as(C.POINTER(C.c_int64))))
            out = np.empty(max(cap, 1), dtype=np.uint8)
        if isinstance(out, np.ndarray):
            out_ptr, cap = out.ctypes.data, (out.nbytes if out_capacity is None else out_capacity)
        else:
            out_ptr, cap = out, out_capacity
        so = np.zeros(n + 1, dtype=np.int64)
        st = (StreamState * n)(*states) if states is not None else None
        check(self.L.pac_encode_wav(self.h, C.byref(params), n, ptr, fo.ctypes.data_as(C.POINTER(C.c_int64)),
                                    int(bool(blob_is_device)), out_ptr, int(cap), int(bool(out_is_device)),
                                    so.ctypes.data_as(C.POINTER(C.c_int64)), st, info))
        if states is not None:
            for i in range(n):
                states[i] = st[i]
        return out, so, list(info)

    def decode_wav(self, params, data, stream_offsets, num_samples):
        """pac_decode_wav: data sections (bytes) -> the decode driver's WAV files
        (bytes, back to back) and their offsets."""
        so = np.ascontiguousarray(stream_offsets, dtype=np.int64)
        n = len(so) - 1
        ns = np.ascontiguousarray(num_samples, dtype=np.int64)
        buf = np.frombuffer(bytes(data), dtype=np.uint8)
        fo = np.zeros(n + 1, dtype=np.int64)
        P64 = C.POINTER(C.c_int64)
        check(self.L.pac_decode_layout(C.byref(params), n, buf.ctypes.data, so.ctypes.data_as(P64), 0,
                                       fo.ctypes.data_as(P64)))
        cap = int(fo[-1]) * params.n_channels * 2 + 44 * n
        out = np.empty(max(cap, 1), dtype=np.uint8)
        wo = np.zeros(n + 1, dtype=np.int64)
        check(self.L.pac_decode_wav(self.h, C.byref(params), n, buf.ctypes.data, so.ctypes.data_as(P64), 0,
                                    ns.ctypes.data_as(P64), out.ctypes.data, cap, 0, wo.ctypes.data_as(P64)))
        return out, wo

    def encode_block(self, params, full_block, state=None):
        fb = np.ascontiguousarray(full_block, dtype=np.float64)
        out = np.empty(8 * 4200, dtype=np.uint8)
        n = C.c_int64()
        fields = BlockFields()
        st = state if state is not None else StreamState()
        check(self.L.pac_encode_block(self.h, C.byref(params), fb.ctypes.data, C.byref(st),
                                      out.ctypes.data, out.nbytes, C.byref(n), C.byref(fields)))
        return out[:n.value].tobytes(), fields, st

    # --- device memory / timing -----------------------------------------
    def alloc(self, nbytes):
        p = C.c_void_p()
        check(self.L.pac_device_alloc(self.h, int(nbytes), C.byref(p)))
        return p.value

    def free(self, ptr):
        check(self.L.pac_device_free(self.h, ptr))

    def to_device(self, dst, arr):
        arr = np.ascontiguousarray(arr)
        check(self.L.pac_copy_to_device(self.h, dst, arr.ctypes.data, arr.nbytes))

    def to_host(self, arr, src):
        check(self.L.pac_copy_to_host(self.h, arr.ctypes.data, src, arr.nbytes))
        return arr

    def synth_white(self, dev_pcm, n_samples, seed):
        check(self.L.pac_synth_white(self.h, dev_pcm, int(n_samples), int(seed)))

    def synth_pink_tones(self, dev_pcm, n_frames, sample_rate, seed):
        check(self.L.pac_synth_pink_tones(self.h, dev_pcm, int(n_frames), int(sample_rate), int(seed)))

    def synth_bursts(self, dev_pcm, n_frames, period, seed):
        check(self.L.pac_synth_bursts(self.h, dev_pcm, int(n_frames), int(period), int(seed)))

    def debug_threshold(self, sample_rate, data, no_drop=False):
        d = np.ascontiguousarray(np.atleast_2d(data), dtype=np.float64)
        n = d.shape[0]
        thr = np.zeros((n, 1024))
        npk = np.zeros(n, dtype=np.int32)
        check(self.L.pac_debug_threshold(self.h, int(sample_rate), n, d.ctypes.data, int(no_drop),
                                         thr.ctypes.data, npk.ctypes.data))
        return thr, npk

    def debug_mdct(self, data):
        d = np.ascontiguousarray(np.atleast_2d(data), dtype=np.float64)
        X = np.zeros((d.shape[0], 1024))
        check(self.L.pac_debug_mdct(self.h, d.shape[0], d.ctypes.data, X.ctypes.data))
        return X

    def debug_mdct_dft(self, data):
        d = np.ascontiguousarray(np.atleast_2d(data), dtype=np.float64)
        X = np.zeros((d.shape[0], 1024))
        check(self.L.pac_debug_mdct_dft(self.h, d.shape[0], d.ctypes.data, X.ctypes.data))
        return X

    def sync(self):
        check(self.L.pac_sync(self.h))

    def set_timing(self, on):
        check(self.L.pac_set_timing(self.h, int(bool(on))))

    def last_timing(self):
        t = Timing()
        check(self.L.pac_last_timing(self.h, C.byref(t)))
        return t


def params(sample_rate, n_channels, profile, target_bits_per_sample=2.27, window=WINDOW_SINE,
           block_switch=False):
    p = Params()
    p.sample_rate = int(sample_rate)
    p.n_channels = int(n_channels)
    p.n_mdct_lines = 1024
    p.n_scale_bits = 4
    p.n_mant_size_bits = 4
    p.n_table_id_bits = 4
    p.target_bits_per_sample = float(target_bits_per_sample)
    p.profile = int(profile)
    p.window = int(window)
    p.block_switch = 1 if block_switch else 0
    return p
