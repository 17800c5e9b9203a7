/*
 * pac_gpu.h -- C-ABI of the MI355X (gfx950) PAC/WAK encoder, libpacgpu.so.
 *
 * Drop-in boundary for the reference's per-block encode path
 * (wisamreid/Perceptual-Audio-Codec).  Plain C types only; no torch types.
 * Every entry point names the reference interface it replaces.  Built by
 * perceptual-audio-codec_amd/build.py (hipcc --offload-arch=gfx950).
 *
 * Conventions: every int-returning function returns PAC_OK (0) or a negative
 * PAC_E_* code; pac_last_error() then holds a thread-local message.  A context
 * is bound to one device and one HIP stream and is not thread-safe; use one
 * context per device / host thread (pacfile.py's encoder is single-threaded).
 */
#ifndef PAC_GPU_H
#define PAC_GPU_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PAC_OK 0
#define PAC_E_ARG (-1)          /* bad argument (reference: raise / assert)          */
#define PAC_E_HIP (-2)          /* HIP runtime failure                               */
#define PAC_E_NOMEM (-3)        /* device or host allocation failed                  */
#define PAC_E_UNSUPPORTED (-4)  /* parameter outside what the reference encoder does */
#define PAC_E_TABLES (-5)       /* Huffman table image missing or malformed          */
#define PAC_E_CAPACITY (-6)     /* output buffer too small                           */

/* Coder variants of the reference repository:
 *  ORIGIN: PerceptualAudioCodec_Origin/codec/ (per-channel, no M/S, .pac)
 *  MASTER: codec/ (M/S decision, Huffman, bit reservoir, .wak)             */
#define PAC_PROFILE_ORIGIN 0
#define PAC_PROFILE_MASTER 1

typedef struct pac_ctx pac_ctx;

/* CodingParams attribute bag (audiofile.py:51-53) as set by the driver
 * (pacfile.py:452-461 / Origin pacfile.py:391-398). */
typedef struct {
    int32_t sample_rate;            /* codingParams.sampleRate                 */
    int32_t n_channels;             /* nChannels (master: 2; 1 = mono ext.)    */
    int32_t n_mdct_lines;           /* codingParams.nMDCTLines (1024)          */
    int32_t n_scale_bits;           /* codingParams.nScaleBits (4)             */
    int32_t n_mant_size_bits;       /* codingParams.nMantSizeBits (4)          */
    int32_t n_table_id_bits;        /* codingParams.nTableIDBits (4, master)   */
    double target_bits_per_sample;  /* codingParams.targetBitsPerSample (2.27) */
    int32_t profile;                /* PAC_PROFILE_*                           */
    int32_t window;                 /* PAC_WINDOW_SINE (the reference), or
                                       PAC_WINDOW_KBD: KBDWindow alpha 4
                                       (window.py:56-78) as the MDCT window of
                                       encoder and decoder -- an extension no
                                       reference coder uses (parity unpinned) */
    int32_t block_switch;           /* 0 (the reference), or 1: block switching
                                       between one N = 2048 and four N = 512
                                       MDCTs per frame with attack detection --
                                       an extension (parity unpinned), master
                                       profile only, whole streams only (no
                                       PAC_STREAM_* continuation flags), not
                                       with pac_encode_block; a short frame is
                                       marked by one bit after the LRMS bits */
} pac_params;
#define PAC_WINDOW_SINE 0
#define PAC_WINDOW_KBD 1

/* Cross-block encoder state of one stream, so that a stream can be encoded
 * across calls (streaming, or an origin stream split over GPUs with a one-hop
 * halo): codingParams.extraBits (codec.py:229,260) and huffman.bitDeposit
 * (Huffman.py:262,353-371), both MASTER only, and the framing flags:
 *   PAC_STREAM_HAS_PRIOR  the stream's first 1024 frames are codingParams.
 *                         priorBlock (pacfile.py:279-282): read as the first
 *                         block's first half, not encoded as a hop of their own
 *                         (without it the prior hop is zeros, pacfile.py:265-268)
 *   PAC_STREAM_NO_FLUSH   no Close() flush block (pacfile.py:355-366): more
 *                         hops follow in a later call
 * A stream with n frames and flags f yields ceil((n - prior) / 1024) blocks
 * plus the flush block unless NO_FLUSH. */
#define PAC_STREAM_HAS_PRIOR 1
#define PAC_STREAM_NO_FLUSH 2
typedef struct {
    int64_t extra_bits;
    int64_t bit_deposit;
    int32_t flags;
    int32_t reserved;
} pac_stream_state;

/* Per-kernel device time of the last encode call (HIP events recorded on the
 * context's stream around each launch, read after the call), ms.
 *   origin: front = k_origin_front, alloc = k_origin_alloc, scan = k_scan_*,
 *           pack = k_origin_pack, thr = 0
 *   master: lrms = k_master_lrms, spec = k_master_spec, thr = k_master_thr, front = k_master_front,
 *           alloc = k_master_tail (second stream, overlapping the next chunk),
 *           scan = k_scan_*, pack = k_master_pack (each summed over the chunks) */
typedef struct {
    float front_ms;
    float alloc_ms;
    float scan_ms;
    float pack_ms;
    float total_ms;     /* origin: first to last event; master: lrms+spec+thr(+thr_short)+front+scan+pack */
    int64_t n_channel_blocks;
    int64_t out_bytes;
    float thr_ms;
    float lrms_ms;
    float thr_short_ms; /* block switching: k_master_thr_short (the short frames' thresholds) */
    float spec_ms;      /* master: k_master_spec (the windowed L/R spectra the thresholds derive from), or the
                           default fused k_master_lrms_spec (LRMS + spectra; lrms_ms is then 0) */
    float emit_ms;      /* master: k_master_emit (the bitstream packing beside the next chunk's tail; pack_ms
                           is then k_master_place, the copy to the file offsets) */
    int32_t chunks;     /* master: pass-1 chunks of the call = launches of each pass-1 kernel (run_master) */
    int32_t repacked;   /* master: 1 if the tail's staging overflowed and the call re-ran through k_master_pack
                           (~2x the encode time; pac_abi.hip pac_encode_streams) */
} pac_timing;

/* The codec.Encode() result of one block (codec.py:129 / Origin codec.py:67). */
typedef struct {
    int32_t n_channels;
    int32_t overall[8];          /* overallScaleFactor[iCh]                     */
    int32_t ba[8][25];           /* bitAlloc[iCh][iBand]                        */
    int32_t sf[8][25];           /* scaleFactor[iCh][iBand]                     */
    int32_t mant[8][1024];       /* signed mantissa code by MDCT line (0 if ba=0) */
    int32_t table_id[8];         /* tableID[iCh] (master)                       */
    int32_t lrms[25];            /* LRMS[iBand] (master)                        */
    int32_t nbytes[8];           /* payload bytes of the channel-block          */
    double smr[8][25];           /* SMR fed to BitAlloc                         */
    /* master: huffmanCodedMantissa[iCh] (codec.py:111-129, Huffman.py:274-309)
     * by MDCT line: the code's bits (an escape is the escape code followed by
     * the ba raw bits of the unsigned mantissa, Huffman.py:296-299) right-aligned,
     * and its length in bits (0 for lines of ba = 0 bands)                   */
    uint64_t huff_code[8][1024];
    int32_t huff_len[8][1024];
} pac_block_fields;

/* --- context ------------------------------------------------------------ */
int pac_ctx_create(int device, pac_ctx **out);
void pac_ctx_destroy(pac_ctx *ctx);
const char *pac_last_error(void);
int pac_version(void);

/* Huffman() constructor (Huffman.py:256-262): the 10 static tables, as the
 * neutral image data/huffman_tables.bin ("PACHUF01"). Required for MASTER. */
int pac_huffman_load(pac_ctx *ctx, const uint8_t *image, int64_t len);

/* ScaleFactorBands(AssignMDCTLinesFromFreqLimits(1024, fs)) (psychoac.py:124-156,
 * 193-213): the 25 band line counts written to the file header. */
int pac_band_layout(int32_t sample_rate, int32_t n_lines_out[25]);

/* --- encode ---------------------------------------------------------------
 * Whole streams: the PACFile.WriteDataBlock loop over every hop plus the
 * Close() flush block (pacfile.py:273-366), for n_streams independent
 * streams that share one pac_params.  pcm holds the streams' interleaved
 * int16 frames back to back; frame_offsets (host, n_streams+1) delimits them.
 * Writes each stream's data section ('<L nBytes' + payload per channel-block,
 * the bytes after the file header) back to back into out and its extent into
 * stream_byte_offsets (host, n_streams+1).  *_is_device: the pointer is
 * device memory (no PCIe copy).  states (host, n_streams, nullable): the
 * framing flags in, the MASTER reservoir in/out (pac_stream_state). */
int pac_encode_streams(pac_ctx *ctx, const pac_params *p, int32_t n_streams,
                       const int16_t *pcm, const int64_t *frame_offsets, int32_t pcm_is_device,
                       uint8_t *out, int64_t out_capacity, int32_t out_is_device,
                       int64_t *stream_byte_offsets, pac_stream_state *states);

/* Upper bound of the data-section bytes pac_encode_streams can produce. */
int64_t pac_encode_bound(const pac_params *p, int32_t n_streams, const int64_t *frame_offsets);

/* One block: codec.Encode(data, codingParams[, huffman]) + the channel-block
 * bytes PACFile.WriteDataBlock writes (pacfile.py:285-351).  full_block (host)
 * holds n_channels x 2048 float64 signed fractions (priorBlock ++ data). */
int pac_encode_block(pac_ctx *ctx, const pac_params *p, const double *full_block,
                     pac_stream_state *state, uint8_t *out, int64_t out_capacity,
                     int64_t *out_bytes, pac_block_fields *fields);

/* Decode n independent .pac/.wak data sections (the bytes after each file's
 * header, back to back, delimited by stream_byte_offsets[n+1] -- what
 * pac_encode_streams writes) into 16-bit PCM, exactly as the reference's
 * decode driver writes the output WAV's frames (pacfile.py:478-499):
 * PACFile.ReadDataBlock (pacfile.py:153-229) + codec.Decode (codec.py:25-65)
 * per block, the first ReadDataBlock result skipped, the final overlap half
 * written, PCMFile.WriteDataBlock's conversion (pcmfile.py:118-147).  With
 * preroll != 0 every ReadDataBlock result is kept (the PACFile plugin
 * surface).  frame_offsets[n+1] (out) are filled first; if pcm_out is NULL
 * or pcm_capacity_frames is too small the call returns PAC_E_CAPACITY after
 * filling them.  float_out (optional, host): the same samples as float64
 * before the int16 conversion.  pcm_out interleaved [frames][n_channels]. */
int pac_decode_streams(pac_ctx *ctx, const pac_params *p, int32_t n_streams, const uint8_t *data,
                       const int64_t *stream_byte_offsets, int32_t data_is_device, int32_t preroll,
                       int16_t *pcm_out, int64_t pcm_capacity_frames, int32_t pcm_is_device,
                       double *float_out, int64_t *frame_offsets);

/* The frame_offsets[n+1] pac_decode_streams produces for data sections in
 * HOST memory, computed on the host (walks the '<L nBytes' prefixes; no device
 * work).  PAC_E_ARG for a malformed section, like pac_decode_streams. */
int pac_decode_layout(const pac_params *p, int32_t n_streams, const uint8_t *data,
                      const int64_t *stream_byte_offsets, int32_t preroll, int64_t *frame_offsets);

/* --- WAV ingest / egress on the device ------------------------------------
 * PCMFile.ReadFileHeader (pcmfile.py:32-65): the 4-byte-step scan for 'fmt '
 * and 'data' as the reference does it.  status 0, or the reference's raise:
 * -1 not RIFF, -2 no 'fmt ', -3 not PCM, -4 not 16-bit, -5 no 'data'.
 * frames = the frames the encode driver reads: num_samples, plus one hop when
 * num_samples is an exact multiple of 1024 and bytes follow the data
 * (PACFile.WriteFileHeader bumps the shared numSamples, pacfile.py:240-242;
 * the hop holds extra_bytes of the file, zero-padded, pcmfile.py:77-79). */
typedef struct {
    int32_t sample_rate, n_channels, bits_per_sample, status;
    int64_t num_samples;    /* header frames (numSamples)                  */
    int64_t data_offset;    /* byte offset of the first sample in the file */
    int64_t frames;         /* frames the encoder reads                    */
    int64_t extra_bytes;
} pac_wav_info;

/* Scan n WAV files held back to back in blob (file_offsets[n+1], host). */
int pac_wav_scan(pac_ctx *ctx, int32_t n_files, const uint8_t *blob, const int64_t *file_offsets,
                 int32_t blob_is_device, pac_wav_info *info);

/* The encode driver (pacfile.py:430-499) for n WAV files held back to back in
 * blob: header scan, frame gather (+ the quirk hop) into the encoder's PCM
 * and pac_encode_streams, all on the device.  Every file must match p's
 * sample rate and channel count.  info_out (host, nullable) gets the scan. */
int pac_encode_wav(pac_ctx *ctx, const pac_params *p, int32_t n_files, const uint8_t *blob,
                   const int64_t *file_offsets, int32_t blob_is_device, uint8_t *out, int64_t out_capacity,
                   int32_t out_is_device, int64_t *stream_byte_offsets, pac_stream_state *states,
                   pac_wav_info *info_out);

/* The decode driver's output WAV files (pacfile.py:478-499): pac_decode_streams
 * + PCMFile.WriteFileHeader from each coded file's numSamples (num_samples,
 * host, n) + the frames, back to back into out (wav_offsets[n+1], host). */
int pac_decode_wav(pac_ctx *ctx, const pac_params *p, int32_t n_streams, const uint8_t *data,
                   const int64_t *stream_byte_offsets, int32_t data_is_device, const int64_t *num_samples,
                   uint8_t *out, int64_t out_capacity, int32_t out_is_device, int64_t *wav_offsets);

/* --- device buffers, sync, timing (benchmarks; data resident in HBM) ----- */
int pac_device_alloc(pac_ctx *ctx, int64_t bytes, void **ptr);
int pac_device_free(pac_ctx *ctx, void *ptr);
int pac_copy_to_device(pac_ctx *ctx, void *dst, const void *src, int64_t bytes);
int pac_copy_to_host(pac_ctx *ctx, void *dst, const void *src, int64_t bytes);
/* Synthetic 48 kHz-style white-noise PCM: N(0,1)*0.25*32767, rint, clip. */
int pac_synth_white(pac_ctx *ctx, int16_t *dev_pcm, int64_t n_samples, uint64_t seed);
/* Synthetic stereo pink noise + 440/1250/5300 Hz tones (BASELINE configs[2]),
 * n_frames interleaved L/R frames. */
int pac_synth_pink_tones(pac_ctx *ctx, int16_t *dev_pcm, int64_t n_frames, int32_t sample_rate,
                         uint64_t seed);
/* Decaying noise bursts (one per `period` frames, hashed onset) added in place
 * to stereo PCM: the transients of the block-switching workload (configs[4]). */
int pac_synth_bursts(pac_ctx *ctx, int16_t *dev_pcm, int64_t n_frames, int64_t period, uint64_t seed);
int pac_sync(pac_ctx *ctx);
int pac_set_timing(pac_ctx *ctx, int32_t enable);
/* Stereo blocks per master-profile chunk (device scratch ~113 KB/block); default 32768,
 * 65536 with block switching (the measured optima on MI355X).  At most 131071
 * (PAC_CHUNK_MAX: the tail's 32-bit buffer offsets); larger values, and a larger
 * PAC_CHUNK_BLOCKS environment value at encode time, give PAC_E_ARG. */
int pac_set_chunk_blocks(pac_ctx *ctx, int64_t blocks);
int pac_last_timing(pac_ctx *ctx, pac_timing *out);
/* Parity probe: calcBTHR (psychoac.py:409-456) of n blocks of 2048 float64
 * samples as the reference receives them (Hann applied inside): the masking
 * threshold per MDCT line and the masker count. */
int pac_debug_threshold(pac_ctx *ctx, int32_t sample_rate, int32_t n, const double *data,
                        int32_t no_drop, double *thr, int32_t *npeaks);
/* Parity probe: SineWindow + MDCT (window.py:27-39, mdct.py:49-82) of n raw
 * 2048-sample blocks -> 1024 lines each (before the overall scale). */
int pac_debug_mdct(pac_ctx *ctx, int32_t n, const double *data, double *X);
/* Parity probe of the master path's MDCT: the same lines derived from the raw
 * blocks' DFT as k_master_lrms_spec derives them from the LRMS spectra
 * (mdct_from_dft; blocks taken in pairs as the L and R of one stereo block). */
int pac_debug_mdct_dft(pac_ctx *ctx, int32_t n, const double *data, double *X);

#ifdef __cplusplus
}
#endif
#endif
