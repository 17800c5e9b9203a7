// pac_decode.hip -- gfx950 kernels of the PAC/WAK decoder:
// PACFile.ReadDataBlock (codec/pacfile.py:153-229, Origin pacfile.py
// ReadDataBlock), Huffman.decodeData (Huffman.py:321-344), codec.Decode
// (codec.py:25-65, Origin codec.py Decode) with vDequantize
// (quantize.py:345-376), IMDCT (mdct.py:72-79), SineWindow, the overlap-add
// and the decode driver's block order (pacfile.py:478-499), and
// PCMFile.WriteDataBlock's sample conversion (pcmfile.py:118-147).
//
//   k_dec_count / k_dec_index  one thread per stream: walk the '<L nBytes'
//                              prefixes -> channel-block offsets
//   k_dec_parse                one LANE per channel-block: the serial bit
//                              parse (band headers, raw mantissas or sign bits
//                              + two-level table Huffman decode, LRMS) from a
//                              64-bit buffer refilled by aligned 32-bit loads
//   k_dec_synth                256 threads per (stream, run of DEC_SEG blocks
//                              [, channel]): dequantize, M/S with the
//                              reference's channel aliasing, IMDCT (DCT-IV via
//                              the 512-point Stockham FFT), sine window,
//                              overlap-add, int16 conversion
#include "pac_wave.h"
#include "pac_kernels.h"
#include "pac_bs.h"

// Two-level Huffman decoding tables (built on the host in pac_huffman_load):
// level 1 indexed by the first l1 bits of the next maxlen bits; an entry is
// (len << 16) | symbol, symbol 0xFFFF = the escape code, or 0x80000000 | the
// offset of a level-2 table indexed by the remaining maxlen - l1 bits.
// Plus the short-code table at sbase: PAC_NTAB x 2^PAC_DEC_SBITS entries
// indexed by the next PAC_DEC_SBITS bits, (len << 16) | symbol for codes of at
// most that length, 0x80000000 for the longer ones (then the two-level
// lookup).  k_dec_parse holds it in LDS: 93-99 % of the symbols (the tables'
// own code-length mass) decode without a global gather.
#define PAC_DEC_SBITS 9
struct PacHuffDec {
    int32_t base[PAC_NTAB];
    int32_t maxlen[PAC_NTAB];
    int32_t l1[PAC_NTAB];
    int32_t sbase;
};

#define DEC_SEG 128     // blocks per synthesis workgroup (+1 preroll block each: 16 -> 64 measured +2 %, 64 -> 128 +0.9 %, 256 as 128)

__global__ void k_dec_count(const uint8_t* __restrict__ data, const int64_t* __restrict__ so, int n,
                            int64_t* __restrict__ cnt) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    int64_t pos = so[s], c = 0;
    const int64_t end = so[s + 1];
    while (pos + 4 <= end) {
        const uint8_t* p = data + pos;
        const uint32_t nb = p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24);
        pos += 4 + (int64_t)nb;
        c++;
    }
    cnt[s] = pos == end ? c : -1;     // -1: the last channel-block runs past the stream
}

__global__ void k_dec_index(const uint8_t* __restrict__ data, const int64_t* __restrict__ so, int n,
                            const int64_t* __restrict__ cb_base, int64_t* __restrict__ cb_off) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    int64_t pos = so[s], g = cb_base[s];
    const int64_t end = so[s + 1];
    while (pos + 4 <= end) {
        const uint8_t* p = data + pos;
        const uint32_t nb = p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24);
        cb_off[g++] = pos;
        pos += 4 + (int64_t)nb;
    }
}

// MSB-first bit reader over one channel-block's bytes: aligned 32-bit loads
// into a 64-bit buffer (one load per 32 bits consumed).  Loads stop at the
// word holding the channel-block's last byte (wend): past it the reader sees
// zero bits, so a truncated or corrupt nBytes can never make it read outside
// the data; the caller compares the bits consumed with 8 nBytes afterwards
// (the reference's PackedBits raises on such input).
//
// The words are loaded two refills AHEAD (pre, pre2): a refill takes the word
// loaded two refills before and issues the load of the next, so its latency
// overlaps the next 64 bits of decoding instead of stalling the parse.
struct DecBits {
    const uint32_t* w;     // aligned word stream: the next word to load (pre, pre2 hold the two before it)
    const uint32_t* wend;  // first word past the channel-block
    uint64_t buf;          // next bits, MSB first
    int nbuf;
    uint32_t pre, pre2;    // the next two words, loaded ahead
    __device__ __forceinline__ static uint32_t be(uint32_t x) { return __builtin_bswap32(x); }
    __device__ __forceinline__ uint32_t next_word() {
        const uint32_t v = pre;
        pre = pre2;
        pre2 = w < wend ? *w : 0u;
        ++w;
        return be(v);
    }
    __device__ __forceinline__ void init(const uint8_t* p, int64_t bit0, const uint8_t* end) {
        // pointer arithmetic from p and end only (no integer round trip): the
        // compiler then keeps them global pointers and reads through
        // global_load, not flat loads (whose waits also drain the LDS lookups)
        wend = reinterpret_cast<const uint32_t*>(end + ((4 - ((uintptr_t)end & 3)) & 3));
        const uint8_t* q = p + (bit0 >> 3);
        const uintptr_t a = (uintptr_t)q;
        w = reinterpret_cast<const uint32_t*>(q - (a & 3));
        pre = w < wend ? *w : 0u;
        pre2 = w + 1 < wend ? w[1] : 0u;
        w += 2;
        const int skip = (int)((a & 3) * 8 + (bit0 & 7));
        buf = (uint64_t)next_word() << 32;
        nbuf = 32;
        refill();
        buf <<= skip;
        nbuf -= skip;
        refill();
    }
    __device__ __forceinline__ void refill() {
        if (nbuf <= 32) {
            buf |= (uint64_t)next_word() << (32 - nbuf);
            nbuf += 32;
        }
    }
    __device__ __forceinline__ uint32_t peek32() const { return (uint32_t)(buf >> 32); }
    __device__ __forceinline__ void skip(int nb) {
        buf <<= nb;
        nbuf -= nb;
        refill();
    }
    __device__ __forceinline__ void advance(int n) {      // any n >= 0
        while (n > 32) { skip(32); n -= 32; }
        skip(n);
    }
    __device__ __forceinline__ uint32_t read(int nb) {     // nb <= 32
        if (nb <= 0) return 0;
        const uint32_t v = (uint32_t)(buf >> (64 - nb));
        skip(nb);
        return v;
    }
};

// bits consumed so far by reader r started at payload p, bit 0
__device__ __forceinline__ int64_t bits_consumed(const DecBits& r, const uint8_t* p) {
    const uintptr_t a0 = (uintptr_t)p & ~(uintptr_t)3;
    const int64_t loaded = ((int64_t)((uintptr_t)(r.w - 2) - a0)) * 8;     // bits taken into buf from a0 (pre, pre2 excluded)
    return loaded - r.nbuf - (int64_t)(((uintptr_t)p & 3) * 8);
}

__device__ __forceinline__ uint32_t dec_huff(DecBits& r, const uint32_t* __restrict__ tab, const PacHuffDec& hd,
                                             const uint32_t* stab, int id, int ba) {
    const uint32_t top = r.peek32();
    uint32_t e = stab[(id << PAC_DEC_SBITS) + (top >> (32 - PAC_DEC_SBITS))];
    if (e >> 31) {                           // a longer code: the two-level tables
        const int ml = hd.maxlen[id], l1 = hd.l1[id];
        const uint32_t idx = top >> (32 - ml);
        e = tab[hd.base[id] + (idx >> (ml - l1))];
        if (e >> 31) e = tab[(e & 0x7fffffffu) + (idx & ((1u << (ml - l1)) - 1u))];
    }
    int len = (e >> 16) & 31;
    uint32_t sym = e & 0xffffu;
    if (!len) { len = 1; sym = 0; }         // not a code of the table: malformed input
    r.skip(len);
    return sym == 0xffffu ? r.read(ba) : sym;   // escape: the raw ba-bit symbol follows
}

// Per-channel-block fields: codes (signed mantissa codes as the reference's
// ReadDataBlock builds them, layout dec_code_at), basf [G][DEC_NBP] (ba | sf <<
// 8), overall [G], lrms [G][DEC_NBP] (master) -- rows of 28 entries, so that
// the parse writes a channel-block's 25 bands as 32-bit words (14 for basf,
// 7 for lrms) instead of one store per band and field.
//
// The codes are tiled: tile (g / 64, l / 8) holds lines l .. l+7 of the 64
// channel-blocks g of one parse wave as 64 runs of 8 codes (1 KB).  The parse
// stages each lane's codes of the current 8-line group in LDS and writes the
// group as one 16-byte store per lane -- 1 KB contiguous per wave, every
// cache line whole at once.  (The plain [G][1024] layout, one 2-byte store per
// line, left every lane its own partly written line open for 64 lines, more
// open lines than the L2 holds: the parse wrote 41.4 KB to HBM per block for
// 4 KB of codes.)  The synthesis reads 16 contiguous bytes per 8 threads.
#define DEC_GRP 8
#define DEC_NBP 28      // bytes per channel-block row of ba / sf / lrms (25 bands, word-padded)
__device__ __forceinline__ int64_t dec_code_at(int64_t g, int l) {
    return (((g >> 6) * (PAC_HALFN / DEC_GRP) + (l / DEC_GRP)) * (WAVE * DEC_GRP)) + ((g & 63) * DEC_GRP) +
           (l % DEC_GRP);
}
struct PacDecWork {
    uint16_t* codes;
    uint16_t* basf;     // [G][DEC_NBP] ba | sf << 8 (one load per line in the synthesis)
    uint8_t* overall;
    uint8_t* lrms;
    int* err;           // set to 1 when a channel-block's fields run past its nBytes
    uint8_t* bsf;       // [G] block switching (pac_bs.h): the short-frame bit, or null: off
};

#define DEC_PARSE_NT 512
__global__ __launch_bounds__(DEC_PARSE_NT) void k_dec_parse(const uint8_t* __restrict__ data,
                                                            const int64_t* __restrict__ cb_off, int64_t G, int master,
                                                            const PacTables* __restrict__ T,
                                                            const uint32_t* __restrict__ htab, PacHuffDec hd,
                                                            PacDecWork D) {
    __shared__ uint32_t stab[PAC_NTAB << PAC_DEC_SBITS];   // 20 KB
    // each lane's codes of the current DEC_GRP-line group (8 KB: 28 KB per
    // workgroup of 8 waves, 4 workgroups = 8 waves per SIMD)
    __shared__ __attribute__((aligned(16))) uint16_t stage[DEC_PARSE_NT][DEC_GRP];
    if (master) {
        for (int i = threadIdx.x; i < (PAC_NTAB << PAC_DEC_SBITS); i += blockDim.x) stab[i] = htab[hd.sbase + i];
        __syncthreads();
    }
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // lanes past G stay in the (wave-uniform) line loops with an empty reader
    // (zero bits: every band unallocated) and store nothing but their staged
    // codes, into the tile padding (the buffer holds whole waves)
    const bool valid = g < G;
    const uint8_t* p = data + (valid ? cb_off[g] : 0);
    const uint32_t nbytes = valid ? (p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24)) : 0u;
    const uint8_t* end = valid ? p + 4 + nbytes : p;
    DecBits r;
    r.init(p + 4, 0, end);
    const uint32_t ov = r.read(4);
    if (valid) D.overall[g] = (uint8_t)ov;
    const int id = master ? (int)r.read(4) - 1 : 0;
    const int tid = id < 0 ? 0 : (id >= PAC_NTAB ? PAC_NTAB - 1 : id);
    uint16_t* st = stage[threadIdx.x];
    int gcur = -1;                        // the staged group (wave-uniform)
    auto flush = [&]() {
        if (gcur >= 0)
            *reinterpret_cast<uint4*>(D.codes + dec_code_at(g, gcur * DEC_GRP)) = *reinterpret_cast<const uint4*>(st);
    };
    int64_t bit = master ? 8 : 4;         // bit position, for the sign-bit reader
    uint32_t bsw = 0u;                    // two bands' ba | sf << 8, stored as a word
    for (int b = 0; b < PAC_NB; ++b) {
        int a = (int)r.read(4);
        if (a) a++;
        const uint32_t sfv = r.read(4);
        bsw |= ((uint32_t)a | (sfv << 8)) << (16 * (b & 1));
        if ((b & 1) == 1 || b == PAC_NB - 1) {   // uniform
            if (valid) *reinterpret_cast<uint32_t*>(D.basf + g * DEC_NBP + (b & ~1)) = bsw;
            bsw = 0u;
        }
        bit += 8;
        if (!__ballot(a != 0)) continue;   // no lane codes the band
        const int lo = T->lower[b], nl = T->nlines[b];
        DecBits sg;                        // master: nl sign bits, then nl Huffman codes
        if (master && a) {
            sg.init(p + 4, bit, end);
            r.advance(nl);
            bit += nl;
        }
        for (int l = lo; l < lo + nl; ++l) {
            if (l / DEC_GRP != gcur) {     // a new group: write the previous one
                flush();
                gcur = l / DEC_GRP;
            }
            if (a) {
                uint32_t c;
                if (!master) {
                    c = r.read(a);
                } else {
                    const uint32_t sym = dec_huff(r, htab, hd, stab, tid, a);
                    c = sym + (sg.read(1) << (a - 1));
                }
                st[l % DEC_GRP] = (uint16_t)c;
            }
        }
        if (a) bit = master ? bits_consumed(r, p + 4) : bit + (int64_t)nl * a;
    }
    flush();
    if (master) {
        uint32_t fw = 0u;
        for (int b = 0; b < PAC_NB; ++b) {
            fw |= r.read(1) << (8 * (b & 3));
            if ((b & 3) == 3 || b == PAC_NB - 1) {
                if (valid) *reinterpret_cast<uint32_t*>(D.lrms + g * DEC_NBP + (b & ~3)) = fw;
                fw = 0u;
            }
        }
    }
    if (D.bsf) {
        const uint32_t f = r.read(1);
        if (valid) D.bsf[g] = (uint8_t)f;
    }
    if (valid && bits_consumed(r, p + 4) > 8 * (int64_t)nbytes) atomicOr(D.err, 1);
}

// vDequantize (quantize.py:345-376) + vDequantizeUniform (:118-145), 4 scale bits
// (32-bit integers: a code has ba <= 16 bits, so q < 2^30 and the largest
// code 2^(ba+15) - 1 < 2^31 -- the same integers as the reference's, one
// conversion each)
__device__ __forceinline__ double pac_dequantize(int scale, int m, int ba) {
    const int smask = 1 << (ba - 1);
    const bool neg = (m & smask) == smask;
    if (neg) m -= smask;
    int q = m << (15 - scale);
    if (scale < 15 && m > 0) q += 1 << (14 - scale);
    const double largest = (double)((1u << (ba + 15)) - 1u);
    const double a = (2.0 * (double)q) / largest;
    return neg ? -a : a;
}

// PCMFile.WriteDataBlock: sign, vQuantizeUniform(|x|, 16), re-sign
__device__ __forceinline__ int16_t pac_float_to_pcm(double x) {
    const bool s = __builtin_signbit(x);
    const double a = s ? -x : x;
    // a < 1: the value is below 2^15, so the 32-bit truncating conversion (one
    // v_cvt_u32_f64) equals the reference's integer cast
    const uint32_t code = a < 1.0 ? (uint32_t)((a * 65535.0 + 1.0) / 2.0) : 32767u;
    const int16_t c = (int16_t)code;
    return s ? (int16_t)-c : c;
}

// IMDCT (mdct.py:72-79) of the lines in L, sine-windowed: w(n) for n < 2048
// from U = 2 DCT-IV(L) (in buf):  n < 512: U[n+512];  512 <= n < 1536:
// -U[1535-n];  n >= 1536: -U[n-1536]
__device__ __forceinline__ double imdct_window_at(const double* U, const PacTables* __restrict__ T, int n,
                                                  int fl) {
    const double y = n < 512 ? U[n + 512] : (n < 1536 ? -U[1535 - n] : -U[n - 1536]);
    return y * (fl ? bs_long_win(T, fl, n) : T->sine[n]);
}

// Block switching: wave k turns short block k's lines (Lc[4 j + k]) into
// U_k = 2 DCT-IV in place; out of line so that the long path keeps its
// register budget
__device__ __forceinline__ void dec_short_imdct(double* Lc, const PacTables* __restrict__ T, double2* buf, int tid) {
    const int k = tid / WAVE;
    wave_dct4_256<false>([&](int j) { return Lc[4 * j + k]; }, T, buf + 256 * k, tid & (WAVE - 1), 2.0,
                  [&](int j, double v) { Lc[4 * j + k] = v; });
}

// Block switching (pac_bs.h): sample p < 2048 of a short frame's synthesis,
// 0 + the windowed IMDCTs (N = 512) of the short blocks covering p in block
// order; Uc[4 j + k] = U_k[j] = 2 DCT-IV of block k's lines.
__device__ __forceinline__ double short_synth_at(const double* Uc, const PacTables* __restrict__ T, int p) {
    double y = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int n = p - 384 - 256 * k;
        if (n < 0 || n >= PAC_NS) continue;
        const int j = n < 128 ? n + 128 : (n < 384 ? 383 - n : n - 384);
        const double u = n < 128 ? Uc[4 * j + k] : -Uc[4 * j + k];
        y = y + u * T->sine_s[n];
    }
    return y;
}

// one synthesis workgroup: blocks [b0, b1) of stream s, channels c0 .. c0+nc-1
// (nc = 1 origin, 2 master), output frames of ReadDataBlock results
// ob = b - 1 (b >= 1; result 0 is the one the driver skips) or, with preroll,
// ob = b; plus the final overlap half when b1 is the stream's last block.
struct PacDecOut {
    int16_t* pcm;          // interleaved [frames][nch]
    double* fpcm;          // optional float64 samples, same layout
    const int64_t* fo;     // [n_streams] first output frame of each stream
    int preroll;
};

// The synthesis holds each block's dequantized lines in registers, in the
// order the DCT-IV's pre-twiddle reads them (lines 2q and 1023 - 2q of
// q = tid, tid + 256: grp_dct4_regs), so the M/S reconstruction is
// thread-local and the plain frames need no LDS copy of the lines.  A stereo
// pair's two samples of a frame go out as one 32-bit store.  Barriers hand off
// LDS only (lds_sync): the code loads and PCM stores stay in flight across
// them.  At most 128 VGPRs: 4 waves per SIMD.  BS (block switching on): 40 KB
// of LDS (FFT scratch, overlap halves, the short frames' lines); without it
// the short and start / stop frames' code is gone (32 KB).  Measured: with
// the field loads of a block sunk by the compiler into "ba != 0" branches
// (one serial round trip per line), 5 waves per SIMD gave 55.7 M blocks/s;
// with them forced into one round trip (below) 4 waves give 63.4 M, and 5
// waves spill (49.8 M).
template <bool BS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_dec_synth(
    const PacTables* __restrict__ T, PacDecWork D, const int64_t* __restrict__ cb_base,
    const int64_t* __restrict__ nblk, const int64_t* __restrict__ seg_base, int n_streams, int nch, int master,
    PacDecOut O) {
    __shared__ double2 buf[1024];                 // IMDCT scratch
    __shared__ double prev[2][PAC_HALFN];         // overlap halves (thread-private slots)
    __shared__ double sl[BS ? PAC_HALFN : 1];     // a short frame's lines (block switching)
    const int tid = threadIdx.x;
    const bool pair = master && nch == 2;          // M/S stereo pair (mono master: per channel)
    const int nc = pair ? 2 : 1;
    const int64_t item = blockIdx.x / (pair ? 1 : nch);
    const int c0 = pair ? 0 : (int)(blockIdx.x % nch);
    // stream of this segment: last s with seg_base[s] <= item
    int lo = 0, hi = n_streams;
    while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (seg_base[mid] <= item) lo = mid; else hi = mid; }
    const int s = lo;
    const int64_t nb = nblk[s];
    const int64_t b0 = (item - seg_base[s]) * DEC_SEG;
    const int64_t b1 = b0 + DEC_SEG < nb ? b0 + DEC_SEG : nb;
    // the thread's four lines (pre-twiddle order), their bands and whether a band covers them
    const int lend = T->lower[PAC_NB - 1] + T->nlines[PAC_NB - 1];
    auto ln = [&](int i) { const int q = (i >> 1) * 256 + tid; return (i & 1) ? 1023 - 2 * q : 2 * q; };
    int bnd0[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bnd0[i] = ln(i) < lend ? T->band_of_line[ln(i)] : -1;
    for (int c = 0; c < nc; ++c)
        for (int i = tid; i < PAC_HALFN; i += 256) prev[c][i] = 0.0;
    const int64_t base = cb_base[s];
    const int64_t fos = O.fo[s];                  // once: the stores below may alias it for the compiler
    const PacTables* const T0 = T;
    const int tid0 = tid;
    for (int64_t b = b0 > 0 ? b0 - 1 : 0; b < b1; ++b) {
        // the tables' base and the thread index, opaque in each block: the
        // compiler recomputes their per-lane addresses in the block instead of
        // holding them live across the loop (163 -> 123 VGPRs, no spills: 4
        // waves per SIMD instead of 3; decode 48.4 -> 51.3 M blocks/s.  At 3
        // waves the recomputation alone is a loss: 45.4)
        // (the pointer is offset by an opaque zero, not itself passed through
        // the asm: it stays a global pointer -- global_load, not flat_load,
        // whose waits also drain the LDS operations)
        int zero = 0, tid = tid0;
        asm volatile("" : "+s"(zero), "+v"(tid));
        const PacTables* __restrict__ T = T0 + zero;
        int bnd[4];                                // the bands too (no per-line field pointers kept)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            bnd[i] = bnd0[i];
            asm volatile("" : "+v"(bnd[i]));
        }
        auto ln = [&](int i) { const int q = (i >> 1) * 256 + tid; return (i & 1) ? 1023 - 2 * q : 2 * q; };
        // vDequantize of the four lines of each channel, / 2^overall (codec.py:25-45)
        // every field loaded unconditionally (a line past the last band reads
        // band 0's and discards it): the loads of a block are one round trip,
        // not ba's and then, under "ba != 0", the scale factor's and code's
        double x[2][4];
        int fba[2][4], fcd[2][4], fov[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (c >= nc) break;
            const int64_t g = base + b * nch + c0 + c;
            fov[c] = D.overall[g];
            // uniform bases (scalar registers) + 32-bit lane offsets: no 64-bit
            // address per load
            const uint16_t* bsg = D.basf + g * DEC_NBP;
            const uint16_t* cdg = D.codes + dec_code_at(g, 0);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const unsigned bi = bnd[i] >= 0 ? (unsigned)bnd[i] : 0u;
                const int l = ln(i);
                fba[c][i] = bsg[bi];                                // ba | sf << 8
                fcd[c][i] = cdg[(unsigned)((l / DEC_GRP) * (WAVE * DEC_GRP) + l % DEC_GRP)];
            }
        }
        // every field in registers before any is used: the compiler would
        // otherwise sink the scale-factor and code loads under "ba != 0" --
        // a second round trip per line (in the ISA of the 5-wave build)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (c >= nc) break;
            asm volatile("" ::"v"(fov[c]));
#pragma unroll
            for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(fba[c][i]), "v"(fcd[c][i]));
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (c >= nc) break;
            // / 2^overall as * 2^-overall: a power of two, the same double
            // (the lines are far from the subnormal range), one multiply
            // instead of a division sequence per line
            const double unscale = __builtin_ldexp(1.0, -fov[c]);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int ba = bnd[i] >= 0 ? (fba[c][i] & 255) : 0;
                const double v = ba ? pac_dequantize(fba[c][i] >> 8, fcd[c][i], ba) : 0.0;
                x[c][i] = v * unscale;
            }
        }
        if (pair) {
            // codec.py:46-54: mdctLineL/R alias mdctLine[0]/[1]; the second
            // assignment reads the updated channel 0: L = M - S, R = (M - S) + S
            const uint8_t* lr = D.lrms + (base + b * nch + 1) * DEC_NBP;   // last channel's bits
            int lf[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) lf[i] = lr[bnd[i] >= 0 ? bnd[i] : 0];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (bnd[i] >= 0 && lf[i]) {
                    const double a = x[0][i] - x[1][i];
                    x[0][i] = a;
                    x[1][i] = a + x[1][i];
                }
            }
        }
        // block switching: this frame short, or a long frame's start / stop shape
        int fl = 0;
        if (BS && D.bsf) {
            const int64_t g0 = base + b * nch;
            fl = (D.bsf[g0] ? PAC_BS_SHORT : 0) | (b > 0 && D.bsf[g0 - nch] ? PAC_BS_PREV : 0) |
                 (b + 1 < nb && D.bsf[g0 + nch] ? PAC_BS_NEXT : 0);
        }
        const bool out = b >= b0 && b >= 1 - (O.preroll ? 1 : 0);
        const int64_t ob = b - 1 + (O.preroll ? 1 : 0);
        uint32_t h0[4] = {0u, 0u, 0u, 0u};         // a pair's channel-0 samples until channel 1's
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (c >= nc) break;
            lds_sync();                            // buf / sl free: the previous transform's reads are done
            const double* U;
            if (BS && (fl & PAC_BS_SHORT)) {       // wave k: U_k = 2 DCT-IV of block k, back into its line slots
#pragma unroll
                for (int i = 0; i < 4; ++i) sl[ln(i)] = x[c][i];
                lds_sync();
                dec_short_imdct(sl, T, buf, tid);
                lds_sync();
                U = sl;
            } else {
                // plain FFT layout: the swizzle's index math would cost this kernel a wave per SIMD
                U = grp_dct4_regs<256, false>(x[c], T, buf, tid, 2.0);
            }
            auto emit16 = [&](int i, double w0, double w1) {      // one sample, 16-bit store
                const double v = prev[c][i] + w0;
                prev[c][i] = w1;
                if (!out) return;
                const int64_t o = (fos + ob * PAC_HALFN + i) * nch + c0 + c;
                O.pcm[o] = pac_float_to_pcm(v);
                if (O.fpcm) O.fpcm[o] = v;
            };
            if (BS && (fl & PAC_BS_SHORT)) {
#pragma unroll 1
                for (int i = tid; i < PAC_HALFN; i += 256)
                    emit16(i, short_synth_at(U, T, i), short_synth_at(U, T, i + PAC_HALFN));
            } else if (BS && fl) {                 // start / stop window
#pragma unroll 1
                for (int i = tid; i < PAC_HALFN; i += 256)
                    emit16(i, imdct_window_at(U, T, i, fl), imdct_window_at(U, T, i + PAC_HALFN, fl));
            } else if (!pair) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int i = k * 256 + tid;
                    emit16(i, imdct_window_at(U, T, i, 0), imdct_window_at(U, T, i + PAC_HALFN, 0));
                }
            } else {                               // a pair's plain frame: (L, R) as one 32-bit store
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int i = k * 256 + tid;
                    const double v = prev[c][i] + imdct_window_at(U, T, i, 0);
                    prev[c][i] = imdct_window_at(U, T, i + PAC_HALFN, 0);
                    if (!out) continue;
                    const int64_t o = (fos + ob * PAC_HALFN + i) * 2;
                    const uint32_t h = (uint16_t)pac_float_to_pcm(v);
                    if (O.fpcm) O.fpcm[o + c] = v;
                    if (c == 0) h0[k] = h;
                    else *reinterpret_cast<uint32_t*>(O.pcm + o) = h0[k] | (h << 16);
                }
            }
        }
    }
    if (b1 == nb && nb > 0) {        // end of file: the saved half alone
        const int64_t ob = nb - 1 + (O.preroll ? 1 : 0);
        for (int c = 0; c < nc; ++c)
            for (int i = tid; i < PAC_HALFN; i += 256) {
                const int64_t o = (fos + ob * PAC_HALFN + i) * nch + c0 + c;
                O.pcm[o] = pac_float_to_pcm(prev[c][i]);
                if (O.fpcm) O.fpcm[o] = prev[c][i];
            }
    }
}
