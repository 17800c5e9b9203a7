// pac_kernels.hip -- gfx950 kernels of the PAC encoder (origin profile).
//
// Pipeline for G channel-blocks (stream s, block b, channel c):
//   k_origin_front   one wave per channel-block: sine window, MDCT, overall
//                    scale (codec.py:237-246 / Origin codec.py:90-98), Hann
//                    spectrum, findpeaks, masker sum, per-band SMR
//                    (Origin psychoac.py:215-314), band peak |line|
//   k_origin_alloc   one LANE per channel-block: greedy BitAlloc
//                    (Origin bitalloc.py:129-202), scale factors, byte size
//   k_scan_*         exclusive scan of channel-block byte sizes -> offsets
//   k_origin_pack    one wave per channel-block: MDCT recomputed (cheaper
//                    than storing 8 KB/line set), mantissas (quantize.py:315),
//                    MSB-first bit packing into LDS (bitpack.py:36-101),
//                    '<L nBytes' + payload (Origin pacfile.py:265-306)
#include "pac_wave.h"
#include "pac_kernels.h"

// ---------------------------------------------------------------------------
// sample access
// ---------------------------------------------------------------------------

__device__ __forceinline__ int upper_bound_i64(const int64_t* __restrict__ a, int n, int64_t v) {
    int lo = 0, hi = n;     // first index with a[idx] > v
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (a[mid] <= v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

struct BlockRef {
    const int16_t* pcm;   // first frame of the stream
    const double* fsrc;   // float samples of this channel-block (per-block API) or null
    int64_t first_frame;  // frame index of sample 0 = (b-1)*1024
    int64_t n_frames;
    int nch, c;
};

__device__ __forceinline__ BlockRef locate(const PacSource& src, int64_t gb, int c) {
    BlockRef r;
    r.nch = src.n_ch;
    r.c = c;
    if (src.fsrc) {           // per-block float path: [gb][nch][2048]
        r.fsrc = src.fsrc + (gb * src.n_ch + c) * PAC_N;
        r.pcm = nullptr;
        r.first_frame = 0;
        r.n_frames = 0;
        return r;
    }
    int s = upper_bound_i64(src.blk_off, src.n_streams + 1, gb) - 1;
    int64_t b = gb - src.blk_off[s];
    int64_t f0 = src.frame_off[s];
    r.pcm = src.pcm + f0 * src.n_ch;
    r.fsrc = nullptr;
    r.first_frame = (b - 1) * PAC_HALFN + (src.lead ? src.lead[s] : 0);
    r.n_frames = src.frame_off[s + 1] - f0;
    return r;
}
// the same for a block whose stream s and index b in it are known (no search)
__device__ __forceinline__ BlockRef locate_sb(const PacSource& src, int s, int64_t b, int64_t gb, int c) {
    if (src.fsrc) return locate(src, gb, c);
    BlockRef r;
    r.nch = src.n_ch;
    r.c = c;
    const int64_t f0 = src.frame_off[s];
    r.pcm = src.pcm + f0 * src.n_ch;
    r.fsrc = nullptr;
    r.first_frame = (b - 1) * PAC_HALFN + (src.lead ? src.lead[s] : 0);
    r.n_frames = src.frame_off[s + 1] - f0;
    return r;
}

// stereo frame i (0..2047) of a block as the two channels' sample codes, one
// 32-bit load (r: the channel-0 BlockPcm of an interleaved stereo source);
// zero outside the stream
struct BlockPcm;
__device__ __forceinline__ double2 stereo_frame(const BlockPcm& r, int i);

// raw signed-fraction sample i (0..2047) of the block: prior hop ++ current
// hop (pacfile.py:279-282), zero outside the stream (pcmfile.py:77-79, the
// zero first prior block pacfile.py:265-268 and the Close() flush block)
__device__ __forceinline__ double sample(const BlockRef& r, int i) {
    if (r.fsrc) return r.fsrc[i];
    int64_t f = r.first_frame + i;
    if (f < 0 || f >= r.n_frames) return 0.0;
    return pac_pcm_to_float(r.pcm[f * r.nch + r.c]);
}

// The same samples with the stream-edge test hoisted: samples [ilo, ihi) of
// the block lie inside the stream; p points at sample ilo of channel c.  The
// int16 samples load through a raw buffer resource over exactly those frames
// (from p): a sample outside them is out of the range and reads 0 -- no
// per-sample branch (under one, each sample's load was waited on before the
// next was issued: a serial round trip per sample).
struct BlockPcm {
    const int16_t* p;
    const double* f;
    int ilo, ihi, nch;
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ explicit BlockPcm(const BlockRef& r) {
        f = r.fsrc;
        nch = r.nch;
        if (f) { p = nullptr; ilo = 0; ihi = PAC_N; rs = __builtin_amdgcn_make_buffer_rsrc(nullptr, 0, 0, 0x00020000); return; }
        const int64_t ff = r.first_frame;
        ilo = ff < 0 ? (int)(-ff) : 0;
        const int64_t top = r.n_frames - ff;
        ihi = top < ilo ? ilo : (top > PAC_N ? PAC_N : (int)top);
        p = r.pcm + ((ff + ilo) * r.nch + r.c);
        rs = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 2 * (ihi - ilo) * nch, 0x00020000);
    }
    // sample i of channel c + u (u: stereo_sample's other channel), 0 outside the stream
    __device__ __forceinline__ int code(int i, int u = 0) const {
        return (int)(short)__builtin_amdgcn_raw_buffer_load_b16(rs, 2 * ((i - ilo) * nch + u), 0, 0);
    }
    __device__ __forceinline__ double operator()(int i) const {
        if (f) return f[i];
        return pac_pcm_to_float(code(i));
    }
    // the same through a plain pointer and a bounds test: for a BlockPcm that
    // differs between the lanes of a wave (k_bs_attack), whose buffer resource
    // could not live in scalar registers (a waterfall loop per load)
    __device__ __forceinline__ double at(int i) const {
        if (f) return f[i];
        int c = 0;
        if (i >= ilo && i < ihi) c = p[(i - ilo) * nch];
        return pac_pcm_to_float(c);
    }
};
__device__ __forceinline__ double2 stereo_frame(const BlockPcm& r, int i) {
    uint32_t w = 0u;
    if (i >= r.ilo && i < r.ihi) w = *reinterpret_cast<const uint32_t*>(r.p + 2 * (i - r.ilo));
    return make_double2(pac_pcm_to_float((int)(int16_t)(w & 0xffffu)), pac_pcm_to_float((int)(int16_t)(w >> 16)));
}

// The block's stereo frames (int16 source) through a raw buffer resource
// whose range is the stream's frames from the block's first in-stream frame
// on: a frame past the stream's end, or before its start (the zero first
// prior block), is out of the range and reads 0 -- no per-frame bounds test,
// one 32-bit load per frame, and a block's offsets stay within 8 KB of the
// base (the range check covers the VGPR and immediate offsets used here).
struct StereoFrames {
    __amdgpu_buffer_rsrc_t rs;
    int off0;     // byte offset of frame 0 of the block (negative before the stream start)
    __device__ __forceinline__ explicit StereoFrames(const BlockRef& r) {
        const int64_t lo = r.first_frame > 0 ? r.first_frame : 0;
        const int64_t n = r.n_frames - lo;
        const int64_t bytes = n <= 0 ? 0 : (n >= (1ll << 29) ? (1ll << 31) : 4 * n);
        rs = __builtin_amdgcn_make_buffer_rsrc((void*)(r.pcm + 2 * lo), 0, (int)bytes, 0x00020000);
        off0 = (int)(4 * (r.first_frame - lo));
    }
    __device__ __forceinline__ double2 operator()(int i) const {
        const unsigned w = __builtin_amdgcn_raw_buffer_load_b32(rs, off0 + 4 * i, 0, 0);
        return make_double2(pac_pcm_to_float((int)(short)(w & 0xffffu)), pac_pcm_to_float((int)w >> 16));
    }
};

// sample i of channel u (0, 1) of a stereo block (r: the channel-0 BlockPcm of
// an interleaved stereo source): one 16-bit load; zero outside the stream
__device__ __forceinline__ double stereo_sample(const BlockPcm& r, int i, int u) {
    return pac_pcm_to_float(r.code(i, u));
}

// xs[i] = x(i) * sine[i] (window.py:27-39, codec.py:240) into LDS, i < 2048
template <int NT>
__device__ __forceinline__ void grp_stage_sine(const BlockRef& r, const PacTables* __restrict__ T,
                                               double* xs, int tid) {
    const BlockPcm x(r);
#pragma unroll
    for (int i0 = 0; i0 < PAC_N; i0 += NT) {
        const int i = i0 + tid;
        xs[i] = __dmul_rn(x(i), T->sine[i]);
    }
}

// ---------------------------------------------------------------------------
// origin front: MDCT, overall scale, threshold, SMR
// ---------------------------------------------------------------------------

#define FRONT_NT 256

// Work item of workgroup `bid` out of n such that each of the 8 XCDs (the
// dispatcher deals workgroups round-robin, bid % 8) sweeps one contiguous
// range of items: neighbouring channel-blocks -- the two channels of a block
// and the next block, which re-reads this block's second hop -- then share
// that XCD's L2 instead of fetching the same PCM lines into several.
__device__ __forceinline__ int64_t xcd_item(int64_t bid, int64_t n) {
    const int64_t x = bid & 7, i = bid >> 3, q = n >> 3, r = n & 7;
    return x * q + (x < r ? x : r) + i;
}

__device__ __forceinline__ double block_max_256(double v, double* red) {
    v = wave_max(v);
    if ((threadIdx.x & (WAVE - 1)) == 0) red[threadIdx.x / WAVE] = v;
    __syncthreads();
    double r = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    __syncthreads();
    return r;
}

// max over the lines of each band (bands b = w, w+4, ... for wave w) of v[l];
// -inf for an empty band
__device__ __forceinline__ void grp_band_max(const PacTables* __restrict__ T, const double* v, int w,
                                             int lane, double* out, int64_t stride, double scale,
                                             bool empty_zero) {
    for (int b = w; b < PAC_NB; b += FRONT_NT / WAVE) {
        const int lo = T->lower[b], n = T->nlines[b];
        double m = -INFINITY;
        for (int l = lo + lane; l < lo + n; l += WAVE) m = fmax(m, v[l]);
        m = wave_max(m);
        if (lane == 0) out[b * stride] = (n == 0 && empty_zero) ? 0.0 : m * scale;
    }
}

// MDCT rows (64 lines) whose lines wave w of the front kernel holds
__device__ __forceinline__ int front_row(int i, int w) { return 4 * i + w; }

// unsigned keys that order like the doubles (for LDS atomic max)
__device__ __forceinline__ unsigned long long pac_order_key(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double pac_order_unkey(unsigned long long k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k));
}

// diagnostic: shader clock of wave w at mark k (first PAC_PROF_WG items only)
#define PROF_MARK(k)                                                                      \
    do {                                                                                  \
        if (src.prof && g < PAC_PROF_WG && lane == 0)                                     \
            src.prof[(g * 4 + w) * PAC_PROF_MARKS + (k)] = (long long)__builtin_amdgcn_s_memtime(); \
    } while (0)

// One 256-thread workgroup per channel-block.  The block is windowed once
// into LDS; the MDCT runs first (lines kept in registers, band peaks taken),
// then the Hann spectrum whose masker list the four waves share; the waves
// claim the 16 masking rows of 64 lines dynamically.
__global__ __launch_bounds__(FRONT_NT, 4) void k_origin_front(PacSource src, const PacTables* __restrict__ T,
                                                           PacOriginWork W, int64_t G) {
    __shared__ double2 buf[1024];          // 16 KB: MDCT scratch / spectrum / masker list / SMR
    __shared__ __attribute__((aligned(16))) double xs[PAC_N];   // 16 KB: sine-windowed block, then the loud masker list
    // the small reduction scratch lives in whichever region is idle at that point
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    const int w = tid / WAVE;
    const int64_t g = xcd_item(blockIdx.x, G);
    const BlockRef r = locate(src, g / src.n_ch, (int)(g % src.n_ch));
    PROF_MARK(0);
    grp_stage_sine<FRONT_NT>(r, T, xs, tid);
    __syncthreads();
    PROF_MARK(1);

    // --- MDCT of the sine-windowed block, overall scale, band peaks ------
    const double* X = grp_mdct<FRONT_NT>([&](int i) { return xs[i]; }, T, buf, tid);
    PROF_MARK(2);
    // band peaks (and the block maximum, slot 25) by LDS atomic max on the
    // bit patterns of |X|, which order like the values
    double x[4];
    unsigned long long* bk = reinterpret_cast<unsigned long long*>(buf + 512);   // free MDCT half
    if (tid < PAC_NB + 1) bk[tid] = 0ull;
    __syncthreads();
    const int lend = T->lower[PAC_NB - 1] + T->nlines[PAC_NB - 1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int l = front_row(i, w) * WAVE + lane;
        x[i] = X[l];
        atomicMax(&bk[l < lend ? T->band_of_line[l] : PAC_NB],
                  (unsigned long long)__double_as_longlong(fabs(x[i])));
    }
    __syncthreads();
    double mx = 0.0;
#pragma unroll
    for (int b = 0; b <= PAC_NB; ++b) mx = fmax(mx, __longlong_as_double((long long)bk[b]));
    const int overall = pac_scale_factor(mx, 5);
    // band peak |line| of the SCALED lines: max|X| * 2^overall (exact scaling)
    if (tid < PAC_NB)
        W.bandpeak[g * PAC_NB + tid] = T->nlines[tid] ? __longlong_as_double((long long)bk[tid]) *
                                                            (double)(1 << overall) : 0.0;
    __syncthreads();                       // bk read by all before the spectrum overwrites it
    PROF_MARK(3);

    // --- side chain: Hann(Sine(x)) spectrum (Origin psychoac.py:223) -------
    grp_spectrum_pow<FRONT_NT>([&](int i) { return __dmul_rn(xs[i], T->hann[i]); }, T, buf,
                               reinterpret_cast<double2*>(xs), tid);
    PROF_MARK(4);
    const MaskerLists L = masker_lists(buf, xs);
    int nm = grp_find_maskers<FRONT_NT>(reinterpret_cast<const double*>(buf), T, 15.0, tid, L);
    PROF_MARK(5);
    if (src.dbg & 1) nm = 0;          // diagnostic: masking sum off
    // Masking rows are claimed dynamically, most expensive first (the order
    // measured on broadband input: middle rows carry the most maskers on both
    // sides); a wave keeps its (row, threshold) pairs in registers, at most 4.
    int* rowctr = L.misc;                  // reset by grp_find_maskers before its last barrier
    double tv0 = 0.0, tv1 = 0.0, tv2 = 0.0, tv3 = 0.0;
    int rids = 0;                          // claimed rows, 4 bits each (wave-uniform)
    int nr = 0;
#pragma unroll 1
    while (nr < 4) {
        int k = 0;
        if (lane == 0) k = atomicAdd(rowctr, 1);
        k = __builtin_amdgcn_readfirstlane(k);
        if (k >= 16) break;
        const int r = (int)((PAC_ROW_ORDER >> (4 * k)) & 15);
        const double thr = wave_masking_row(L, nm, T, lane, r);
        switch (nr) {
            case 0: tv0 = thr; break;
            case 1: tv1 = thr; break;
            case 2: tv2 = thr; break;
            default: tv3 = thr; break;
        }
        rids |= r << (4 * nr);
        PROF_MARK(10 + nr);
        ++nr;
    }
    PROF_MARK(6);
    __syncthreads();
    PROF_MARK(7);
    double* thr_l = reinterpret_cast<double*>(buf);        // masker list is done
    if (nr > 0) thr_l[(rids & 15) * WAVE + lane] = tv0;
    if (nr > 1) thr_l[((rids >> 4) & 15) * WAVE + lane] = tv1;
    if (nr > 2) thr_l[((rids >> 8) & 15) * WAVE + lane] = tv2;
    if (nr > 3) thr_l[((rids >> 12) & 15) * WAVE + lane] = tv3;
    __syncthreads();
    // SMR (Origin psychoac.py:281-314) and its band maxima: SPL(4 x^2) - SPL(I)
    // as the intensity ratio (pac_spl_ratio; the thresholds are intensities),
    // atomic max on the positive doubles' bit patterns, one log10 per band
    unsigned long long* sk = reinterpret_cast<unsigned long long*>(buf + 512);
    if (tid < PAC_NB) sk[tid] = 0ull;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int l = front_row(i, w) * WAVE + lane;
        const double q = pac_spl_ratio(4.0 * (x[i] * x[i]), thr_l[l]);
        if (l < lend) atomicMax(&sk[T->band_of_line[l]], (unsigned long long)__double_as_longlong(q));
    }
    __syncthreads();
    if (tid < PAC_NB)
        W.smr[g * PAC_NB + tid] = T->nlines[tid] ? pac_ratio_db(__longlong_as_double((long long)sk[tid])) : 0.0;
    PROF_MARK(8);
    if (tid == 0) W.overall[g] = (uint8_t)overall;
}

// ---------------------------------------------------------------------------
// origin bit allocation: one lane per channel-block
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_origin_alloc(const PacTables* __restrict__ T, PacOriginWork W,
                                                      int64_t G, double bitBudget, int maxMantBits) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    double nf[PAC_NB];
    int alloc[PAC_NB];
    int nl[PAC_NB];
#pragma unroll
    for (int b = 0; b < PAC_NB; ++b) {
        nf[b] = W.smr[g * PAC_NB + b];
        alloc[b] = 0;
        nl[b] = T->nlines[b];
    }
    double remaining = bitBudget;
    long counter = 0;
    int n_ninf = 0;
    // Origin bitalloc.py:175-194; stops early once no band can take bits any
    // more (the remaining iterations would only lower noise floors).
    while (remaining > 0) {
        if (n_ninf == PAC_NB) break;
        int im = 0;
        double best = nf[0];
#pragma unroll
        for (int b = 1; b < PAC_NB; ++b)
            if (nf[b] > best) { best = nf[b]; im = b; }
        bool stuck = false;
#pragma unroll
        for (int b = 0; b < PAC_NB; ++b) {
            if (b != im) continue;
            if (alloc[b] < maxMantBits && (remaining - nl[b]) >= 0) {
                alloc[b] += 1;
                remaining -= nl[b];
            } else if (alloc[b] >= maxMantBits) {
                if (nf[b] != -INFINITY) n_ninf++;
                nf[b] = -INFINITY;
            } else {
                stuck = true;
            }
            nf[b] -= 6.0;
        }
        counter++;
        if ((double)counter > bitBudget) break;
        if (stuck) {
            bool any = false;
#pragma unroll
            for (int b = 0; b < PAC_NB; ++b)
                any |= (alloc[b] < maxMantBits) && (nf[b] != -INFINITY) && (remaining - nl[b]) >= 0;
            if (!any) break;
        }
    }
    int bits = 4;
#pragma unroll
    for (int b = 0; b < PAC_NB; ++b) {
        int a = alloc[b];
        if (a < 2) a = 0;
        if (a > maxMantBits) a = maxMantBits;
        W.ba[g * PAC_NB + b] = (uint8_t)a;
        W.sf[g * PAC_NB + b] = (uint8_t)pac_scale_factor(W.bandpeak[g * PAC_NB + b], a);
        bits += 8 + a * nl[b];
    }
    W.nbytes[g] = 4 + (bits + 7) / 8;
}

// ---------------------------------------------------------------------------
// exclusive scan of int32 sizes -> int64 offsets (3 kernels, 2048 per tile)
// ---------------------------------------------------------------------------

__device__ __forceinline__ int64_t block_exclusive_scan_256(int64_t v, int64_t* sh, int64_t* total) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        int64_t w = t >= o ? sh[t - o] : 0;
        __syncthreads();
        sh[t] += w;
        __syncthreads();
    }
    int64_t incl = sh[t];
    *total = sh[255];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(256) void k_scan_tiles(const int32_t* __restrict__ sz, int64_t n,
                                                    int64_t* __restrict__ tile_sums) {
    __shared__ int64_t sh[256];
    int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    int64_t acc = 0;
    for (int k = 0; k < SCAN_TILE / 256; ++k) {
        int64_t i = base + k * 256 + threadIdx.x;
        acc += i < n ? sz[i] : 0;
    }
    int64_t tot;
    block_exclusive_scan_256(acc, sh, &tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_scan_sums(int64_t* __restrict__ tile_sums, int64_t ntiles,
                                                   int64_t* __restrict__ grand_total) {
    __shared__ int64_t sh[256];
    int64_t carry = 0;
    for (int64_t b0 = 0; b0 < ntiles; b0 += 256) {
        int64_t i = b0 + threadIdx.x;
        int64_t v = i < ntiles ? tile_sums[i] : 0;
        int64_t tot;
        int64_t ex = block_exclusive_scan_256(v, sh, &tot);
        if (i < ntiles) tile_sums[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *grand_total = carry;
}

__global__ __launch_bounds__(256) void k_scan_apply(const int32_t* __restrict__ sz, int64_t n,
                                                    const int64_t* __restrict__ tile_sums,
                                                    int64_t* __restrict__ off) {
    __shared__ int64_t sh[256];
    int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    // each thread owns 8 consecutive elements
    int64_t i0 = base + threadIdx.x * 8;
    int64_t v[8], acc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int64_t i = i0 + k;
        v[k] = i < n ? sz[i] : 0;
        acc += v[k];
    }
    int64_t tot;
    int64_t ex = block_exclusive_scan_256(acc, sh, &tot) + tile_sums[blockIdx.x];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int64_t i = i0 + k;
        if (i < n) off[i] = ex;
        ex += v[k];
    }
}

// ---------------------------------------------------------------------------
// bit packing helpers (MSB-first, bitpack.py:36-101), LDS u32 words
// ---------------------------------------------------------------------------

// The packed stream is kept as big-endian 32-bit words in LDS (stream bit i =
// bit 31 - (i & 31) of word i >> 5), so a field of w <= 32 bits at bit p is at
// most two atomicOr's; bytes come out as byte 3 - (i & 3) of word i >> 2.
__device__ __forceinline__ void put_bits(uint32_t* words, int p, uint32_t v, int w) {
    if (w <= 0) return;
    const int o = p & 31;
    const uint64_t x = (uint64_t)(v & (w >= 32 ? 0xffffffffu : ((1u << w) - 1u))) << (64 - o - w);
    atomicOr(&words[p >> 5], (uint32_t)(x >> 32));
    if (o + w > 32) atomicOr(&words[(p >> 5) + 1], (uint32_t)x);
}
__device__ __forceinline__ uint8_t be_byte(const uint32_t* words, int i) {
    return (uint8_t)(words[i >> 2] >> (24 - 8 * (i & 3)));
}

__device__ __forceinline__ void store_block_bytes(uint8_t* __restrict__ out, const uint32_t* words,
                                                  int nbytes, int lane) {
    if (lane < 4) out[lane] = (uint8_t)((uint32_t)nbytes >> (8 * lane));   // '<L' nBytes
    for (int i = lane; i < nbytes; i += WAVE) out[4 + i] = be_byte(words, i);
}

#define PACK_WORDS 640   // >= (4 + 25*8 + 16*1024 + 25 + 1024)/32 bits

// ---------------------------------------------------------------------------
// origin pack: one wave per channel-block
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(FRONT_NT) void k_origin_pack(PacSource src, const PacTables* __restrict__ T,
                                                          PacOriginWork W, int64_t G,
                                                          const int64_t* __restrict__ off,
                                                          uint8_t* __restrict__ out, int64_t cap) {
    __shared__ double2 buf[1024];        // MDCT: lines in the first 8 KB
    __shared__ uint32_t words[PACK_WORDS];
    __shared__ int start[PAC_NB];
    __shared__ int bas[PAC_NB], sfs[PAC_NB];
    const int tid = threadIdx.x;
    const int64_t g = xcd_item(blockIdx.x, G);
    const BlockRef r = locate(src, g / src.n_ch, (int)(g % src.n_ch));
    // loads that depend only on g, issued before the MDCT (latency-bound chain)
    const int overall = W.overall[g];
    const int nbytes = W.nbytes[g] - 4;
    const int64_t og = off[g];
    int bl[4], lo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        bl[j] = T->band_of_line[j * FRONT_NT + tid];
        lo[j] = T->lower[bl[j]];
    }
    for (int i = tid; i < PACK_WORDS; i += FRONT_NT) words[i] = 0;
    if (tid < PAC_NB) {
        bas[tid] = W.ba[g * PAC_NB + tid];
        sfs[tid] = W.sf[g * PAC_NB + tid];
    }
    const BlockPcm xp(r);
    const double* X = grp_mdct<FRONT_NT>([&](int i) { return __dmul_rn(xp(i), T->sine[i]); }, T, buf, tid);
    // (same arithmetic as the front kernel's staged xs: identical lines)
    if (tid == 0) {
        int p = 4;
        for (int b = 0; b < PAC_NB; ++b) { start[b] = p; p += 8 + bas[b] * T->nlines[b]; }
    }
    __syncthreads();
    const double gain = (double)(1 << overall);
    if (tid == 0) put_bits(words, 0, (uint32_t)overall, 4);
    if (tid < PAC_NB) {
        int ba = bas[tid];
        put_bits(words, start[tid], (uint32_t)(ba ? ba - 1 : 0), 4);
        put_bits(words, start[tid] + 4, (uint32_t)sfs[tid], 4);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int l = j * FRONT_NT + tid;
        int b = bl[j];
        int ba = bas[b];
        if (ba) {
            uint32_t m = pac_mantissa(X[l] * gain, sfs[b], ba);
            put_bits(words, start[b] + 8 + (l - lo[j]) * ba, m, ba);
        }
    }
    __syncthreads();
    if (og + 4 + nbytes > cap) return;     // host reports PAC_E_CAPACITY from the total
    uint8_t* o = out + og;
    if (tid < 4) o[tid] = (uint8_t)((uint32_t)nbytes >> (8 * tid));   // '<L' nBytes
    for (int i = tid; i < nbytes; i += FRONT_NT) o[4 + i] = be_byte(words, i);
}

// ---------------------------------------------------------------------------
// debug / parity probe: the masking threshold of arbitrary 2048-sample blocks
// (data already windowed as calcBTHR receives it; Hann applied here)
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(64) void k_debug_threshold(const PacTables* __restrict__ T,
                                                        const double* __restrict__ data, int no_drop,
                                                        double* __restrict__ thr_out,
                                                        int32_t* __restrict__ npeaks) {
    __shared__ double2 buf[1024];
    __shared__ double2 tmp[1024];
    const int lane = threadIdx.x;
    const double* d = data + (int64_t)blockIdx.x * PAC_N;
    wave_spectrum_pow([&](int i) { return __dmul_rn(d[i], T->hann[i]); }, T, buf, tmp, lane);
    const MaskerLists L = masker_lists(buf, tmp);
    const int nm = grp_find_maskers<WAVE>(reinterpret_cast<const double*>(buf), T, no_drop ? 0.0 : 15.0, lane, L);
#pragma unroll 1
    for (int q = 0; q < 16; ++q)
        thr_out[(int64_t)blockIdx.x * PAC_HALFN + q * WAVE + lane] = pac_spl(wave_masking_row(L, nm, T, lane, q));
    if (lane == 0) npeaks[blockIdx.x] = nm;
}

// MDCT probe: mdct.py:49-82 of n raw (unwindowed) blocks, sine window applied
__global__ __launch_bounds__(64) void k_debug_mdct(const PacTables* __restrict__ T,
                                                   const double* __restrict__ data, double* __restrict__ X) {
    __shared__ double2 buf[1024];
    const int lane = threadIdx.x;
    const double* d = data + (int64_t)blockIdx.x * PAC_N;
    const double* Xs = wave_mdct([&](int i) { return __dmul_rn(d[i], T->sine[i]); }, T, buf, lane);
    for (int k = lane; k < PAC_HALFN; k += WAVE) X[(int64_t)blockIdx.x * PAC_HALFN + k] = Xs[k];
}

// ---------------------------------------------------------------------------
// synthetic input (bench): counter-hash Gaussian PCM, 48 kHz stereo config 2
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// sample n of a stream: N(0,1) * 0.25 * 32767, rounded, clipped to int16
// (Box-Muller from two 53-bit uniforms; host mirror: pac_amd.synth.white_pcm)
__global__ void k_synth_white(int16_t* __restrict__ pcm, int64_t n, uint64_t seed) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) {
        uint64_t h1 = splitmix64(seed ^ (2 * (uint64_t)i));
        uint64_t h2 = splitmix64(seed ^ (2 * (uint64_t)i + 1));
        double u1 = ((double)(h1 >> 11) + 1.0) * 0x1.0p-53;   // (0,1]
        double u2 = (double)(h2 >> 11) * 0x1.0p-53;           // [0,1)
        double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
        double v = __builtin_rint(z * 0.25 * 32767.0);
        v = v > 32767.0 ? 32767.0 : (v < -32768.0 ? -32768.0 : v);
        pcm[i] = (int16_t)v;
    }
}

// synthetic config-3 input (bench): pink noise + tones, stereo interleaved.
// Pink: Voss-McCartney sum of 16 octave-held uniform hashes (counter based,
// so every sample is independent work); tones 440/1250/5300 Hz as in
// pac_amd.synth.pink_tones_pcm.  L = 0.1 p1 + tones, R = 0.07 p1 + 0.03 p2 + 0.8 tones.
__device__ __forceinline__ double voss_pink(uint64_t seed, int64_t i) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint64_t h = splitmix64(seed ^ ((uint64_t)k << 56) ^ (uint64_t)(i >> k));
        acc += (double)(h >> 11) * 0x1.0p-52 - 1.0;        // uniform [-1, 1)
    }
    return acc * 0.4330127018922193;                          // / sqrt(16/3): unit variance
}
__global__ void k_synth_pink_tones(int16_t* __restrict__ pcm, int64_t n_frames, double fs, uint64_t seed) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (; i < n_frames; i += stride) {
        const double t = (double)i / fs;
        const double tones = 0.2 * sin(6.283185307179586 * 440.0 * t) +
                             0.1 * sin(6.283185307179586 * 1250.0 * t) +
                             0.05 * sin(6.283185307179586 * 5300.0 * t);
        const double p1 = voss_pink(seed, i), p2 = voss_pink(seed ^ 0x5bd1e995ull, i);
        double v[2] = {0.1 * p1 + tones, 0.07 * p1 + 0.03 * p2 + 0.8 * tones};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            double x = __builtin_rint(v[c] * 32767.0);
            x = x > 32767.0 ? 32767.0 : (x < -32768.0 ? -32768.0 : x);
            pcm[2 * i + c] = (int16_t)x;
        }
    }
}

// synthetic configs[4] input (bench, block switching): decaying noise bursts
// added in place to stereo interleaved PCM.  One burst per period of `period`
// frames, its onset at a hashed offset in [0, period - 2560); burst sample at
// d frames after the onset = gaussian(hash) * env, env = exp(-d / 500) over
// 2560 frames, amplitude 0.4 (L) / 0.3 (R) of full scale; saturating int16.
__global__ void k_synth_bursts(int16_t* __restrict__ pcm, int64_t n_frames, int64_t period, uint64_t seed) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (; i < n_frames; i += stride) {
        const int64_t per = i / period;
        const int64_t t0 = per * period + (int64_t)(splitmix64(seed ^ 0x9e3779b97f4a7c15ull ^ (uint64_t)per) %
                                                    (uint64_t)(period - 2560));
        const int64_t d = i - t0;
        if (d < 0 || d >= 2560) continue;
        const double env = exp(-(double)d / 500.0);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const uint64_t h1 = splitmix64(seed ^ (4 * (uint64_t)i + 2 * c));
            const uint64_t h2 = splitmix64(seed ^ (4 * (uint64_t)i + 2 * c + 1));
            const double u1 = ((double)(h1 >> 11) + 1.0) * 0x1.0p-53, u2 = (double)(h2 >> 11) * 0x1.0p-53;
            const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
            double x = (double)pcm[2 * i + c] + __builtin_rint(z * (c ? 0.3 : 0.4) * 32767.0 * env);
            x = x > 32767.0 ? 32767.0 : (x < -32768.0 ? -32768.0 : x);
            pcm[2 * i + c] = (int16_t)x;
        }
    }
}
