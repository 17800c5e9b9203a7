// pac_wave.h -- one-wavefront building blocks of the per-block encode path on
// gfx950: radix-2 FFTs staged in LDS, the sine-window MDCT (N/4-point complex
// FFT form of mdct.py:49-82), the Hann-window side-chain spectrum
// (psychoac.py:428), findpeaks + masker SPL (psychoac.py:158-191, 442-449) and
// the masking-threshold sum (psychoac.py:447-456).
//
// Every function here is executed by ONE 64-lane wave that owns its LDS
// scratch; "wave sync" is __syncthreads() on a 64-thread workgroup, or a
// wave barrier when several independent waves share a workgroup.
#pragma once
#include "pac_common.h"

#define WAVE 64

// The barriers of these kernels hand off LDS only (no workgroup passes data
// to itself through global memory), so their fences are restricted to the
// local address space: they drain LDS operations (lgkmcnt) but leave global
// loads in flight -- a plain workgroup fence also waits for every outstanding
// global load (vmcnt), which serialised table and threshold loads with the
// barriers of each FFT stage.

__device__ __forceinline__ void wave_sync() {
    // LDS hand-off between lanes of one wave: drain this wave's LDS ops and
    // keep the compiler from moving LDS accesses across (waves never share LDS).
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// workgroup barrier for an LDS hand-off
__device__ __forceinline__ void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}


// Cross-lane moves of a double through DPP (VALU, no LDS round trip).  Lanes
// outside ROWMASK (or without a source) get `old`.
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ double dpp_f64(double old, double v) {
    const long long b = __double_as_longlong(v), o = __double_as_longlong(old);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, CTRL, ROWMASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), CTRL, ROWMASK, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
// full-row DPP patterns (every lane has a source): bound_ctrl, no old value
template <int CTRL>
__device__ __forceinline__ double dpp_full_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
#define PAC_DPP_QXOR1 0xB1     // quad_perm [1,0,3,2]
#define PAC_DPP_QXOR2 0x4E     // quad_perm [2,3,0,1]
#define PAC_DPP_HMIRROR 0x141  // row_half_mirror
#define PAC_DPP_MIRROR 0x140   // row_mirror
#define PAC_DPP_BCAST15 0x142
#define PAC_DPP_BCAST31 0x143
// Wave-wide reductions (wave-uniform result; the same value on every lane)
__device__ __forceinline__ double wave_sum_f64(double v) {
    v += dpp_full_f64<PAC_DPP_QXOR1>(v);
    v += dpp_full_f64<PAC_DPP_QXOR2>(v);
    v += dpp_full_f64<PAC_DPP_HMIRROR>(v);
    v += dpp_full_f64<PAC_DPP_MIRROR>(v);              // row sums
    v += dpp_f64<PAC_DPP_BCAST15, 0xa>(0.0, v);        // rows 1, 3 += rows 0, 2
    v += dpp_f64<PAC_DPP_BCAST31, 0xc>(0.0, v);        // rows 2, 3 += rows 0 + 1
    return readlane_f64(v, 63);
}
__device__ __forceinline__ int wave_sum_i(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, PAC_DPP_QXOR1, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, PAC_DPP_QXOR2, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, PAC_DPP_HMIRROR, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, PAC_DPP_MIRROR, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, PAC_DPP_BCAST15, 0xa, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, PAC_DPP_BCAST31, 0xc, 0xf, false);
    return __builtin_amdgcn_readlane(v, 63);
}
template <bool MAX>
__device__ __forceinline__ double wave_ext_f64(double v) {
    // compare-select (no NaN canonicalisation: the operands are never NaN)
    auto f = [](double a, double b) { return MAX ? (a > b ? a : b) : (a < b ? a : b); };
    v = f(v, dpp_full_f64<PAC_DPP_QXOR1>(v));
    v = f(v, dpp_full_f64<PAC_DPP_QXOR2>(v));
    v = f(v, dpp_full_f64<PAC_DPP_HMIRROR>(v));
    v = f(v, dpp_full_f64<PAC_DPP_MIRROR>(v));
    v = f(v, dpp_f64<PAC_DPP_BCAST15, 0xa>(v, v));
    v = f(v, dpp_f64<PAC_DPP_BCAST31, 0xc>(v, v));
    return readlane_f64(v, 63);
}

__device__ __forceinline__ unsigned brev(unsigned x, int bits) {
    return __builtin_bitreverse32(x) >> (32 - bits);
}

template <int NT>
__device__ __forceinline__ void grp_sync() {
    if constexpr (NT == WAVE) wave_sync(); else lds_sync();
}

// In-place radix-2 DIT FFT of n = 2^LOG complex values that were stored in
// bit-reversed order, by a group of NT threads (one wave or a workgroup).
// Twiddles: tw[k] = exp(-2 pi i k / 1024), k < 512.
template <int LOG, int NT>
__device__ __forceinline__ void grp_fft(double2* buf, const double2* __restrict__ tw, int tid) {
    constexpr int n = 1 << LOG;
#pragma unroll 1
    for (int s = 1; s <= LOG; ++s) {
        const int half = 1 << (s - 1);
        const int tstride = 1024 >> s;
        grp_sync<NT>();
#pragma unroll
        for (int t0 = 0; t0 < n / 2; t0 += NT) {
            int t = t0 + tid;
            int k = t & (half - 1);
            int i = ((t >> (s - 1)) << s) + k;
            double2 w = tw[k * tstride];
            double2 a = buf[i], b = buf[i + half];
            double2 bw = cmul(b, w);
            buf[i] = make_double2(__dadd_rn(a.x, bw.x), __dadd_rn(a.y, bw.y));
            buf[i + half] = make_double2(__dsub_rn(a.x, bw.x), __dsub_rn(a.y, bw.y));
        }
    }
    grp_sync<NT>();
}

// Bank-conflict-free LDS layout of the Stockham stage buffers.  MI355X LDS
// banking: ds_read_b128 serves 16-lane groups over a 256-B bank row,
// ds_write_b128 8-lane groups over 128 B, so the stride-4 and stride-16
// writes of the first stages cost 4-way / 2-way conflicts in the plain
// layout.  Element i of an intermediate stage buffer is stored at
// i ^ fft_swz(i), fft_swz a GF(2)-linear function of index bits 3..7 (found
// by exhaustive search over the stages' access patterns, N = 128..1024): every
// read and write of every stage is conflict-free (2/3 of the plain layout's
// LDS cycles).  The first stage reads and the last stage writes the plain
// layout, so callers never see it.  Linear: fft_swz(a + b) =
// fft_swz(a) ^ fft_swz(b) for bit-disjoint a, b (one swizzle per butterfly,
// the other offsets are compile-time constants).
// the twiddles W^e, W^2e, W^3e (e = k 256/Ns) of a radix-4 stage Ns >= 4 from the
// stage-major table after fft_tw (PacTables::fft_tw4): one contiguous run per
// wave instead of three strided reads of fft_tw (3x fewer cache lines in the
// late stages); the same values, bit-identical
__device__ __forceinline__ const double2* tw4_of(const double2* __restrict__ tw, int Ns, int k) {
    return tw + PAC_HALFN + 3 * ((Ns - 4) / 3 + k);
}

__host__ __device__ constexpr int fft_swz(int i) {
    return (((i >> 3) & 1) * 1) ^ (((i >> 4) & 1) * 14) ^ (((i >> 5) & 1) * 2) ^ (((i >> 6) & 1) * 1) ^
           (((i >> 7) & 1) * 7);
}

// Self-sorting (Stockham) FFT of n = 2^LOG complex values in natural order,
// radix-4 stages (+ one radix-2 stage for odd LOG), ping-ponging between src
// and dst; every read is unit-stride across lanes and no bit-reversal
// permutation is needed.  Returns the buffer holding the result (always dst:
// LOG = 10 has 5 stages, LOG = 9 has 4 + 1).  tw[k] = exp(-2 pi i k / 1024).
template <int LOG, int NT, bool SWZ = true>   // SWZ = false: plain layout (fewer VGPRs, bit-identical)
__device__ __forceinline__ double2* grp_fft_stockham(double2* src, double2* dst,
                                                     const double2* __restrict__ tw, int tid) {
    constexpr int N = 1 << LOG;
    constexpr int N4 = N / 4;
#pragma unroll
    for (int st = 0; st < LOG / 2; ++st) {
        const int Ns = 1 << (2 * st);
        grp_sync<NT>();
#pragma unroll
        for (int j0 = 0; j0 < N4; j0 += NT) {
            const int j = j0 + tid;
            if (N4 % NT != 0 && j >= N4) break;
            const int k = j & (Ns - 1);
            const bool swi = SWZ && st > 0, swo = SWZ && (st + 1 < LOG / 2 || (LOG & 1));   // plain in first, out last
            const int xj = swi ? fft_swz(j) : 0;
            double2 v0 = src[j ^ xj], v1 = src[(j + N4) ^ xj ^ (swi ? fft_swz(N4) : 0)];
            double2 v2 = src[(j + 2 * N4) ^ xj ^ (swi ? fft_swz(2 * N4) : 0)];
            double2 v3 = src[(j + 3 * N4) ^ xj ^ (swi ? fft_swz(3 * N4) : 0)];
            if (Ns > 1) {                               // angles -2 pi k r / (4 Ns)
                const double2* w = tw4_of(tw, Ns, k);
                v1 = cmul(v1, w[0]);
                v2 = cmul(v2, w[1]);
                v3 = cmul(v3, w[2]);
            }
            const double2 a0 = make_double2(v0.x + v2.x, v0.y + v2.y);
            const double2 a1 = make_double2(v0.x - v2.x, v0.y - v2.y);
            const double2 a2 = make_double2(v1.x + v3.x, v1.y + v3.y);
            const double2 a3 = make_double2(v1.y - v3.y, v3.x - v1.x);   // -i (v1 - v3)
            const int o = ((j - k) << 2) + k;
            const int xo = swo ? fft_swz(o) : 0;
            dst[o ^ xo] = make_double2(a0.x + a2.x, a0.y + a2.y);
            dst[(o + Ns) ^ xo ^ (swo ? fft_swz(Ns) : 0)] = make_double2(a1.x + a3.x, a1.y + a3.y);
            dst[(o + 2 * Ns) ^ xo ^ (swo ? fft_swz(2 * Ns) : 0)] = make_double2(a0.x - a2.x, a0.y - a2.y);
            dst[(o + 3 * Ns) ^ xo ^ (swo ? fft_swz(3 * Ns) : 0)] = make_double2(a1.x - a3.x, a1.y - a3.y);
        }
        double2* t = src; src = dst; dst = t;
    }
    if (LOG & 1) {                                     // last stage, radix 2, Ns = N/2
        grp_sync<NT>();
#pragma unroll
        for (int j0 = 0; j0 < N / 2; j0 += NT) {
            const int j = j0 + tid;
            if ((N / 2) % NT != 0 && j >= N / 2) break;
            const int xj = SWZ ? fft_swz(j) : 0;
            const double2 v0 = src[j ^ xj];
            const double2 v1 = cmul(src[(j + N / 2) ^ xj ^ (SWZ ? fft_swz(N / 2) : 0)], tw[j * (1024 / N)]);
            dst[j] = make_double2(v0.x + v1.x, v0.y + v1.y);
            dst[j + N / 2] = make_double2(v0.x - v1.x, v0.y - v1.y);
        }
        double2* t = src; src = dst; dst = t;
    }
    grp_sync<NT>();
    return src;
}

// The same Stockham FFT in ONE buffer: each stage reads its four inputs into
// registers, waits until every thread has read, then writes its outputs in
// place of them -- identical arithmetic (bit-identical results) with half the
// LDS.  Result in buf.
template <int LOG, int NT>
__device__ __forceinline__ void grp_fft_stockham_1buf(double2* buf, const double2* __restrict__ tw, int tid) {
    constexpr int N = 1 << LOG;
    constexpr int N4 = N / 4;
    constexpr int J = N4 >= NT ? N4 / NT : 1;
    static_assert(N4 % NT == 0 || N4 < NT, "stage items per thread");
#pragma unroll
    for (int st = 0; st < LOG / 2; ++st) {
        const int Ns = 1 << (2 * st);
        double2 v[J][4];
        grp_sync<NT>();
#pragma unroll
        for (int q = 0; q < J; ++q) {
            const int j = q * NT + tid;
            if (N4 < NT && j >= N4) break;
            const int k = j & (Ns - 1);
            const bool swi = st > 0;
            const int xj = swi ? fft_swz(j) : 0;
            v[q][0] = buf[j ^ xj];
            v[q][1] = buf[(j + N4) ^ xj ^ (swi ? fft_swz(N4) : 0)];
            v[q][2] = buf[(j + 2 * N4) ^ xj ^ (swi ? fft_swz(2 * N4) : 0)];
            v[q][3] = buf[(j + 3 * N4) ^ xj ^ (swi ? fft_swz(3 * N4) : 0)];
            if (Ns > 1) {
                const double2* w = tw4_of(tw, Ns, k);
                v[q][1] = cmul(v[q][1], w[0]);
                v[q][2] = cmul(v[q][2], w[1]);
                v[q][3] = cmul(v[q][3], w[2]);
            }
        }
        grp_sync<NT>();
#pragma unroll
        for (int q = 0; q < J; ++q) {
            const int j = q * NT + tid;
            if (N4 < NT && j >= N4) break;
            const int k = j & (Ns - 1);
            const double2 a0 = make_double2(v[q][0].x + v[q][2].x, v[q][0].y + v[q][2].y);
            const double2 a1 = make_double2(v[q][0].x - v[q][2].x, v[q][0].y - v[q][2].y);
            const double2 a2 = make_double2(v[q][1].x + v[q][3].x, v[q][1].y + v[q][3].y);
            const double2 a3 = make_double2(v[q][1].y - v[q][3].y, v[q][3].x - v[q][1].x);
            const int o = ((j - k) << 2) + k;
            const bool swo = st + 1 < LOG / 2 || (LOG & 1);
            const int xo = swo ? fft_swz(o) : 0;
            buf[o ^ xo] = make_double2(a0.x + a2.x, a0.y + a2.y);
            buf[(o + Ns) ^ xo ^ (swo ? fft_swz(Ns) : 0)] = make_double2(a1.x + a3.x, a1.y + a3.y);
            buf[(o + 2 * Ns) ^ xo ^ (swo ? fft_swz(2 * Ns) : 0)] = make_double2(a0.x - a2.x, a0.y - a2.y);
            buf[(o + 3 * Ns) ^ xo ^ (swo ? fft_swz(3 * Ns) : 0)] = make_double2(a1.x - a3.x, a1.y - a3.y);
        }
    }
    if (LOG & 1) {
        constexpr int J2 = (N / 2) >= NT ? (N / 2) / NT : 1;
        double2 v0[J2], v1[J2];
        grp_sync<NT>();
#pragma unroll
        for (int q = 0; q < J2; ++q) {
            const int j = q * NT + tid;
            if ((N / 2) < NT && j >= N / 2) break;
            const int xj = fft_swz(j);
            v0[q] = buf[j ^ xj];
            v1[q] = cmul(buf[(j + N / 2) ^ xj ^ fft_swz(N / 2)], tw[j * (1024 / N)]);
        }
        grp_sync<NT>();
#pragma unroll
        for (int q = 0; q < J2; ++q) {
            const int j = q * NT + tid;
            if ((N / 2) < NT && j >= N / 2) break;
            buf[j] = make_double2(v0[q].x + v1[q].x, v0[q].y + v1[q].y);
            buf[j + N / 2] = make_double2(v0[q].x - v1[q].x, v0[q].y - v1[q].y);
        }
    }
    grp_sync<NT>();
}

// Two independent one-buffer Stockham FFTs (buffers a and b) advanced stage by
// stage together: each thread's butterflies of both in flight, one pair of
// barriers per stage for both.  grp_fft_stockham_1buf's arithmetic with the
// twiddle products as fused multiply-adds (cmul_fma).
// The first stage takes its inputs from ld(n) = (a[n], b[n]) as a double4
// (the staged sample pairs, computed from global memory) instead of LDS: no
// staging pass and no first-stage barriers (the caller guarantees that no
// thread still reads a or b).
template <int LOG, int NT, class LD>
__device__ __forceinline__ void grp_fft_stockham_1buf_x2(double2* a, double2* b, const double2* __restrict__ tw,
                                                         int tid, const LD& ld) {
    constexpr int N = 1 << LOG;
    constexpr int N4 = N / 4;
    static_assert(N4 % NT == 0 && !(LOG & 1), "one radix-4 butterfly set per thread and stage");
    constexpr int J = N4 / NT;
    double2* bufs[2] = {a, b};
#pragma unroll
    for (int st = 0; st < LOG / 2; ++st) {
        const int Ns = 1 << (2 * st);
        double2 v[2][J][4];
        if (st == 0) {
#pragma unroll
            for (int q = 0; q < J; ++q)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const double4 x = ld(q * NT + tid + i * N4);
                    v[0][q][i] = make_double2(x.x, x.y);
                    v[1][q][i] = make_double2(x.z, x.w);
                }
        } else {
            grp_sync<NT>();
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int q = 0; q < J; ++q) {
                    const int j = q * NT + tid;
                    const int k = j & (Ns - 1);
                    const int xj = fft_swz(j);
                    v[u][q][0] = bufs[u][j ^ xj];
                    v[u][q][1] = bufs[u][(j + N4) ^ xj ^ fft_swz(N4)];
                    v[u][q][2] = bufs[u][(j + 2 * N4) ^ xj ^ fft_swz(2 * N4)];
                    v[u][q][3] = bufs[u][(j + 3 * N4) ^ xj ^ fft_swz(3 * N4)];
                    const double2* w = tw4_of(tw, Ns, k);
                    v[u][q][1] = cmul_fma(v[u][q][1], w[0]);
                    v[u][q][2] = cmul_fma(v[u][q][2], w[1]);
                    v[u][q][3] = cmul_fma(v[u][q][3], w[2]);
                }
            grp_sync<NT>();
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int q = 0; q < J; ++q) {
                const int j = q * NT + tid;
                const int k = j & (Ns - 1);
                const double2* w = v[u][q];
                const double2 a0 = make_double2(w[0].x + w[2].x, w[0].y + w[2].y);
                const double2 a1 = make_double2(w[0].x - w[2].x, w[0].y - w[2].y);
                const double2 a2 = make_double2(w[1].x + w[3].x, w[1].y + w[3].y);
                const double2 a3 = make_double2(w[1].y - w[3].y, w[3].x - w[1].x);
                const int o = ((j - k) << 2) + k;
                const bool swo = st + 1 < LOG / 2;      // LOG even here
                const int xo = swo ? fft_swz(o) : 0;
                bufs[u][o ^ xo] = make_double2(a0.x + a2.x, a0.y + a2.y);
                bufs[u][(o + Ns) ^ xo ^ (swo ? fft_swz(Ns) : 0)] = make_double2(a1.x + a3.x, a1.y + a3.y);
                bufs[u][(o + 2 * Ns) ^ xo ^ (swo ? fft_swz(2 * Ns) : 0)] = make_double2(a0.x - a2.x, a0.y - a2.y);
                bufs[u][(o + 3 * Ns) ^ xo ^ (swo ? fft_swz(3 * Ns) : 0)] = make_double2(a1.x - a3.x, a1.y - a3.y);
            }
    }
    grp_sync<NT>();
}

// Two independent ping-pong Stockham FFTs (src/dst pairs a, b) of N = 2^LOG
// points, LOG odd, N4 = N/4 = NT/2 (a 512-point pair on 256 threads), stage by
// stage together (one barrier per stage for both, bit-identical to
// grp_fft_stockham on each); returns the result buffers of a and b.  The
// radix-4 stages split the threads, not the butterflies --
// threads [0, N4) run FFT a, [N4, NT) FFT b, one butterfly each (no idle
// half-workgroup) -- and the first stage takes its inputs from ld(n, u)
// (element n of FFT u, computed from global memory) instead of LDS: no
// staging pass, no first-stage barrier.
template <int LOG, int NT, class LD>
__device__ __forceinline__ void grp_fft_stockham_x2_ld(double2* sa, double2* da, double2* sb, double2* db,
                                                       const double2* __restrict__ tw, int tid, const LD& ld,
                                                       double2** ra, double2** rb) {
    constexpr int N = 1 << LOG;
    constexpr int N4 = N / 4;
    static_assert(2 * N4 == NT && (LOG & 1), "a 2^odd pair split over the workgroup");
    const int u = tid / N4, j = tid % N4;           // u wave-uniform (N4 a multiple of the wave)
#pragma unroll
    for (int st = 0; st < LOG / 2; ++st) {
        const int Ns = 1 << (2 * st);
        const double2* src = u ? sb : sa;
        double2* dst = u ? db : da;
        const int k = j & (Ns - 1);
        double2 v0, v1, v2, v3;
        if (st == 0) {
            v0 = ld(j, u);
            v1 = ld(j + N4, u);
            v2 = ld(j + 2 * N4, u);
            v3 = ld(j + 3 * N4, u);
        } else {
            grp_sync<NT>();
            const int xj = fft_swz(j);
            v0 = src[j ^ xj];
            v1 = src[(j + N4) ^ xj ^ fft_swz(N4)];
            v2 = src[(j + 2 * N4) ^ xj ^ fft_swz(2 * N4)];
            v3 = src[(j + 3 * N4) ^ xj ^ fft_swz(3 * N4)];
            const double2* w = tw4_of(tw, Ns, k);
            v1 = cmul(v1, w[0]);
            v2 = cmul(v2, w[1]);
            v3 = cmul(v3, w[2]);
        }
        const double2 a0 = make_double2(v0.x + v2.x, v0.y + v2.y);
        const double2 a1 = make_double2(v0.x - v2.x, v0.y - v2.y);
        const double2 a2 = make_double2(v1.x + v3.x, v1.y + v3.y);
        const double2 a3 = make_double2(v1.y - v3.y, v3.x - v1.x);
        const int o = ((j - k) << 2) + k;
        const int xo = fft_swz(o);                  // LOG odd: every radix-4 stage writes swizzled
        dst[o ^ xo] = make_double2(a0.x + a2.x, a0.y + a2.y);
        dst[(o + Ns) ^ xo ^ fft_swz(Ns)] = make_double2(a1.x + a3.x, a1.y + a3.y);
        dst[(o + 2 * Ns) ^ xo ^ fft_swz(2 * Ns)] = make_double2(a0.x - a2.x, a0.y - a2.y);
        dst[(o + 3 * Ns) ^ xo ^ fft_swz(3 * Ns)] = make_double2(a1.x - a3.x, a1.y - a3.y);
        double2* t = sa; sa = da; da = t;
        t = sb; sb = db; db = t;
    }
    grp_sync<NT>();                                 // last stage, radix 2, Ns = N/2
#pragma unroll
    for (int w = 0; w < 2; ++w) {
        const double2* src = w ? sb : sa;
        double2* dst = w ? db : da;
#pragma unroll
        for (int j0 = 0; j0 < N / 2; j0 += NT) {
            const int jj = j0 + tid;
            const int xj = fft_swz(jj);
            const double2 v0 = src[jj ^ xj];
            const double2 v1 = cmul(src[(jj + N / 2) ^ xj ^ fft_swz(N / 2)], tw[jj * (1024 / N)]);
            dst[jj] = make_double2(v0.x + v1.x, v0.y + v1.y);
            dst[jj + N / 2] = make_double2(v0.x - v1.x, v0.y - v1.y);
        }
    }
    double2* t = sa; sa = da; da = t;
    t = sb; sb = db; db = t;
    grp_sync<NT>();
    *ra = sa;
    *rb = sb;
}

// DCT-IV of 1024 values v(j), scaled by sc (a power of two):
//   X[k] = sc * sum_j v(j) cos(pi/1024 (j + 1/2)(k + 1/2)),
// via the 512-point complex Stockham FFT (even/odd interleave, pre- and
// post-twiddles).  buf: 1024 double2 of LDS; X = (double*)buf on return (first
// 8 KB), the second 8 KB is free scratch.
template <int NT, bool SWZ = true, class V>
__device__ __forceinline__ double* grp_dct4(const V& v, const PacTables* __restrict__ T, double2* buf, int tid,
                                            double sc) {
#pragma unroll
    for (int q0 = 0; q0 < 512; q0 += NT) {
        const int q = q0 + tid;
        buf[q] = cmul(make_double2(v(2 * q), v(1023 - 2 * q)), T->mdct_pre[q]);
    }
    const double2* Y = grp_fft_stockham<9, NT, SWZ>(buf, buf + 512, T->fft_tw, tid);   // = buf + 512
    double* X = reinterpret_cast<double*>(buf);
#pragma unroll
    for (int q0 = 0; q0 < 512; q0 += NT) {
        const int q = q0 + tid;
        const double2 y = cmul(Y[q], T->mdct_post[q]);
        X[2 * q] = y.x * sc;
        X[1023 - 2 * q] = -y.y * sc;
    }
    grp_sync<NT>();
    return X;
}

// grp_dct4 with its input already in registers, in the pre-twiddle's order:
// x[2 i] = v(2 q), x[2 i + 1] = v(1023 - 2 q) for q = i NT + tid (no LDS
// staging of the input).  Bit-identical to grp_dct4.
template <int NT, bool SWZ = true>
__device__ __forceinline__ double* grp_dct4_regs(const double (&x)[1024 / NT], const PacTables* __restrict__ T,
                                                 double2* buf, int tid, double sc) {
#pragma unroll
    for (int i = 0; i < 512 / NT; ++i) {
        const int q = i * NT + tid;
        buf[q] = cmul(make_double2(x[2 * i], x[2 * i + 1]), T->mdct_pre[q]);
    }
    const double2* Y = grp_fft_stockham<9, NT, SWZ>(buf, buf + 512, T->fft_tw, tid);
    double* X = reinterpret_cast<double*>(buf);
#pragma unroll
    for (int q0 = 0; q0 < 512; q0 += NT) {
        const int q = q0 + tid;
        const double2 y = cmul(Y[q], T->mdct_post[q]);
        X[2 * q] = y.x * sc;
        X[1023 - 2 * q] = -y.y * sc;
    }
    grp_sync<NT>();
    return X;
}

// MDCT (mdct.py:49-82, N = 2048, 2/N in the forward transform) of the
// sine-windowed block xs(i) = x(i) * sine[i] (window.py:27-39, applied in
// place in codec.py:240): the DCT-IV of the folded block [a b c d] ->
// (-c_r - d, a - b_r), times 1/1024.  buf: 1024 double2 of LDS.  Output: the
// 1024 lines as doubles in the first 8 KB of buf (X = (double*)buf).  An
// exactly-zero line keeps the reference's sign (mdct_zero_neg).
template <int NT, class XS>
__device__ __forceinline__ double* grp_mdct(const XS& xs, const PacTables* __restrict__ T,
                                            double2* buf, int tid) {
    auto fold = [&](int n) {
        return n < 512 ? __dsub_rn(-xs(1535 - n), xs(1536 + n)) : __dsub_rn(xs(n - 512), xs(1535 - n));
    };
    double* X = grp_dct4<NT>(fold, T, buf, tid, 1.0 / 1024.0);
#pragma unroll
    for (int k0 = 0; k0 < 1024; k0 += NT) {
        const int k = k0 + tid;
        if (X[k] == 0.0) X[k] = T->mdct_zero_neg[k] ? -0.0 : 0.0;
    }
    grp_sync<NT>();
    return X;
}

// Two MDCTs at once (grp_mdct of channel 0 into bufA and of channel 1 into
// bufB, FFTs stage by stage together; xu(i, u) = windowed sample i of channel
// u): bit-identical to two grp_mdct calls.
template <int NT, class XU>
__device__ __forceinline__ void grp_mdct2(const XU& xu, const PacTables* __restrict__ T,
                                          double2* bufA, double2* bufB, int tid) {
    auto fold = [&](int n, int u) {
        if (n < 512) return __dsub_rn(-xu(1535 - n, u), xu(1536 + n, u));
        return __dsub_rn(xu(n - 512, u), xu(1535 - n, u));
    };
    double2 *Ya, *Yb;
    // staged by every thread for both channels (one load per sample; feeding
    // the first stage directly from global memory was slower here: each
    // thread of the split stages would load its own channel's samples, twice
    // the loads, and spilled)
#pragma unroll
    for (int q0 = 0; q0 < 512; q0 += NT) {
        const int q = q0 + tid;
        const double2 pq = T->mdct_pre[q];
        bufA[q] = cmul(make_double2(fold(2 * q, 0), fold(1023 - 2 * q, 0)), pq);
        bufB[q] = cmul(make_double2(fold(2 * q, 1), fold(1023 - 2 * q, 1)), pq);
    }
    grp_sync<NT>();
    grp_fft_stockham_x2_ld<9, NT>(bufA, bufA + 512, bufB, bufB + 512, T->fft_tw, tid,
                                  [&](int n, int u) { return (u ? bufB : bufA)[n]; }, &Ya, &Yb);
    double* XA = reinterpret_cast<double*>(bufA);
    double* XB = reinterpret_cast<double*>(bufB);
#pragma unroll
    for (int q0 = 0; q0 < 512; q0 += NT) {
        const int q = q0 + tid;
        const double2 ya = cmul(Ya[q], T->mdct_post[q]), yb = cmul(Yb[q], T->mdct_post[q]);
        XA[2 * q] = ya.x * (1.0 / 1024.0);
        XA[1023 - 2 * q] = -ya.y * (1.0 / 1024.0);
        XB[2 * q] = yb.x * (1.0 / 1024.0);
        XB[1023 - 2 * q] = -yb.y * (1.0 / 1024.0);
    }
    grp_sync<NT>();
#pragma unroll
    for (int k0 = 0; k0 < 1024; k0 += NT) {
        const int k = k0 + tid;
        if (XA[k] == 0.0) XA[k] = T->mdct_zero_neg[k] ? -0.0 : 0.0;
        if (XB[k] == 0.0) XB[k] = T->mdct_zero_neg[k] ? -0.0 : 0.0;
    }
    grp_sync<NT>();
}

// |FFT(d)[k]|^2, k < 1024, of a real 2048-sample block d(i) via a 1024-point
// complex Stockham FFT.  buf and tmp: 1024 double2 of LDS each; the input
// pairs are staged in buf, the FFT ends in tmp, and on return
// ((double*)buf)[k] = Re^2 + Im^2, dense (tmp is free again).  (findpeaks compares |X| and
// the masker SPL sums |X|^2 (psychoac.py:442-449); both only need the square.)
// (grp_spectrum_pow_pairs: the staged pairs come from dp(n) = (d(2n), d(2n+1)).)
template <int NT, class DP>
__device__ __forceinline__ void grp_spectrum_pow_pairs(const DP& dp, const PacTables* __restrict__ T,
                                                       double2* buf, double2* tmp, int tid) {
#pragma unroll 4
    for (int n0 = 0; n0 < 1024; n0 += NT) {
        const int n = n0 + tid;
        buf[n] = dp(n);
    }
    const double2* Z = grp_fft_stockham<10, NT>(buf, tmp, T->fft_tw, tid);   // = tmp
    // split: X[k] = (Z[k] + conj Z[M-k])/2 - i/2 W^k (Z[k] - conj Z[M-k]).
    // Pair p < 512 owns bins (p, 1024-p); pair 0 owns the self-paired bins 0 and 512.
#pragma unroll
    for (int p0 = 0; p0 < 512; p0 += NT) {
        const int p = p0 + tid;
        int kk[2];
        kk[0] = p;
        kk[1] = p ? 1024 - p : 512;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const double2 A = Z[kk[side]];
            const double2 Bc = Z[(1024 - kk[side]) & 1023];
            double2 e = make_double2(0.5 * (A.x + Bc.x), 0.5 * (A.y - Bc.y));
            double2 o = make_double2(0.5 * (A.x - Bc.x), 0.5 * (A.y + Bc.y));
            double2 wo = cmul(T->rfft_tw[kk[side]], o);
            double xr = e.x + wo.y;
            double xi = e.y - wo.x;
            reinterpret_cast<double*>(buf)[kk[side]] = __builtin_fma(xr, xr, xi * xi);
        }
    }
    grp_sync<NT>();
}
template <int NT, class DS>
__device__ __forceinline__ void grp_spectrum_pow(const DS& d, const PacTables* __restrict__ T,
                                                 double2* buf, double2* tmp, int tid) {
    grp_spectrum_pow_pairs<NT>([&](int n) { return make_double2(d(2 * n), d(2 * n + 1)); }, T, buf, tmp, tid);
}

// one-wave aliases used by the single-wave kernels
template <int LOG>
__device__ __forceinline__ void wave_fft(double2* buf, const double2* __restrict__ tw, int lane) {
    grp_fft<LOG, WAVE>(buf, tw, lane);
}
template <class XS>
__device__ __forceinline__ double* wave_mdct(const XS& xs, const PacTables* __restrict__ T,
                                             double2* buf, int lane) {
    return grp_mdct<WAVE>(xs, T, buf, lane);
}
template <class DS>
__device__ __forceinline__ void wave_spectrum_pow(const DS& d, const PacTables* __restrict__ T,
                                                  double2* buf, double2* tmp, int lane) {
    grp_spectrum_pow<WAVE>(d, T, buf, tmp, lane);
}

// ---------------------------------------------------------------------------
// masking threshold (psychoac.py:409-456)
// ---------------------------------------------------------------------------
//
// Per MDCT line l the reference adds, in ascending masker order from 0,
//   10^((SPL_m + spread_m(dz) - drop - 96) / 10),   dz = Bark(f_l) - Bark(f_m),
// spread (psychoac.py:111-116) = (0.367 max(SPL_m - 40, 0) [dz >= 0] - 27) (|dz| - 1/2) for |dz| > 1/2.
// In base 2 with B_m = (SPL_m - drop - 96) log2(10)/10 and the slopes
// KL = -27 log2(10)/10 (line below the masker), ku_m = (0.367 max(SPL_m-40,0) - 27) log2(10)/10
// (line above it), the maskers of line l split into three zones by the rank
// bounds U(l) = #{m : dz > 1/2}, V(l) = #{m : dz >= -1/2} (maskers are in
// ascending frequency):
//   flat   U <= m < V:  E_m = 2^B_m                 -> dd prefix sums, one difference per line
//   lower  m >= V:      2^(B_m + KL (z_m - 1/2)) * 2^(-KL z_l)   -> one suffix sum per threshold
//   upper  m < U:       2^(B_m + ku_m (z_l - z_m - 1/2))
//     quiet maskers (SPL_m <= 40: ku_m = KL exactly) factor the same way:
//                       2^(B_m - KL (z_m + 1/2)) * 2^(KL z_l)     -> one prefix sum per threshold
//     loud maskers (the rest) keep their own slopes: per 64-line row, a Taylor
//     series in the slope spread ("moment form") or the direct sum, over the
//     compacted list of loud maskers only.
// All terms are positive, so every regrouping above changes the result by a
// few ulp at most (no cancellation); exponents are evaluated in double-double.
#define PAC_LOG2_10_OVER_10 0.33219280948873624   // log2(10)/10
#define PAC_KL (-27.0 * PAC_LOG2_10_OVER_10)       // lower slope, and the slope of quiet maskers
#define PAC_LN2 0.6931471805599453
// order in which the 16 masking rows (64 lines each) are claimed by the waves
// of a threshold kernel, 4 bits per row, most expensive first (measured on
// broadband input: the middle rows carry the most maskers on both sides)
#define PAC_ROW_ORDER 0xf0e1dc4528b9a763ull
#define PAC_MOM_MIN 24      // fewest common loud maskers for the moment form
#define PAC_MOM_DMAX 40     // highest Taylor degree of the moment form
#define PAC_MOM_K 4         // maskers per lane held in registers by the moment form (per group)

// 2^(h + l) for a double-double exponent (|l| << ulp(h)): exp2(h) * (1 + l ln2)
__device__ __forceinline__ double pac_exp2_dd(double h, double l) {
    return pac_exp2(h) * __builtin_fma(l, PAC_LN2, 1.0);
}

// c + k * (a - b) as a double-double (TwoSum, TwoProduct via fma, TwoSum)
__device__ __forceinline__ void dd_affine(double c, double k, double a, double b, double& hi, double& lo) {
    double s = a - b;
    double bb = s - a;
    double err = (a - (s - bb)) + (-b - bb);
    double ph = k * s;
    double pl = __builtin_fma(k, s, -ph) + k * err;
    double t = c + ph;
    double cc = t - c;
    double e2 = (c - (t - cc)) + (ph - cc);
    hi = t;
    lo = e2 + pl;
}

__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
    s = a + b;
    const double bb = s - a;
    e = (a - (s - bb)) + (b - bb);
}
// (ah + al) + (bh + bl), renormalised
__device__ __forceinline__ void dd_add(double ah, double al, double bh, double bl, double& h, double& l) {
    double s, e;
    two_sum(ah, bh, s, e);
    e += al + bl;
    h = s + e;
    l = e - (h - s);
}

// The per-threshold masker lists in LDS.  Region A (16 KB, the spectrum's
// buffer once the maskers are extracted): four arrays of 512 doubles indexed
// by masker rank m = 0..nm (nm <= 511):
//   pfh/pfl  exclusive dd prefix of E_m            (flat zone)
//   sl       suffix sum from m of 2^(B + KL(z - 1/2))   (lower side; sl[nm] = 0)
//   su       exclusive prefix of 2^(B - KL(z + 1/2)) over quiet maskers (upper side)
// Region B (16 KB, the FFT scratch): the loud maskers' z, B, ku (12 KB; the
// peak-compaction scratch kidx lives in their first 2 KB until they are
// written), lpre[m] = #loud maskers of rank < m, a few counters, and
// rank[k] (k < 1024) = #maskers with bin < k -- so a threshold workgroup
// needs exactly the two 16 KB regions (5 workgroups per CU).
struct MaskerLists {
    double *pfh, *pfl, *sl, *su;
    double *lz, *lB, *lku;
    int16_t* lpre;
    int* misc;       // [0] row counter of the claiming loop, [1] loud count
    int* cnt;        // 32 ints: ballot segment counts
    int* kidx;       // 512 ints: compacted peak bins (aliases lz: dead before lz is written)
    int16_t* rank;
};
__device__ __forceinline__ MaskerLists masker_lists(void* regA, void* regB) {
    MaskerLists L;
    double* a = reinterpret_cast<double*>(regA);
    L.pfh = a;
    L.pfl = a + 512;
    L.sl = a + 1024;
    L.su = a + 1536;
    char* b = reinterpret_cast<char*>(regB);
    L.lz = reinterpret_cast<double*>(b);
    L.lB = reinterpret_cast<double*>(b + 4096);
    L.lku = reinterpret_cast<double*>(b + 8192);
    L.lpre = reinterpret_cast<int16_t*>(b + 12288);
    L.misc = reinterpret_cast<int*>(b + 13312);
    L.cnt = reinterpret_cast<int*>(b + 13312 + 64);
    L.kidx = reinterpret_cast<int*>(b);
    L.rank = reinterpret_cast<int16_t*>(b + 14336);
    return L;
}

// Physical slot of element m of the four prefix arrays (pfh, pfl, sl, su):
// bits 1-2 XOR bits 5-6.  The scans' lane owns 8 consecutive elements
// (m = 8 L + k), read and written as four 16-byte pairs; the pair of lane L
// at step c then lands in 16-byte bank slot 4 (L & 3) + (c ^ ((L >> 2) & 3)),
// distinct across every ds_read_b128 lane group (the plain layout is a 4-way
// conflict), while lane-consecutive accesses (the list writes) stay
// conflict-free and a row's gathers pay one XOR per index.
__device__ __forceinline__ int lsw(int m) { return m ^ (((m >> 5) & 3) << 1); }

// DPP scans across the 64 lanes (gfx9 row_shr / row_bcast / wave_shr; lanes
// without a source get the identity 0): inclusive prefix of a double, and of a
// double-double (hi, lo) pair
#define PAC_DPP_SHR(n) (0x110 + (n))
#define PAC_DPP_WSHR1 0x138     // wave_shr:1 (lane i <- lane i - 1)
#define PAC_DPP_WSHL1 0x130     // wave_shl:1 (lane i <- lane i + 1)
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ void scan_step(double& x) { x += dpp_f64<CTRL, RM>(0.0, x); }
__device__ __forceinline__ double wave_incl_scan_f64(double x) {
    scan_step<PAC_DPP_SHR(1)>(x);
    scan_step<PAC_DPP_SHR(2)>(x);
    scan_step<PAC_DPP_SHR(4)>(x);
    scan_step<PAC_DPP_SHR(8)>(x);
    scan_step<PAC_DPP_BCAST15, 0xa>(x);
    scan_step<PAC_DPP_BCAST31, 0xc>(x);
    return x;
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ void scan_step_dd(double& h, double& l) {
    const double yh = dpp_f64<CTRL, RM>(0.0, h), yl = dpp_f64<CTRL, RM>(0.0, l);
    dd_add(yh, yl, h, l, h, l);
}
__device__ __forceinline__ void wave_incl_scan_dd(double& h, double& l) {
    scan_step_dd<PAC_DPP_SHR(1)>(h, l);
    scan_step_dd<PAC_DPP_SHR(2)>(h, l);
    scan_step_dd<PAC_DPP_SHR(4)>(h, l);
    scan_step_dd<PAC_DPP_SHR(8)>(h, l);
    scan_step_dd<PAC_DPP_BCAST15, 0xa>(h, l);
    scan_step_dd<PAC_DPP_BCAST31, 0xc>(h, l);
}

// The three scans of the masker lists over m = 0..511 (elements zero at m >= nm),
// one wave each (lane j owns 8 consecutive elements: an in-lane running sum,
// a DPP scan of the lane totals, the lane's carry added back), no carries pass:
//   pfh/pfl: exclusive prefix of E as an unnormalised double-double (hi, sum of
//            the hi additions' rounding errors): |error| ~ n eps^2 of the prefix
//   su:      exclusive prefix; sl: inclusive suffix (lanes own the segments in
//            reverse order, so the lane scan runs downwards in m)
__device__ __forceinline__ void wave_scan_flat_dd(const MaskerLists& L, int lane) {
    const int m0 = 8 * lane, sw = ((lane >> 2) & 3) << 1;   // lsw(m0 + k) = m0 + (k ^ sw)
    double x[8], eh[8], el[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = L.pfh[m0 + (k ^ sw)];
    double rh = 0.0, rl = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        eh[k] = rh;
        el[k] = rl;
        double sx, e;
        two_sum(rh, x[k], sx, e);
        rh = sx;
        rl += e;
    }
    double th = rh, tl = rl;      // inclusive scan of the lane totals
    wave_incl_scan_dd(th, tl);
    const double ch = dpp_f64<PAC_DPP_WSHR1>(0.0, th), cl = dpp_f64<PAC_DPP_WSHR1>(0.0, tl);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        double sx, e;
        two_sum(ch, eh[k], sx, e);
        L.pfh[m0 + (k ^ sw)] = sx;
        L.pfl[m0 + (k ^ sw)] = (cl + el[k]) + e;
    }
}
__device__ __forceinline__ void wave_scan_excl8(double* v, int lane) {
    const int m0 = 8 * lane, sw = ((lane >> 2) & 3) << 1;
    double x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = v[m0 + (k ^ sw)];
    double run = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) { const double t = x[k]; x[k] = run; run += t; }
    const double c = dpp_f64<PAC_DPP_WSHR1>(0.0, wave_incl_scan_f64(run));
#pragma unroll
    for (int k = 0; k < 8; ++k) v[m0 + (k ^ sw)] = c + x[k];
}
__device__ __forceinline__ void wave_scan_suffix8(double* v, int lane) {
    const int bl = WAVE - 1 - lane;
    const int m0 = 8 * bl, sw = ((bl >> 2) & 3) << 1;
    double x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = v[m0 + (k ^ sw)];
    double run = 0.0;
#pragma unroll
    for (int k = 7; k >= 0; --k) { run += x[k]; x[k] = run; }
    const double c = dpp_f64<PAC_DPP_WSHR1>(0.0, wave_incl_scan_f64(run));
#pragma unroll
    for (int k = 0; k < 8; ++k) v[m0 + (k ^ sw)] = c + x[k];
}
template <int NT>
__device__ __forceinline__ void grp_scan_lists(const MaskerLists& L, int tid) {
    const int lane = tid & (WAVE - 1);
    if constexpr (NT >= 3 * WAVE) {
        const int w = tid / WAVE;
        if (w == 0) wave_scan_flat_dd(L, lane);
        else if (w == 1) wave_scan_suffix8(L.sl, lane);
        else if (w == 2) wave_scan_excl8(L.su, lane);
    } else {
        wave_scan_flat_dd(L, lane);
        wave_scan_suffix8(L.sl, lane);
        wave_scan_excl8(L.su, lane);
    }
    grp_sync<NT>();
}

// sum(|X[k-3:k+3]|^2) of a peak bin k (psychoac.py:448: Python slice
// semantics -- empty for k < 3, cut at the spectrum's end n -- and the builtin
// sum from 0 in bin order) as six independent LDS reads; a peak has k <= n-2,
// so only the sixth bin can fall past the end (it is read, in bounds of the
// caller's buffer, and not added)
__device__ __forceinline__ double slice6_sum(const double* pw, int k, int n) {
    if (k < 3) return 0.0;
    const double* q = pw + (k - 3);
    const double a = q[0], b = q[1], c = q[2], d = q[3], e = q[4], f = q[5];
    const double s = __dadd_rn(__dadd_rn(__dadd_rn(__dadd_rn(a, b), c), d), e);
    return k + 2 < n ? __dadd_rn(s, f) : s;
}

// Exclusive prefix of the A*NW segment counts c[i] (segment i = a * NW + w:
// bin-order chunks of the NW waves): lanes 0..A*NW-1 scan them by DPP row
// shifts inside one 16-lane row, and each wave reads its own A entries by
// readlane -- instead of every thread summing all of them serially.
template <int A, int NW>
__device__ __forceinline__ void seg_prefix(const int* c, int lane, int w, int (&out)[A], int* total) {
    static_assert(A * NW <= 16, "one DPP row");
    const int v = lane < A * NW ? c[lane] : 0;
    int s = v;
    s += __builtin_amdgcn_update_dpp(0, s, PAC_DPP_SHR(1), 0xf, 0xf, false);
    s += __builtin_amdgcn_update_dpp(0, s, PAC_DPP_SHR(2), 0xf, 0xf, false);
    s += __builtin_amdgcn_update_dpp(0, s, PAC_DPP_SHR(4), 0xf, 0xf, false);
    s += __builtin_amdgcn_update_dpp(0, s, PAC_DPP_SHR(8), 0xf, 0xf, false);
    const int ex = s - v;
    const int wu = __builtin_amdgcn_readfirstlane(w);
#pragma unroll
    for (int a = 0; a < A; ++a) out[a] = __builtin_amdgcn_readlane(ex, a * NW + wu);
    *total = __builtin_amdgcn_readlane(s, 15);
}

// findpeaks (psychoac.py:158-191) on |X|^2 held in pw[k] (the floor
// 10 log10|X| > -30 is the equivalent |X|^2 > T->peak_floor2), masker SPL from the
// 6-bin slice X[k-3:k+3] (psychoac.py:448, Python slice semantics), then the
// masker lists (MaskerLists) built by a group of NT threads.  Peaks are
// compacted first (ballots, bin order = the reference's summation order) so
// that the SPL (a log10 each) is evaluated once per masker.  Returns nm.
template <int NT>
__device__ __forceinline__ int grp_find_maskers(const double* pw, const PacTables* __restrict__ T, double drop,
                                                int tid, const MaskerLists& L) {
    constexpr int J = 1024 / NT;
    constexpr int NW = NT / WAVE;
    int* cnt = L.cnt;                // [J][NW] peak counts of the (j, wave) segments, in bin order
    int* kidx = L.kidx;
    const int lane = tid & (WAVE - 1);
    const int w = tid / WAVE;
    const double floor2 = T->peak_floor2;
    unsigned long long bal[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int k = j * NT + tid;
        bool pk = false;
        if (k >= 1 && k <= 1022) {
            const double m = pw[k];
            pk = m > pw[k - 1] && m > pw[k + 1] && m > floor2;
        }
        bal[j] = __ballot(pk);
        if (lane == 0) cnt[j * NW + w] = __popcll(bal[j]);
    }
    grp_sync<NT>();
    int tot;
    int pj[J];                       // exclusive prefix of this wave's segment counts
    seg_prefix<J, NW>(cnt, lane, w, pj, &tot);
    const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int idx = pj[j] + __popcll(bal[j] & below);
        L.rank[j * NT + tid] = (int16_t)idx;
        if ((bal[j] >> lane) & 1ull) kidx[idx] = j * NT + tid;
    }
    grp_sync<NT>();
    tot = __builtin_amdgcn_readfirstlane(tot);
    constexpr int R = (PAC_MAXMASK + NT - 1) / NT;
    double rz[R], rB[R], rku[R], rE[R], rPL[R], rPU[R];
    unsigned long long lb[R];
    int* cnt2 = cnt + 16;            // [R][NW] loud counts
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int idx = q * NT + tid;
        bool loud = false;
        rz[q] = rB[q] = rku[q] = rE[q] = rPL[q] = rPU[q] = 0.0;
        if (idx < tot) {
            const int k = kidx[idx];
            // the masker's table entries first, unconditionally: their global
            // latency then overlaps the SPL's log10 (a pow_pu load under the
            // loud test was issued after it and waited on at once)
            const double tz = T->bark_bin[k], tpl = T->pow_pl[k], tpu = T->pow_pu[k];
            const double s = slice6_sum(pw, k, 1024);
            const double csp = 8.0 / 3.0 * 4.0 / (2048.0 * 2048.0);
            const double sp = pac_spl(csp * s);
            double lev = sp - 40.0;
            lev = 0.367 * (0.0 > lev ? 0.0 : lev);       // builtin max(SPL-40, 0)
            loud = lev != 0.0;                            // else ku == KL exactly
            rB[q] = (sp - drop - 96.0) * PAC_LOG2_10_OVER_10;
            rz[q] = tz;
            rku[q] = (lev - 27.0) * PAC_LOG2_10_OVER_10;
            rE[q] = pac_exp2(rB[q]);
            rPL[q] = rE[q] * tpl;                          // 2^(B + KL (z - 1/2))
            if (!loud) rPU[q] = rE[q] * tpu;               // 2^(B - KL (z + 1/2))
        }
        lb[q] = __ballot(loud);
        if (lane == 0) cnt2[q * NW + w] = __popcll(lb[q]);
    }
    grp_sync<NT>();   // every |X|^2 read done before the lists overwrite buf; loud counts visible
    int nloud;
    int pq[R];                       // exclusive prefix of this wave's loud counts
    seg_prefix<R, NW>(cnt2, lane, w, pq, &nloud);
#pragma unroll
    for (int q = 0; q < R; ++q) {           // R * NT = 512: every slot, zero past nm
        const int idx = q * NT + tid;
        const int pi = lsw(idx);
        L.pfh[pi] = rE[q];
        L.sl[pi] = rPL[q];
        L.su[pi] = rPU[q];
        if (idx < tot) {
            const int j = pq[q] + __popcll(lb[q] & below);
            L.lpre[idx] = (int16_t)j;
            if ((lb[q] >> lane) & 1ull) { L.lz[j] = rz[q]; L.lB[j] = rB[q]; L.lku[j] = rku[q]; }
        }
    }
    // the rows' claiming counter (misc[0]) reset here: visible after the scans'
    // barrier, so the caller's row loop needs no barrier of its own
    if (tid == 0) { L.lpre[tot] = (int16_t)nloud; L.misc[1] = nloud; L.misc[0] = 0; }
    grp_sync<NT>();
    grp_scan_lists<NT>(L, tid);
    return tot;
}

// wave-uniform results, returned in scalar registers (uniform loop bounds);
// DPP reductions as wave_sum_i (no LDS round trip)
template <bool MAX>
__device__ __forceinline__ int wave_ext_i(int v) {
    auto f = [](int a, int b) { return MAX ? (a > b ? a : b) : (a < b ? a : b); };
    v = f(v, __builtin_amdgcn_update_dpp(v, v, PAC_DPP_QXOR1, 0xf, 0xf, false));
    v = f(v, __builtin_amdgcn_update_dpp(v, v, PAC_DPP_QXOR2, 0xf, 0xf, false));
    v = f(v, __builtin_amdgcn_update_dpp(v, v, PAC_DPP_HMIRROR, 0xf, 0xf, false));
    v = f(v, __builtin_amdgcn_update_dpp(v, v, PAC_DPP_MIRROR, 0xf, 0xf, false));
    v = f(v, __builtin_amdgcn_update_dpp(v, v, PAC_DPP_BCAST15, 0xa, 0xf, false));
    v = f(v, __builtin_amdgcn_update_dpp(v, v, PAC_DPP_BCAST31, 0xc, 0xf, false));
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_or_i(int v) {
    v |= __builtin_amdgcn_update_dpp(0, v, PAC_DPP_QXOR1, 0xf, 0xf, false);
    v |= __builtin_amdgcn_update_dpp(0, v, PAC_DPP_QXOR2, 0xf, 0xf, false);
    v |= __builtin_amdgcn_update_dpp(0, v, PAC_DPP_HMIRROR, 0xf, 0xf, false);
    v |= __builtin_amdgcn_update_dpp(0, v, PAC_DPP_MIRROR, 0xf, 0xf, false);
    v |= __builtin_amdgcn_update_dpp(0, v, PAC_DPP_BCAST15, 0xa, 0xf, false);
    v |= __builtin_amdgcn_update_dpp(0, v, PAC_DPP_BCAST31, 0xc, 0xf, false);
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_min_i(int v) { return wave_ext_i<false>(v); }
__device__ __forceinline__ int wave_max_i(int v) { return wave_ext_i<true>(v); }

// v_min_f64 / v_max_f64 without the canonicalising v_max_f64 x, x the compiler
// adds around fmin/fmax in IEEE mode (the operands are never NaN)
__device__ __forceinline__ double vmin_f64(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double vmax_f64(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// Wave extremum read from lane 0: four full-row DPP steps (bound_ctrl, every
// lane has a source), then rows 0|1 and 2|3 by v_permlane16_swap and the
// halves by v_permlane32_swap -- 3 VALU per step instead of the
// compare-select and row_bcast copies of wave_ext_f64.
template <bool MAX>
__device__ __forceinline__ double wave_ext0_f64(double v) {
    auto f = [](double a, double b) { return MAX ? vmax_f64(a, b) : vmin_f64(a, b); };
    v = f(v, dpp_full_f64<PAC_DPP_QXOR1>(v));
    v = f(v, dpp_full_f64<PAC_DPP_QXOR2>(v));
    v = f(v, dpp_full_f64<PAC_DPP_HMIRROR>(v));
    v = f(v, dpp_full_f64<PAC_DPP_MIRROR>(v));
    {
        const long long b = __double_as_longlong(v);
        const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
        const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
        v = f(__longlong_as_double(((long long)hi[0] << 32) | (long long)lo[0]),
              __longlong_as_double(((long long)hi[1] << 32) | (long long)lo[1]));
    }
    {
        const long long b = __double_as_longlong(v);
        const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
        v = f(__longlong_as_double(((long long)hi[0] << 32) | (long long)lo[0]),
              __longlong_as_double(((long long)hi[1] << 32) | (long long)lo[1]));
    }
    return readlane_f64(v, 0);
}
// wave maximum of non-NaN doubles, wave-uniform (DPP + permlane swaps, no
// ds_bpermute round trips)
__device__ __forceinline__ double wave_max(double v) { return wave_ext0_f64<true>(v); }
// integer minimum, the same shape (DPP steps fold into v_min_i32_dpp)
__device__ __forceinline__ int wave_min0_i(int v) {
    v = min(v, __builtin_amdgcn_mov_dpp(v, PAC_DPP_QXOR1, 0xf, 0xf, true));
    v = min(v, __builtin_amdgcn_mov_dpp(v, PAC_DPP_QXOR2, 0xf, 0xf, true));
    v = min(v, __builtin_amdgcn_mov_dpp(v, PAC_DPP_HMIRROR, 0xf, 0xf, true));
    v = min(v, __builtin_amdgcn_mov_dpp(v, PAC_DPP_MIRROR, 0xf, 0xf, true));
    const auto p = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    v = min((int)p[0], (int)p[1]);
    const auto q = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    v = min((int)q[0], (int)q[1]);
    return __builtin_amdgcn_readlane(v, 0);
}

// diagnostic build (-DPAC_ROWPROF): cycle and size counters of the masking rows
#ifdef PAC_ROWPROF
__device__ unsigned long long pac_rowprof[1024 * 16];   // spread over 1024 lines: no hot address
#define RP_T(v) long long v = (long long)__builtin_amdgcn_s_memtime()
#define RP_ADD(i_, v_) do { if (lane == 0) atomicAdd(&pac_rowprof[(blockIdx.x & 1023) * 16 + (i_)], (unsigned long long)(v_)); } while (0)
#else
#define RP_T(v) do {} while (0)
#define RP_ADD(i_, v_) do {} while (0)
#endif

// Sum over the wave of 4 per-lane doubles v[0..3] at once (a reduce-scatter:
// each step halves the values a lane carries, exchanging the other half with
// its partner lane -- v_permlane32_swap / v_permlane16_swap for lane bits 5
// and 4 -- then a DPP sum over the row of 16 lanes that holds each index),
// ~2.7x fewer VALU instructions than 4 wave sums.  S[t] = sum_lanes v[t],
// wave-uniform (scalar registers).  Pairwise tree order.
#define PAC_DPP_ROR8 0x128     // row_ror:8 (lane i <- lane i ^ 8 within a row)
__device__ __forceinline__ void dswap32(double& a, double& b) {
    const long long ia = __double_as_longlong(a), ib = __double_as_longlong(b);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ia, (unsigned)ib, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ia >> 32), (unsigned)(ib >> 32), false, false);
    a = __longlong_as_double(((long long)hi[0] << 32) | (long long)lo[0]);
    b = __longlong_as_double(((long long)hi[1] << 32) | (long long)lo[1]);
}
__device__ __forceinline__ void dswap16(double& a, double& b) {
    const long long ia = __double_as_longlong(a), ib = __double_as_longlong(b);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ia, (unsigned)ib, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ia >> 32), (unsigned)(ib >> 32), false, false);
    a = __longlong_as_double(((long long)hi[0] << 32) | (long long)lo[0]);
    b = __longlong_as_double(((long long)hi[1] << 32) | (long long)lo[1]);
}
__device__ __forceinline__ void wave_sum4_f64(double (&v)[4], double (&S)[4]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {          // bit 5: lanes 0-31 keep index k, lanes 32-63 index k + 2
        double a = v[k], b = v[k + 2];
        dswap32(a, b);
        v[k] = a + b;
    }
    {                                      // bit 4: rows 0, 2 keep index 0, rows 1, 3 index 1
        double a = v[0], b = v[1];
        dswap16(a, b);
        v[0] = a + b;
    }
    // index 2 b5 + b4 (= lane >> 4): the sum over the row of 16 lanes holding it
    v[0] += dpp_full_f64<PAC_DPP_ROR8>(v[0]);
    v[0] += dpp_full_f64<PAC_DPP_HMIRROR>(v[0]);
    v[0] += dpp_full_f64<PAC_DPP_QXOR1>(v[0]);
    v[0] += dpp_full_f64<PAC_DPP_QXOR2>(v[0]);
#pragma unroll
    for (int t = 0; t < 4; ++t) S[t] = readlane_f64(v[0], 16 * t);
}

// One group of the moment form: KK loud maskers per lane (ranks g0 + 64 k +
// lane < ua), sum_d q_d(l) S_d with q_d = x^d / d! (per line) and the moments
// S_d = sum_m 2^beta_m (ku_m - kc)^d (wave sums, four degrees at a time).
template <int KK>
__device__ __forceinline__ double mom_group(const MaskerLists& L, const PacTables* __restrict__ T, int g0, int ua,
                                            int lane, double zm, double kc, double x, int D) {
    double pk[KK], ck[KK];
#pragma unroll
    for (int k = 0; k < KK; ++k) {
        const int m = g0 + k * WAVE + lane;
        pk[k] = 0.0;
        ck[k] = 0.0;
        if (m < ua) {
            const double ku = L.lku[m];
            pk[k] = pac_exp2_v(__builtin_fma((zm - L.lz[m]) - 0.5, ku, L.lB[m]));
            ck[k] = ku - kc;
        }
    }
    double acc = 0.0, q = 1.0;
    for (int d0 = 0; d0 <= D; d0 += 4) {
        double v[4], S[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            double part = pk[0];
#pragma unroll
            for (int k = 1; k < KK; ++k) part += pk[k];
            v[t] = part;
#pragma unroll
            for (int k = 0; k < KK; ++k) pk[k] *= ck[k];
        }
        wave_sum4_f64(v, S);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            if (d0 + t > D) break;          // wave-uniform
            acc = __builtin_fma(S[t], q, acc);
            q = (q * x) * T->inv_int[d0 + t + 1];
        }
    }
    return acc;
}

// Masking threshold of MDCT row r (lines l = 64 r + lane) by one wave from the
// masker lists, as the intensity I(l) + Intensity(Thresh(f_l)) whose SPL()
// is the reference's threshold (the SMRs take it as an intensity,
// pac_spl_ratio).
//
// PRUNE (an MLD variant's row, k_master_thr mode 1): the row is only needed
// where its MLD threshold could fall below the M/S threshold it is min-ed with
// (psychoac.py:582-591: THR_S = max(BTHR_S, min(BTHR_M, MLD_M)) and
// symmetrically), i.e. on lines with ref_hi > ref_lo (hi = BTHR_M, lo = BTHR_S
// for MLD_M) where MLD < ref_hi.  The flat, lower and quiet-upper zones plus
// the threshold in quiet are a lower bound of the row's intensity (the loud
// upper-side terms are positive and added first, and rounding to nearest is
// monotone), and the MLD intensity is nondecreasing in it; if on every such
// line the bound's MLD intensity already exceeds ref_hi by a 2^-40 margin
// (far beyond the polynomials' few-ulp non-monotonicity), min(ref_hi, MLD) is
// ref_hi whatever the rest of the sum, and the row returns -1 (not needed:
// the front's +inf gives the same combination).  On the bench signal 12 of
// the ~14 MLD_M rows of a block end here, before the loud-masker sums.
// The decision is returned in *gone as a scalar (readfirstlane of the ballot),
// so that the caller's skip is an SCC branch: a per-lane test of the returned
// value would put the caller's skip / continue under an exec mask around the
// next row's full-wave ballots and DPP (the shape of the round-5 hang).
#define PAC_PRUNE_MARGIN 1.0000000000009095      // 1 + 2^-40
template <bool PRUNE = false>
__device__ __forceinline__ double wave_masking_row(const MaskerLists& L, int nm, const PacTables* __restrict__ T,
                                                   int lane, int r, double ref_hi = 0.0, double ref_lo = 0.0,
                                                   int* gone = nullptr) {
    const int l = r * WAVE + lane;
    const double zl = T->bark_line[l];
    const double zr = T->bark_line[r * WAVE];           // smallest z of the row
    const double zt = T->bark_line[r * WAVE + WAVE - 1];
    const int U = L.rank[T->mask_ku[l]];
    const int V = L.rank[T->mask_kv[l]];
    RP_T(t0);
    // flat zone [U, V): difference of the dd prefix sums (positive terms)
    double fs, fe;
    const int pV = lsw(V), pU = lsw(U);
    two_sum(L.pfh[pV], -L.pfh[pU], fs, fe);
    const double flat = fs + (fe + (L.pfl[pV] - L.pfl[pU]));
    // lower side and the quiet maskers of the upper side: factored sums
    const double lower = L.sl[pV] * T->pow_mkl[l];
    const double upq = L.su[pU] * T->pow_kl[l];
    const double tiq = T->tiq[l];
    if constexpr (PRUNE) {
        const double lb = ((upq + flat) + lower) + tiq;
        const bool need = ref_hi > ref_lo && !(pac_mld_intensity(lb, T->mld[l]) > ref_hi * PAC_PRUNE_MARGIN);
        const int none = __builtin_amdgcn_readfirstlane(__ballot(need) == 0ull ? 1 : 0);
        *gone = none;
        if (none) return 0.0;                          // scalar: the row is not needed
    }
    RP_T(t1);
    // loud maskers below the line: loud-list ranks [0, Ul)
    const int Ul = L.lpre[U];
    // U(l) is nondecreasing in l (mask_ku is a two-pointer sweep over the
    // ascending bark_line; rank and lpre are prefix counts): the row's
    // extremes are lanes 0 and 63
    const int umin = __builtin_amdgcn_readlane(Ul, 0), umax = __builtin_amdgcn_readlane(Ul, WAVE - 1);
    double up = 0.0;
    int m0 = umax, ua = umax;
    bool direct = true;
    int D = -1;
    if (umax > 0) {
        // I(l) >= lb = min over the row of ((upq + flat) + lower) + tiq; the cut is
        // floor(log2 lb) - 64 from the exponent field (conservative).  frexp_exp is
        // nondecreasing on positive doubles, so the minimum exponent is lb's.
        const int elb = wave_min0_i(__builtin_amdgcn_frexp_exp(((upq + flat) + lower) + tiq));
        const double l2cut = (double)(elb - 65);
        for (int base = 0; base < umax; base += WAVE) {   // first loud masker that is not negligible
            const int m = base + lane;
            int keep = 1;
            if (m < umax) {
                const double ku = L.lku[m];
                const double t = __builtin_fma(fmax((zr - L.lz[m]) - 0.5, 0.0), ku, L.lB[m]);
                keep = !(ku < 0.0 && t < l2cut);
            }
            const unsigned long long kb = __ballot(keep);
            if (kb) { m0 = base + __builtin_ctzll(kb); break; }
        }
        m0 = __builtin_amdgcn_readfirstlane(m0 < umax ? m0 : umax);
    }
    RP_T(t2);
    // exponents relative to the row middle: 2^(beta_m + ku_m (z_l - z_mid)),
    // beta_m = B_m + ku_m ((z_mid - z_m) - 1/2)
    const double zm = 0.5 * (zr + zt);
    const double dl = zl - zm;
    ua = umin > m0 ? (umin < umax ? umin : umax) : m0;
    // Loud maskers [m0, ua) lie below every line of the row.  Their sum factors as
    //   2^(kc dl) * sum_d (dl ln2)^d / d! * S_d,   S_d = sum_m 2^beta_m (ku_m - kc)^d,
    // kc the middle of their slopes: the Taylor series of 2^((ku_m - kc) dl),
    // truncated where its remainder is below 2^-57 of every term.
    if (ua - m0 >= PAC_MOM_MIN) {
        double kmn = INFINITY, kmx = -INFINITY;
        for (int m = m0 + lane; m < ua; m += WAVE) {
            const double k = L.lku[m];
            kmn = vmin_f64(kmn, k);
            kmx = vmax_f64(kmx, k);
        }
        kmn = wave_ext0_f64<false>(kmn);
        kmx = wave_ext0_f64<true>(kmx);
        const double adl = fmax(zm - zr, zt - zm);       // max |z_l - z_mid| over the row
        const double kc = 0.5 * (kmn + kmx);
        const double eps = (0.5 * (kmx - kmn) * adl) * PAC_LN2 * 1.0000001;
        // smallest D with e^eps eps^(D+1)/(D+1)! <= 2^-57 (uniform): lane j tests
        // eps against its bound; PAC_MOM_DMAX + 1 (no moment form) past the table
        const unsigned long long ok = __ballot(eps <= T->mom_eps[lane]);
        D = ok ? (int)__builtin_ctzll(ok) : PAC_MOM_DMAX + 1;
        if (D <= PAC_MOM_DMAX) {
            direct = false;
            const double x = dl * PAC_LN2;
            double acc = 0.0;
            // the sum is linear in the moments: groups of up to PAC_MOM_K maskers per lane
            for (int g0 = m0; g0 < ua; g0 += PAC_MOM_K * WAVE) {
                const int K = (ua - g0 + WAVE - 1) / WAVE;       // wave-uniform
                if (K == 1) acc += mom_group<1>(L, T, g0, ua, lane, zm, kc, x, D);
                else if (K == 2) acc += mom_group<2>(L, T, g0, ua, lane, zm, kc, x, D);
                else if (K == 3) acc += mom_group<3>(L, T, g0, ua, lane, zm, kc, x, D);
                else acc += mom_group<4>(L, T, g0, ua, lane, zm, kc, x, D);
            }
            up = acc * pac_exp2_v(kc * dl);
        }
    }
    RP_T(t3);
    // the direct terms in the line's own form, B_m + ku_m ((z_l - z_m) - 1/2) --
    // the reference's (|dz| - 1/2) slope product (psychoac.py:111-116) -- one
    // fused multiply-add fewer than the row-middle form the moment form needs
    if (direct) {
#pragma unroll 2
        for (int m = m0; m < ua; ++m)               // m < umin <= Ul on every lane
            up += pac_exp2_v(__builtin_fma((zl - L.lz[m]) - 0.5, L.lku[m], L.lB[m]));
    }
#pragma unroll 2
    for (int m = ua; m < umax; ++m) {
        const double t = pac_exp2_v(__builtin_fma((zl - L.lz[m]) - 0.5, L.lku[m], L.lB[m]));
        up += (m < Ul) ? t : 0.0;
    }
    RP_T(t4);
#ifdef PAC_ROWPROF
    RP_ADD(0, 1); RP_ADD(1, t1 - t0); RP_ADD(2, t2 - t1); RP_ADD(3, t3 - t2); RP_ADD(4, t4 - t3);
    RP_ADD(5, nm); RP_ADD(6, L.misc[1]); RP_ADD(7, direct ? 0 : 1); RP_ADD(8, direct ? 0 : D);
    RP_ADD(9, ua - m0); RP_ADD(10, umax - ua); RP_ADD(11, m0); RP_ADD(12, umax);
#endif
    return (((up + upq) + flat) + lower) + tiq;      // the intensity; SPL() by the caller where needed
}
