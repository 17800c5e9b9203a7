// pac_bs.h -- block switching: an EXTENSION, not in the
// reference (pacfile.py:23,48 has no block switching), so parity is unpinned;
// the HIP path is checked against oracle/pac_oracle.c's restatement of this
// design:
//   - every frame still takes one 1024-sample hop.  A frame is LONG (one
//     N = 2048 MDCT, mdct.py a = b = 1024) or SHORT (four N = 512 MDCTs at
//     buffer offsets 384 + 256 k, mdct.py a = b = 256).  The short spectra are
//     interleaved (line 4 j + k = line j of block k), so the 25-band layout, bit
//     allocation, quantizer, Huffman and bitstream are the long ones;
//   - a long frame next to a short one takes the short window's slope over
//     the short blocks' overlap and 0 / 1 outside it (start / stop shapes);
//   - attack: first-difference energy of a 128-sample segment of the frame's
//     new half > PAC_BS_RATIO x the mean of the 8 segments before it and
//     > PAC_BS_EMIN; a frame is short when it or the frame before has one;
//   - the masking model of a short block is calcBTHR (psychoac.py:409-456) at
//     N = 512, evaluated per short block and interleaved like the lines;
//   - one bit after the LRMS bits marks a short frame (master profile only).
#pragma once
#include "pac_wave.h"

#define PAC_BS_SHORT 1
#define PAC_BS_PREV 2
#define PAC_BS_NEXT 4
#define PAC_BS_RATIO 10.0
#define PAC_BS_EMIN 1e-3
#define PAC_NS 512
#define PAC_HALFS 256

// MDCT window of a long frame with block-switching flags fl: the long window,
// with the short window's slope (and 0 / 1) on a side whose neighbour is short
__device__ __forceinline__ double bs_long_win(const PacTables* __restrict__ T, int fl, int n) {
    if (n < PAC_HALFN) {
        if (!(fl & PAC_BS_PREV)) return T->sine[n];
        return n < 384 ? 0.0 : (n < 640 ? T->sine_s[n - 384] : 1.0);
    }
    if (!(fl & PAC_BS_NEXT)) return T->sine[n];
    return n < 1408 ? 1.0 : (n < 1664 ? T->sine_s[n - 1152] : 0.0);
}

// DCT-IV of 256 values v(j) by one wave, scaled by sc:
//   X[k] = sc * sum_j v(j) cos(pi/256 (j + 1/2)(k + 1/2)),
// via the 128-point Stockham FFT (the 1024-line grp_dct4 at M = 256).
// scr: 256 double2 of LDS private to the wave; out(k, X[k]) receives the lines.
template <bool SWZ = true, class V, class OUT>
__device__ __forceinline__ void wave_dct4_256(const V& v, const PacTables* __restrict__ T, double2* scr, int lane,
                                              double sc, const OUT& out) {
#pragma unroll
    for (int q0 = 0; q0 < 128; q0 += WAVE) {
        const int q = q0 + lane;
        scr[q] = cmul(make_double2(v(2 * q), v(255 - 2 * q)), T->mdct_pre_s[q]);
    }
    const double2* Y = grp_fft_stockham<7, WAVE, SWZ>(scr, scr + 128, T->fft_tw, lane);
#pragma unroll
    for (int q0 = 0; q0 < 128; q0 += WAVE) {
        const int q = q0 + lane;
        const double2 y = cmul(Y[q], T->mdct_post_s[q]);
        out(2 * q, y.x * sc);
        out(255 - 2 * q, -y.y * sc);
    }
    wave_sync();
}

// MDCT (mdct.py:49-82, N = 512, 2/N forward) of short block k of a frame,
// xs(i) = x(384 + 256 k + i) * sine_s[i], by one wave; line j goes to
// X[4 j + k] (interleaved).  An exactly-zero line is +0.0 (the oracle's
// convention for this extension).
template <class XR>
__device__ __forceinline__ void wave_short_mdct(const XR& x, const PacTables* __restrict__ T, int k, double2* scr,
                                                double* X, int lane) {
    const int o = 384 + 256 * k;
    auto xs = [&](int i) { return __dmul_rn(x(o + i), T->sine_s[i]); };
    auto fold = [&](int n) {
        return n < 128 ? __dsub_rn(-xs(383 - n), xs(384 + n)) : __dsub_rn(xs(n - 128), xs(383 - n));
    };
    wave_dct4_256(fold, T, scr, lane, 1.0 / 256.0, [&](int j, double v) { X[4 * j + k] = v == 0.0 ? 0.0 : v; });
}

// the four short MDCTs of a frame by the four waves of a 256-thread
// workgroup (wave k: block k), scratch: 256 double2 per wave
template <class XR>
__device__ __forceinline__ void grp_short_mdct(const XR& x, const PacTables* __restrict__ T, double2* scr0,
                                               double2* scr1, double* X, int tid) {
    const int k = tid / WAVE;
    double2* scr = (k < 2 ? scr0 : scr1) + 256 * (k & 1);
    wave_short_mdct(x, T, k, scr, X, tid & (WAVE - 1));
    __syncthreads();
}

// |FFT(d)[k]|^2, k < 256, of a real 512-sample short block d(i) by one wave:
// 256-point complex Stockham FFT of the sample pairs + the real split
// (twiddles exp(-2 pi i k / 512) = rfft_tw[4 k]).  buf, tmp: 256 double2 each;
// on return pw[k] holds the powers (pw may alias tmp: the FFT ends in buf).
template <class DS>
__device__ __forceinline__ void wave_spectrum_pow_short(const DS& d, const PacTables* __restrict__ T, double2* buf,
                                                        double2* tmp, double* pw, int lane) {
#pragma unroll
    for (int n0 = 0; n0 < 256; n0 += WAVE) {
        const int n = n0 + lane;
        buf[n] = make_double2(d(2 * n), d(2 * n + 1));
    }
    const double2* Z = grp_fft_stockham<8, WAVE>(buf, tmp, T->fft_tw, lane);
#pragma unroll
    for (int p0 = 0; p0 < 128; p0 += WAVE) {
        const int p = p0 + lane;
        int kk[2];
        kk[0] = p;
        kk[1] = p ? 256 - p : 128;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const double2 A = Z[kk[side]];
            const double2 Bc = Z[(256 - kk[side]) & 255];
            const double2 e = make_double2(0.5 * (A.x + Bc.x), 0.5 * (A.y - Bc.y));
            const double2 o = make_double2(0.5 * (A.x - Bc.x), 0.5 * (A.y + Bc.y));
            const double2 wo = cmul(T->rfft_tw[4 * kk[side]], o);
            const double xr = e.x + wo.y, xi = e.y - wo.x;
            pw[kk[side]] = __builtin_fma(xr, xr, xi * xi);
        }
    }
    wave_sync();
}

// exclusive prefix over the wave of per-lane pairs (elements 2 lane, 2 lane + 1)
__device__ __forceinline__ void wave_excl_scan2(double a, double b, double* e0, double* e1) {
    const double inc = wave_incl_scan_f64(a + b);
    const double before = dpp_f64<PAC_DPP_WSHR1>(0.0, inc);     // the previous lanes' sum
    *e0 = before;
    *e1 = before + a;
}

// calcBTHR (psychoac.py:409-456) of a short block at N = 512 by one wave, from
// the powers pw[256]: findpeaks (psychoac.py:158-191, the same floor and BW
// slice as the long model), masker SPL, then per line the masking sum of
// psychoac.py:111-116,447-456 split by the rank bounds U(l) = #{dz > 1/2},
// V(l) = #{dz >= -1/2} (maskers ascend in frequency) as in pac_wave.h:
//   flat  U <= m < V:  2^B_m                        (direct, few maskers)
//   lower m >= V:      2^(-KL z_l) * suffix sum of 2^(B_m + KL (z_m - 1/2))
//   upper m < U, quiet (SPL <= 40: slope KL exactly):
//                      2^(KL z_l) * prefix sum of 2^(B_m - KL (z_m + 1/2))
//   upper m < U, loud: 2^(B_m + ku_m (z_l - z_m - 1/2)) directly
// All terms are positive: the regrouping moves the sum by a few ulp.  Then +
// threshold in quiet, as an intensity.  R: the wave's 8 KB of LDS, pw at R + 4096 (2 KB).
// out(l, thr) for l < 256 in the 64-line rows whose bit is set in `rows`.
template <class OUT>
__device__ __forceinline__ void wave_threshold_short(char* R, const PacTables* __restrict__ T, double drop, int lane,
                                                     int rows, const OUT& out) {
    const double* pw = reinterpret_cast<const double*>(R + 4096);
    int* kidx = reinterpret_cast<int*>(R + 3584);
    const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
    int nm = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int k = q * WAVE + lane;
        bool pk = false;
        if (k >= 1 && k <= 254) {
            const double m = pw[k];
            pk = m > pw[k - 1] && m > pw[k + 1] && m > T->peak_floor2;
        }
        const unsigned long long bal = __ballot(pk);
        if (pk) kidx[nm + __popcll(bal & below)] = k;
        nm += __popcll(bal);
    }
    wave_sync();
    // per masker m = lane, 64 + lane: level, position and the factored terms,
    // in registers until every read of pw / kidx is done
    const double csp = 8.0 / 3.0 * 4.0 / (512.0 * 512.0);
    double z[2], B[2], ku[2], E[2], P[2], Q[2];
    bool loud[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int m = h * WAVE + lane;
        loud[h] = false;
        z[h] = B[h] = ku[h] = E[h] = P[h] = Q[h] = 0.0;
        if (m < nm) {
            const int k = kidx[m];
            const double s = slice6_sum(pw, k, 256);
            const double sp = pac_spl(csp * s);
            double lev = sp - 40.0;
            lev = 0.367 * (0.0 > lev ? 0.0 : lev);
            loud[h] = lev != 0.0;
            z[h] = T->bark_bin_s[k];
            B[h] = (sp - drop - 96.0) * PAC_LOG2_10_OVER_10;
            ku[h] = (lev - 27.0) * PAC_LOG2_10_OVER_10;
            E[h] = pac_exp2(B[h]);
            double hh, lo;
            dd_affine(B[h], PAC_KL, z[h], 0.5, hh, lo);          // B + KL (z - 1/2)
            P[h] = pac_exp2_dd(hh, lo);
            if (!loud[h]) {
                dd_affine(B[h], PAC_KL, -0.5, z[h], hh, lo);     // B - KL (z + 1/2)
                Q[h] = pac_exp2_dd(hh, lo);
            }
        }
    }
    wave_sync();
    double* Lz = reinterpret_cast<double*>(R);            // [128] masker Bark positions
    double* LE = reinterpret_cast<double*>(R + 1024);     // [128] 2^B
    double* LP = reinterpret_cast<double*>(R + 2048);     // [128] suffix sums of P (P then)
    double* LQ = reinterpret_cast<double*>(R + 3080);     // [128] exclusive prefix sums of Q (Q then)
    double* lz = reinterpret_cast<double*>(R + 4104);     // loud maskers: z, B, ku
    double* lB = reinterpret_cast<double*>(R + 5128);
    double* lku = reinterpret_cast<double*>(R + 6152);
    int16_t* lpre = reinterpret_cast<int16_t*>(R + 7176); // [129] #loud maskers below m
    int nloud = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int m = h * WAVE + lane;
        Lz[m] = z[h];
        LE[m] = E[h];
        LP[m] = P[h];
        LQ[m] = Q[h];
        const unsigned long long lb = __ballot(loud[h]);
        const int j = nloud + __popcll(lb & below);
        lpre[m] = (int16_t)j;
        if (loud[h]) { lz[j] = z[h]; lB[j] = B[h]; lku[j] = ku[h]; }
        nloud += __popcll(lb);
    }
    wave_sync();
    {   // pairs in masker order; the suffix of P as a prefix over the mirrored order
        const double q0 = LQ[2 * lane], q1 = LQ[2 * lane + 1];
        const double r0v = LP[127 - 2 * lane], r1v = LP[126 - 2 * lane];
        double e0, e1, r0, r1;
        wave_excl_scan2(q0, q1, &e0, &e1);
        wave_excl_scan2(r0v, r1v, &r0, &r1);
        wave_sync();
        LQ[2 * lane] = e0;
        LQ[2 * lane + 1] = e1;
        LP[127 - 2 * lane] = r0 + r0v;
        LP[126 - 2 * lane] = r1 + r1v;
    }
    wave_sync();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (!((rows >> q) & 1)) continue;          // wave-uniform
        const int l = q * WAVE + lane;
        const double zl = T->bark_line_s[l];
        // U = #maskers with zl - z > 1/2, V = #maskers with zl - z >= -1/2
        int U = 0, V = 0;
#pragma unroll
        for (int st = 64; st; st >>= 1) {
            if (U + st <= nm && __dsub_rn(zl, Lz[U + st - 1]) > 0.5) U += st;
            if (V + st <= nm && __dsub_rn(zl, Lz[V + st - 1]) >= -0.5) V += st;
        }
        double flat = 0.0;
        for (int m = U; m < V; ++m) flat += LE[m];
        const double lower = (V < nm ? LP[V] : 0.0) * T->pow_mkl_s[l];
        const double upq = LQ[U] * T->pow_kl_s[l];
        const int Ul = U < nm ? lpre[U] : nloud;
        const int umax = __builtin_amdgcn_readlane(Ul, WAVE - 1);   // U nondecreasing in l (zl ascending)
        double up = 0.0;
        for (int j = 0; j < umax; ++j) {
            const double t = pac_exp2(__builtin_fma(__dsub_rn(zl, lz[j]) - 0.5, lku[j], lB[j]));
            up += j < Ul ? t : 0.0;
        }
        out(l, (((up + upq) + flat) + lower) + T->tiq_s[l]);      // the intensity (as wave_masking_row)
    }
}
