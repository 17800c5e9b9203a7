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
template <class V, class OUT>
__device__ __forceinline__ void wave_dct4_256(const V& v, const PacTables* __restrict__ T, double2* scr, int lane,
                                              double sc, const OUT& out) {
#pragma unroll
    for (int q0 = 0; q0 < 128; q0 += WAVE) {
        const int q = q0 + lane;
        scr[q] = cmul(make_double2(v(2 * q), v(255 - 2 * q)), T->mdct_pre_s[q]);
    }
    const double2* Y = grp_fft_stockham<7, WAVE>(scr, scr + 128, T->fft_tw, lane);
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

// calcBTHR (psychoac.py:409-456) of a short block at N = 512 by one wave, from
// the powers pw[256]: findpeaks (psychoac.py:158-191, the same floor and BW
// slice as the long model), masker SPL, then the direct masking sum per line
// in ascending masker order, + threshold in quiet, SPL.  mz/mS/mlev: 128
// doubles of LDS each.  out(l, thr) for l < 256 in the 64-line rows whose bit
// is set in `rows` (the others are not needed: not computed).
template <class OUT>
__device__ __forceinline__ void wave_threshold_short(const double* pw, const PacTables* __restrict__ T, double drop,
                                                     double* mz, double* mS, double* mlev, int* kidx, int lane,
                                                     int rows, const OUT& out) {
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
    const double csp = 8.0 / 3.0 * 4.0 / (512.0 * 512.0);
    for (int m = lane; m < nm; m += WAVE) {
        const int k = kidx[m];
        double s = 0.0;
        if (k >= 3) {
            const int hi = k + 3 < 256 ? k + 3 : 256;
            for (int i = k - 3; i < hi; ++i) s = __dadd_rn(s, pw[i]);
        }
        const double sp = pac_spl(csp * s);
        double lev = sp - 40.0;
        mlev[m] = 0.367 * (0.0 > lev ? 0.0 : lev);
        mS[m] = sp;
        mz[m] = T->bark_bin_s[k];
    }
    wave_sync();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (!((rows >> q) & 1)) continue;          // wave-uniform
        const int l = q * WAVE + lane;
        const double zl = T->bark_line_s[l];
        double I = 0.0;
        for (int m = 0; m < nm; ++m) {
            const double dz = __dsub_rn(zl, mz[m]);
            const double A = (dz >= 0 ? mlev[m] : 0.0) - 27.0;
            const double ad = fabs(dz);
            const double B = ad > 0.5 ? ad - 0.5 : 0.0;
            const double spl = __dsub_rn(__dadd_rn(mS[m], __dmul_rn(A, B)), drop);
            I = __dadd_rn(I, pac_exp2(__dmul_rn(__dsub_rn(spl, 96.0), PAC_LOG2_10_OVER_10)));
        }
        out(l, pac_spl(__dadd_rn(I, T->tiq_s[l])));
    }
}
