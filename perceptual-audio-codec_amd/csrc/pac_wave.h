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

__device__ __forceinline__ void wave_sync() {
    // LDS hand-off between lanes of one wave: drain this wave's LDS ops and
    // keep the compiler from moving accesses across (waves never share LDS).
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        double w = __shfl_xor(v, o, WAVE);
        v = w > v ? w : v;
    }
    return v;
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
    v += dpp_f64<PAC_DPP_QXOR1>(0.0, v);
    v += dpp_f64<PAC_DPP_QXOR2>(0.0, v);
    v += dpp_f64<PAC_DPP_HMIRROR>(0.0, v);
    v += dpp_f64<PAC_DPP_MIRROR>(0.0, v);              // row sums
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
    auto f = [](double a, double b) { return MAX ? fmax(a, b) : fmin(a, b); };
    v = f(v, dpp_f64<PAC_DPP_QXOR1>(v, v));
    v = f(v, dpp_f64<PAC_DPP_QXOR2>(v, v));
    v = f(v, dpp_f64<PAC_DPP_HMIRROR>(v, v));
    v = f(v, dpp_f64<PAC_DPP_MIRROR>(v, v));
    v = f(v, dpp_f64<PAC_DPP_BCAST15, 0xa>(v, v));
    v = f(v, dpp_f64<PAC_DPP_BCAST31, 0xc>(v, v));
    return readlane_f64(v, 63);
}

__device__ __forceinline__ unsigned brev(unsigned x, int bits) {
    return __builtin_bitreverse32(x) >> (32 - bits);
}

template <int NT>
__device__ __forceinline__ void grp_sync() {
    if constexpr (NT == WAVE) wave_sync(); else __syncthreads();
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

// Self-sorting (Stockham) FFT of n = 2^LOG complex values in natural order,
// radix-4 stages (+ one radix-2 stage for odd LOG), ping-ponging between src
// and dst; every read is unit-stride across lanes and no bit-reversal
// permutation is needed.  Returns the buffer holding the result (always dst:
// LOG = 10 has 5 stages, LOG = 9 has 4 + 1).  tw[k] = exp(-2 pi i k / 1024).
template <int LOG, int NT>
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
            double2 v0 = src[j], v1 = src[j + N4], v2 = src[j + 2 * N4], v3 = src[j + 3 * N4];
            if (Ns > 1) {
                const int e = k * (256 / Ns);           // angle -2 pi k r / (4 Ns)
                v1 = cmul(v1, tw[e]);
                v2 = cmul(v2, tw[2 * e]);
                v3 = cmul(v3, tw[3 * e]);
            }
            const double2 a0 = make_double2(v0.x + v2.x, v0.y + v2.y);
            const double2 a1 = make_double2(v0.x - v2.x, v0.y - v2.y);
            const double2 a2 = make_double2(v1.x + v3.x, v1.y + v3.y);
            const double2 a3 = make_double2(v1.y - v3.y, v3.x - v1.x);   // -i (v1 - v3)
            const int o = ((j - k) << 2) + k;
            dst[o] = make_double2(a0.x + a2.x, a0.y + a2.y);
            dst[o + Ns] = make_double2(a1.x + a3.x, a1.y + a3.y);
            dst[o + 2 * Ns] = make_double2(a0.x - a2.x, a0.y - a2.y);
            dst[o + 3 * Ns] = make_double2(a1.x - a3.x, a1.y - a3.y);
        }
        double2* t = src; src = dst; dst = t;
    }
    if (LOG & 1) {                                     // last stage, radix 2, Ns = N/2
        grp_sync<NT>();
#pragma unroll
        for (int j0 = 0; j0 < N / 2; j0 += NT) {
            const int j = j0 + tid;
            if ((N / 2) % NT != 0 && j >= N / 2) break;
            const double2 v0 = src[j];
            const double2 v1 = cmul(src[j + N / 2], tw[j * (1024 / N)]);
            dst[j] = make_double2(v0.x + v1.x, v0.y + v1.y);
            dst[j + N / 2] = make_double2(v0.x - v1.x, v0.y - v1.y);
        }
        double2* t = src; src = dst; dst = t;
    }
    grp_sync<NT>();
    return src;
}

// DCT-IV of 1024 values v(j), scaled by sc (a power of two):
//   X[k] = sc * sum_j v(j) cos(pi/1024 (j + 1/2)(k + 1/2)),
// via the 512-point complex Stockham FFT (even/odd interleave, pre- and
// post-twiddles).  buf: 1024 double2 of LDS; X = (double*)buf on return (first
// 8 KB), the second 8 KB is free scratch.
template <int NT, class V>
__device__ __forceinline__ double* grp_dct4(const V& v, const PacTables* __restrict__ T, double2* buf, int tid,
                                            double sc) {
#pragma unroll
    for (int q0 = 0; q0 < 512; q0 += NT) {
        const int q = q0 + tid;
        buf[q] = cmul(make_double2(v(2 * q), v(1023 - 2 * q)), T->mdct_pre[q]);
    }
    const double2* Y = grp_fft_stockham<9, NT>(buf, buf + 512, T->fft_tw, tid);   // = buf + 512
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

// |FFT(d)[k]|^2, k < 1024, of a real 2048-sample block d(i) via a 1024-point
// complex Stockham FFT.  buf and tmp: 1024 double2 of LDS each; the input
// pairs are staged in buf, the FFT ends in tmp, and on return
// buf[k].x = Re^2 + Im^2 (tmp is free again).  (findpeaks compares |X| and
// the masker SPL sums |X|^2 (psychoac.py:442-449); both only need the square.)
template <int NT, class DS>
__device__ __forceinline__ void grp_spectrum_pow(const DS& d, const PacTables* __restrict__ T,
                                                 double2* buf, double2* tmp, int tid) {
#pragma unroll 4
    for (int n0 = 0; n0 < 1024; n0 += NT) {
        int n = n0 + tid;
        buf[n] = make_double2(d(2 * n), d(2 * n + 1));
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
            buf[kk[side]].x = __builtin_fma(xr, xr, xi * xi);
        }
    }
    grp_sync<NT>();
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

// Masker list in LDS, structure of arrays over the 16 KB scratch (2048 doubles):
//   z[m]   Bark(f_m)                                       [0, 512)
//   B[m]   (SPL_m - drop - 96) * log2(10)/10               [512, 1024)
//   ku[m]  (0.367*max(SPL_m-40,0) - 27) * log2(10)/10      [1024, 1536)
//   E[m]   2^B[m] = 10^((SPL_m - drop - 96)/10)            [1536, 2048)
// Maskers are in ascending frequency, the reference's summation order.
#define PAC_LOG2_10_OVER_10 0.33219280948873624   // log2(10)/10
#define PAC_KL (-27.0 * PAC_LOG2_10_OVER_10)       // lower slope (dz < 0), psychoac.py:116
#define PAC_LN2 0.6931471805599453
// order in which the 16 masking rows (64 lines each) are claimed by the waves
// of a threshold kernel, 4 bits per row, most expensive first (measured on
// broadband input: the middle rows carry the most maskers on both sides)
#define PAC_ROW_ORDER 0xf0e1dc4528b9a763ull
#define PAC_MOM_MIN 24      // fewest common upper maskers for the moment form
#define PAC_MOM_DMAX 40     // highest Taylor degree of the moment form

__device__ __forceinline__ double* mk_z(double2* buf) { return reinterpret_cast<double*>(buf); }
__device__ __forceinline__ double* mk_B(double2* buf) { return reinterpret_cast<double*>(buf) + 512; }
__device__ __forceinline__ double* mk_ku(double2* buf) { return reinterpret_cast<double*>(buf) + 1024; }
__device__ __forceinline__ double* mk_E(double2* buf) { return reinterpret_cast<double*>(buf) + 1536; }

// findpeaks (psychoac.py:158-191) on |X|^2 held in buf[k].x (the floor
// 10 log10|X| > -30 is the equivalent |X|^2 > T->peak_floor2), masker SPL from the
// 6-bin slice X[k-3:k+3] (psychoac.py:448, Python slice semantics), then the
// compacted masker list (ascending bin order) written over buf by a group of
// NT threads.  scratch: LDS of 16 + 512 ints.  Returns the masker count.
// Peaks are compacted first (ballots, bin order = the reference's summation
// order) so that the SPL (a log10 each) is evaluated once per masker.
// rank[k] (k < 1024) = #maskers with bin < k, for the zone bounds of the
// masking sum (PacTables::mask_ku / mask_kv).
template <int NT>
__device__ __forceinline__ int grp_find_maskers(double2* buf, const PacTables* __restrict__ T,
                                                double drop, int tid, int* scratch, int16_t* rank) {
    constexpr int J = 1024 / NT;
    constexpr int NW = NT / WAVE;
    int* cnt = scratch;              // [J][NW] peak counts of the (j, wave) segments, in bin order
    int* kidx = scratch + 16;        // compacted peak bins
    const int lane = tid & (WAVE - 1);
    const int w = tid / WAVE;
    const double floor2 = T->peak_floor2;
    unsigned long long bal[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int k = j * NT + tid;
        bool pk = false;
        if (k >= 1 && k <= 1022) {
            const double m = buf[k].x;
            pk = m > buf[k - 1].x && m > buf[k + 1].x && m > floor2;
        }
        bal[j] = __ballot(pk);
        if (lane == 0) cnt[j * NW + w] = __popcll(bal[j]);
    }
    grp_sync<NT>();
    int pre[J * NW];                 // exclusive prefix of the segment counts
    int tot = 0;
#pragma unroll
    for (int i = 0; i < J * NW; ++i) { pre[i] = tot; tot += cnt[i]; }
    const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int idx = pre[j * NW + w] + __popcll(bal[j] & below);
        rank[j * NT + tid] = (int16_t)idx;
        if ((bal[j] >> lane) & 1ull) kidx[idx] = j * NT + tid;
    }
    grp_sync<NT>();
    tot = __builtin_amdgcn_readfirstlane(tot);
    constexpr int R = (PAC_MAXMASK + NT - 1) / NT;
    double rz[R], rB[R], rku[R], rE[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int idx = q * NT + tid;
        if (idx < tot) {
            const int k = kidx[idx];
            double s = 0.0;
            if (k >= 3) {
                const int hi = k + 3 < 1024 ? k + 3 : 1024;
                for (int i = k - 3; i < hi; ++i) s = __dadd_rn(s, buf[i].x);   // builtin sum, from 0
            }
            const double csp = 8.0 / 3.0 * 4.0 / (2048.0 * 2048.0);
            const double sp = pac_spl(csp * s);
            double lev = sp - 40.0;
            lev = 0.367 * (0.0 > lev ? 0.0 : lev);       // builtin max(SPL-40, 0)
            rB[q] = (sp - drop - 96.0) * PAC_LOG2_10_OVER_10;
            rz[q] = T->bark_bin[k];
            rku[q] = (lev - 27.0) * PAC_LOG2_10_OVER_10;
            rE[q] = pac_exp2(rB[q]);
        }
    }
    grp_sync<NT>();   // every |X|^2 read done before the list overwrites buf
    double* mz = mk_z(buf);
    double* mB = mk_B(buf);
    double* mku = mk_ku(buf);
    double* mE = mk_E(buf);
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int idx = q * NT + tid;
        if (idx < tot) { mz[idx] = rz[q]; mB[idx] = rB[q]; mku[idx] = rku[q]; mE[idx] = rE[q]; }
    }
    grp_sync<NT>();
    return tot;
}

__device__ __forceinline__ int wave_find_maskers(double2* buf, const PacTables* __restrict__ T,
                                                 double drop, int lane, int* scratch, int16_t* rank) {
    return grp_find_maskers<WAVE>(buf, T, drop, lane, scratch, rank);
}

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

// wave-uniform results, returned in scalar registers (uniform loop bounds)
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { int w = __shfl_xor(v, o, WAVE); v = w < v ? w : v; }
    return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { int w = __shfl_xor(v, o, WAVE); v = w > v ? w : v; }
    return __builtin_amdgcn_readfirstlane(v);
}

// Masking threshold (psychoac.py:447-456): for each MDCT line
//   I(l) = sum_m 10^((spl_m(l) - 96)/10) + Intensity(Thresh(f_l)),  thr = SPL(I)
// with spl_m(l) = SPL_m + spread(dz) - drop, dz = Bark(f_l) - Bark(f_m).
// The sum splits by dz (the reference's slope selection, psychoac.py:111-116):
//   dz >  1/2 (masker below the line): 2^(beta_m + ku_m (z_l - z_r)) per pair,
//              beta_m = B_m + ku_m ((z_r - z_m) - 1/2) once per (row, masker);
//              a leading run of maskers whose largest term over the row is
//              below 2^-64 of a lower bound of every line's total is skipped;
//   |dz| <= 1/2 (flat):                E_m = 2^B_m                no exp;
//   dz < -1/2 (masker above the line): 2^(B_m + KL (z_m - 1/2 - z_r)) * 2^(KL (z_r - z_l))
//              -- the lower slope is the constant -27 dB/Bark, so these terms
//              factor into per-row suffix sums over maskers (one exp2 per
//              masker per row instead of per line), exponents in double-double.
// Every line adds its terms in ascending masker order; the loops are split so
// that only the ragged ends of each zone need a per-lane test.  Values agree
// with the direct sum to ~1e-15 relative.  Lane owns line l = 64 r + lane.
// beta: 512 doubles of LDS private to the calling wave.
// diagnostic build (-DPAC_ROWPROF): cycle and size counters of the masking rows
#ifdef PAC_ROWPROF
__device__ unsigned long long pac_rowprof[1024 * 16];   // spread over 1024 lines: no hot address
#define RP_T(v) long long v = (long long)__builtin_amdgcn_s_memtime()
#define RP_ADD(i, x) do { if (lane == 0) atomicAdd(&pac_rowprof[(blockIdx.x & 1023) * 16 + (i)], (unsigned long long)(x)); } while (0)
#else
#define RP_T(v) do {} while (0)
#define RP_ADD(i, x) do {} while (0)
#endif

__device__ __forceinline__ double wave_masking_row(const double2* buf, int nm, const PacTables* __restrict__ T,
                                                   int lane, int r, double* beta, const int16_t* rank) {
    const double* mz = mk_z(const_cast<double2*>(buf));
    const double* mB = mk_B(const_cast<double2*>(buf));
    const double* mku = mk_ku(const_cast<double2*>(buf));
    const double* mE = mk_E(const_cast<double2*>(buf));
    const int l = r * WAVE + lane;
    const double zl = T->bark_line[l];
    const double zr = T->bark_line[r * WAVE];          // row reference = smallest z
    // U = #{m : zl - z_m > 1/2}, V = #{m : zl - z_m >= -1/2} (prefixes: z_m ascending),
    // from the host-built bin bounds and the maskers' bin ranks
    const int U = rank[T->mask_ku[l]];
    const int V = rank[T->mask_kv[l]];
    RP_T(t0);
    // --- lower side: suffix sums of P_m = 2^(B_m + KL (z_m - 1/2 - zr)) over m >= vmin,
    //     gathered at each lane's V by a cross-lane shuffle (no LDS)
    const int vmin = wave_min_i(V);
    double carry = 0.0, sv = 0.0;
    for (int top = nm; top > vmin; top -= WAVE) {
        const int m = top - WAVE + lane;
        double x = 0.0;
        if (m >= vmin) {
            double h, lo2;
            dd_affine(mB[m], PAC_KL, mz[m] - 0.5, zr, h, lo2);
            x = pac_exp2_dd(h, lo2);
        }
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {            // inclusive suffix scan in the chunk
            double y = __shfl_down(x, o, WAVE);
            if (lane + o < 64) x += y;
        }
        const double tot = __shfl(x, 0, WAVE);
        const int idx = V - (top - WAVE);
        const double g = __shfl(x, idx & 63, WAVE) + carry;
        if (idx >= 0 && idx < WAVE) sv = g;
        carry += tot;
    }
    double lower = 0.0;
    if (V < nm) {
        double h, lo2;
        dd_affine(0.0, -PAC_KL, zl, zr, h, lo2);
        lower = sv * pac_exp2_dd(h, lo2);
    }
    RP_T(t1);
    // --- flat zone [U, V), ascending: ragged head, common middle, ragged tail
    double flat = 0.0;
    const int umin = wave_min_i(U), umax = wave_max_i(U), vmax = wave_max_i(V);
    const int fa = umax < vmax ? umax : vmax;
    const int fb = fa > vmin ? fa : vmin;
    const int span = wave_max_i(V - U);           // longest flat zone of the row
    if (span < vmax - umin) {                     // each lane walks its own zone
        for (int i = 0; i < span; ++i) {
            const int m = U + i;
            const double e = mE[m < V ? m : 0];
            flat += (m < V) ? e : 0.0;
        }
    } else {                                      // or the row's union of zones
        for (int m = umin; m < fa; ++m) {
            const double e = mE[m];
            flat += (m >= U && m < V) ? e : 0.0;
        }
        for (int m = fa; m < fb; ++m) flat += mE[m];   // U <= umax <= m < vmin <= V on every lane
        for (int m = fb; m < vmax; ++m) {
            const double e = mE[m];
            flat += (m >= U && m < V) ? e : 0.0;
        }
    }
    RP_T(t2);
    // --- upper side, ascending
    const double tiq = T->tiq[l];
    const double lb = wave_ext_f64<false>(tiq + flat + lower);   // I(l) >= lb on every lane
    // floor(log2 lb) - 64 from the exponent field: a conservative cut
    const double l2cut = (double)(__builtin_amdgcn_frexp_exp(lb) - 65);
    int m0 = umax;                    // first masker that is not negligible (64 tested at once)
    for (int base = 0; base < umax; base += WAVE) {
        const int m = base + lane;
        int keep = 1;
        if (m < umax) {
            const double ku = mku[m];
            const double t = __builtin_fma(fmax((zr - mz[m]) - 0.5, 0.0), ku, mB[m]);
            keep = !(ku < 0.0 && t < l2cut);
        }
        const unsigned long long kb = __ballot(keep);
        if (kb) { m0 = base + __builtin_ctzll(kb); break; }
    }
    m0 = __builtin_amdgcn_readfirstlane(m0 < umax ? m0 : umax);
    RP_T(t3);
    // exponents relative to the row middle: 2^(beta_m + ku_m (z_l - z_mid))
    const double zm = 0.5 * (zr + T->bark_line[r * WAVE + WAVE - 1]);
    for (int m = m0 + lane; m < umax; m += WAVE)
        beta[m] = __builtin_fma((zm - mz[m]) - 0.5, mku[m], mB[m]);
    wave_sync();
    const double dl = zl - zm;
    double up = 0.0;
    const int ua = umin > m0 ? (umin < umax ? umin : umax) : m0;
    // Maskers [m0, ua) lie below every line of the row.  Their sum factors as
    //   2^(kc dl) * sum_d (dl ln2)^d / d! * S_d,   S_d = sum_m 2^beta_m (ku_m - kc)^d,
    // kc the middle of their slopes: the Taylor series of 2^((ku_m - kc) dl),
    // truncated where its remainder is below 2^-57 of every term.
    bool direct = true;
    if (ua - m0 >= PAC_MOM_MIN) {
        double kmn = INFINITY, kmx = -INFINITY;
        for (int m = m0 + lane; m < ua; m += WAVE) {
            const double k = mku[m];
            kmn = fmin(kmn, k);
            kmx = fmax(kmx, k);
        }
        kmn = wave_ext_f64<false>(kmn);
        kmx = wave_ext_f64<true>(kmx);
        // max |z_l - z_mid| over the row (ascending z: an end line)
        const double adl = fmax(zm - zr, T->bark_line[r * WAVE + WAVE - 1] - zm);
        const double kc = 0.5 * (kmn + kmx);
        const double eps = (0.5 * (kmx - kmn) * adl) * PAC_LN2 * 1.0000001;
        // smallest D with e^eps eps^(D+1)/(D+1)! <= 2^-57 (uniform): lane j tests
        // eps against its bound; PAC_MOM_DMAX + 1 (no moment form) past the table
        const unsigned long long ok = __ballot(eps <= T->mom_eps[lane]);
        const int D = ok ? (int)__builtin_ctzll(ok) : PAC_MOM_DMAX + 1;
#ifdef PAC_ROWPROF
        RP_ADD(8, D);
#endif
        if (D <= PAC_MOM_DMAX) {
            direct = false;
            const double x = dl * PAC_LN2;
            const double invl = T->inv_int[lane];      // 1/j in lane j
            double acc = 0.0, q = 1.0;
            if (ua - m0 <= 2 * WAVE) {                 // two maskers per lane, in registers
                const int ma = m0 + lane, mb = ma + WAVE;
                double p0 = 0.0, c0 = 0.0, p1 = 0.0, c1 = 0.0;
                if (ma < ua) { p0 = pac_exp2(beta[ma]); c0 = mku[ma] - kc; }
                if (mb < ua) { p1 = pac_exp2(beta[mb]); c1 = mku[mb] - kc; }
                for (int d = 0; d <= D; ++d) {
                    acc = __builtin_fma(wave_sum_f64(p0 + p1), q, acc);
                    p0 *= c0;
                    p1 *= c1;
                    q = (q * x) * readlane_f64(invl, d + 1);
                }
            } else {
                for (int m = m0 + lane; m < ua; m += WAVE) beta[m] = pac_exp2(beta[m]);   // own slots
                for (int d = 0; d <= D; ++d) {
                    double part = 0.0;
                    for (int m = m0 + lane; m < ua; m += WAVE) {
                        const double p = beta[m];
                        part += p;
                        beta[m] = p * (mku[m] - kc);
                    }
                    acc = __builtin_fma(wave_sum_f64(part), q, acc);
                    q = (q * x) * readlane_f64(invl, d + 1);
                }
            }
            up = acc * pac_exp2(kc * dl);
        }
    }
    RP_T(t4);
    if (direct) {
#pragma unroll 2
        for (int m = m0; m < ua; ++m)               // m < umin <= U on every lane
            up += pac_exp2(__builtin_fma(dl, mku[m], beta[m]));
    }
#pragma unroll 2
    for (int m = ua; m < umax; ++m) {
        const double t = pac_exp2(__builtin_fma(dl, mku[m], beta[m]));
        up += (m < U) ? t : 0.0;
    }
    wave_sync();                                    // beta is rewritten by the next row
    RP_T(t5);
#ifdef PAC_ROWPROF
    RP_ADD(0, 1); RP_ADD(1, t1 - t0); RP_ADD(2, t2 - t1); RP_ADD(3, t3 - t2); RP_ADD(4, t4 - t3);
    RP_ADD(5, t5 - t4); RP_ADD(6, nm); RP_ADD(7, direct ? 0 : 1); RP_ADD(9, ua - m0);
    RP_ADD(10, umax - ua); RP_ADD(11, vmax - umin); RP_ADD(12, nm - vmin); RP_ADD(13, m0);
    RP_ADD(14, direct ? (ua - m0) : 0);
#endif
    return pac_spl(((up + flat) + lower) + tiq);
}

// all 16 rows by one wave
__device__ __forceinline__ void wave_masking(const double2* buf, int nm, const PacTables* __restrict__ T,
                                             int lane, double thr[16], double* beta, const int16_t* rank) {
#pragma unroll 1
    for (int r = 0; r < 16; ++r) thr[r] = wave_masking_row(buf, nm, T, lane, r, beta, rank);
}
