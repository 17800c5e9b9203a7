// pac_common.h -- shared constants, device-table layout and device math for the
// MI355X (gfx950) PAC/WAK encoder.  Compiled only by hipcc for gfx950.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PAC_N 2048        // MDCT window (2 x nMDCTLines), pacfile.py:452
#define PAC_HALFN 1024    // nMDCTLines
#define PAC_NB 25         // Zwicker critical bands, psychoac.py:122
#define PAC_NTAB 10       // static Huffman tables, Huffman.py:256-262
#define PAC_NSYM 32768    // unsigned mantissa symbols (ba <= 16 -> 15 magnitude bits)
#define PAC_MAXMASK 512   // findpeaks can return at most 511 peaks in 1..1022
#define PAC_CHUNK_MAX 131071   // largest master chunk (blocks): the tail's 32-bit raw-buffer offsets (pac_master.hip)

// Constant tables, generated on the host in float64 with libm following the
// reference's numpy expressions (see pac_abi.hip build_tables) and uploaded once
// per sample rate.  Read-only in every kernel.
struct PacTables {
    double sine[PAC_N];           // window.py:27-39
    double hann[PAC_N];           // window.py:41-53
    double2 mdct_pre[PAC_HALFN / 2];   // exp(-i pi (q+1/4)/M)   (DCT-IV fold, M=1024)
    double2 mdct_post[PAC_HALFN / 2];  // exp(-i pi q / M)
    // MDCT line k of the sine-windowed block from the raw block's DFT bins X[k],
    // X[k+1] (k_master_lrms_spec, pac_master.hip mdct_from_dft):
    // (cos a, sin a, cos b, sin b) / N, a, b = 2 pi n0 (k + 1/2)/N -+ pi/(2N)
    double4 mdct_tw2[PAC_HALFN];
    double2 fft_tw[PAC_HALFN];         // exp(-2 pi i k / 1024), k < 1024
    // the radix-4 Stockham stages' twiddles W^e, W^2e, W^3e (e = k 256/Ns, k < Ns)
    // stage-major, stage Ns = 4^s at [3 ((Ns - 4)/3 + k)] (tw4_of): right after
    // fft_tw, so a kernel reaches them from the same pointer
    double2 fft_tw4[3 * (4 + 16 + 64 + 256)];
    double2 rfft_tw[PAC_HALFN];        // exp(-2 pi i k / 2048), k < 1024
    double2 rfft_tw2[PAC_HALFN];       // exp(-2 pi i k / 2048) / 2 (the side kernel's fused split)
    double bark_line[PAC_HALFN];  // Bark(MDCTFreqs)                psychoac.py:434,95
    double tiq[PAC_HALFN];        // Intensity(Thresh(MDCTFreqs))   psychoac.py:437
    double bark_bin[PAC_HALFN];   // Bark(k * (fs//N))              psychoac.py:186-188
    double mld[PAC_HALFN];        // MLD_F(MDCT_freqs) / max        psychoac.py:349-372
    int32_t nlines[PAC_NB];       // AssignMDCTLinesFromFreqLimits  psychoac.py:124-156
    int32_t lower[PAC_NB];        // ScaleFactorBands                psychoac.py:203-213
    int32_t band_of_line[PAC_HALFN];
    // sign of an exactly-zero MDCT line: the reference's post-twiddle
    // Re(F * exp(-i phi_k)) with F = +0 gives (+0*cos) - (+0*sin), i.e. -0.0
    // iff cos(phi_k) < 0 <= sin(phi_k) (mdct.py:355).  vMantissa keeps -0.0's
    // sign bit (quantize.py:333), so silent blocks depend on it.
    uint8_t mdct_zero_neg[PAC_HALFN];
    int32_t sample_rate;
    int32_t sine_win;             // 1: the MDCT window is the sine window (mdct_tw2 applies)
    // findpeaks floor 10 log10|X| > -30 (psychoac.py:168) as |X|^2 > peak_floor2:
    // the square of the largest double m with 10*log10(m) <= -30 (host libm)
    double peak_floor2;
    double inv_int[64];           // 1/i (inv_int[0] unused)
    // moment form of the masking sum (pac_wave.h): mom_eps[D] = largest eps with
    // e^eps eps^(D+1)/(D+1)! <= 2^-57 (Taylor remainder), +inf past PAC_MOM_DMAX
    double mom_eps[64];
    // leaves of numpy's pairwise complex sum over each band's FFT bins (the
    // LRMS decision, codec.py:96-102): band, first element, length in doubles
    int32_t lr_nleaf;
    int32_t lr_first_leaf[PAC_NB];
    int16_t lr_leaf_band[64], lr_leaf_e0[64], lr_leaf_n[64];
    // masking-side bin bounds per MDCT line l (psychoac.py:111-116 slope choice):
    // bin k carries a masker "below" l iff k < mask_ku[l]  (z_l - z_k >  1/2),
    // "below or flat" iff k < mask_kv[l]                  (z_l - z_k >= -1/2);
    // exact double comparisons, fl(z_l - z) is monotone in z.  With the rank
    // of each bin among the maskers this gives the zone bounds U, V per line.
    int16_t mask_ku[PAC_HALFN], mask_kv[PAC_HALFN];
    // factored masking sums (pac_wave.h): 2^(KL z_l) and 2^(-KL z_l) per line,
    // KL = -27 log2(10)/10 as the device rounds it, evaluated in long double
    double pow_kl[PAC_HALFN], pow_mkl[PAC_HALFN];
    // the masker lists' factored terms per FFT bin k (grp_find_maskers):
    // 2^(KL (z_k - 1/2)) and 2^(-KL (z_k + 1/2)), z_k = Bark(k fs//N), long double
    double pow_pl[PAC_HALFN], pow_pu[PAC_HALFN];
    // block-switching extension (pac_bs.h): the short transform (N = 512,
    // 256 lines), its window, and the masking model's tables at N = 512
    double sine_s[512];               // short MDCT window (sine, or KBD alpha 4)
    double hann_s[512];
    double2 mdct_pre_s[128];          // exp(-i pi (q+1/4)/256)
    double2 mdct_post_s[128];         // exp(-i pi q / 256)
    double bark_line_s[256], tiq_s[256], bark_bin_s[256], mld_s[256];
    double pow_kl_s[256], pow_mkl_s[256];   // 2^(KL z_l), 2^(-KL z_l) of the short lines
    // line l's band b = band_of_line[l] with its span: lower[b] | (lower[b] +
    // nlines[b] - 1) << 10 | b << 20 (k_master_front: one load per line, at
    // the kernel's start, instead of lower[b], nlines[b] behind band_of_line)
    int32_t band_span[PAC_HALFN];
};

// Huffman tables (Huffman.py, exported by tests/golden/export_huffman_tables.py)
struct PacHuffTables {
    uint8_t len[PAC_NTAB][PAC_NSYM];     // 0 = symbol absent -> escape
    uint32_t bits[PAC_NTAB][PAC_NSYM];
    int32_t esc_len[PAC_NTAB];
    uint32_t esc_bits[PAC_NTAB];
};

// ---------------------------------------------------------------------------
// device math
// ---------------------------------------------------------------------------

// 2^y for y in about [-1000, 1000]: y = n + f, |f| <= 1/2, degree-10 Chebyshev
// fit of 2^f (tools/fit_exp2.py: 3.7e-16 relative as evaluated), then ldexp.
__device__ __forceinline__ double pac_exp2(double y) {
    double n = __builtin_rint(y);
    double f = y - n;
    double p = 7.072585949269223e-09;
    p = __builtin_fma(p, f, 1.0208690299958306e-07);
    p = __builtin_fma(p, f, 1.321544258792169e-06);
    p = __builtin_fma(p, f, 1.5252657260200837e-05);
    p = __builtin_fma(p, f, 0.0001540353044173605);
    p = __builtin_fma(p, f, 0.0013333558230164974);
    p = __builtin_fma(p, f, 0.009618129107606888);
    p = __builtin_fma(p, f, 0.05550410866444772);
    p = __builtin_fma(p, f, 0.24022650695910097);
    p = __builtin_fma(p, f, 0.69314718055995);
    p = __builtin_fma(p, f, 1.0);
    return __builtin_ldexp(p, (int)n);
}
// The same 2^y (bit-identical: the same fused multiply-adds in the same order)
// with the Horner steps as VOP3 v_fma_f64 on VGPR coefficients.  Where the
// coefficients live in VGPRs (SGPR-tight kernels: the masking rows), the
// compiler otherwise shrinks each step to the two-address v_fmac_f64 and pays
// a v_mov_b64 copy of the coefficient per step.
__device__ __forceinline__ double fma_v(double a, double b, double c) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ double pac_exp2_v(double y) {
    double n = __builtin_rint(y);
    double f = y - n;
    double p = 7.072585949269223e-09;
    p = fma_v(p, f, 1.0208690299958306e-07);
    p = fma_v(p, f, 1.321544258792169e-06);
    p = fma_v(p, f, 1.5252657260200837e-05);
    p = fma_v(p, f, 0.0001540353044173605);
    p = fma_v(p, f, 0.0013333558230164974);
    p = fma_v(p, f, 0.009618129107606888);
    p = fma_v(p, f, 0.05550410866444772);
    p = fma_v(p, f, 0.24022650695910097);
    p = fma_v(p, f, 0.69314718055995);
    p = __builtin_fma(p, f, 1.0);
    return __builtin_ldexp(p, (int)n);
}

// log10(x) for positive normal x, ~35 VALU instead of the library's ~100:
// x = 2^k m, m in [sqrt(1/2), sqrt(2)), ln m = f - (f^2/2 - s (f^2/2 + R(s^2))),
// s = f/(2+f) (the classic atanh-series reduction with its minimax R), then
// k log10(2) in two parts.  Within 2 ulp of glibc's log10 (0.8 % of inputs
// differ at all, 2e7 random inputs in [1e-13.5, 1e6.5]).
__device__ __forceinline__ double pac_log10_pos(double x) {
    int k = __builtin_amdgcn_frexp_exp(x);
    double m = __builtin_amdgcn_frexp_mant(x);          // [0.5, 1)
    const bool lo = m < 0.70710678118654752440;
    m = __builtin_ldexp(m, lo ? 1 : 0);
    k -= lo ? 1 : 0;
    const double f = m - 1.0;
    const double d = 2.0 + f;
    double r = __builtin_amdgcn_rcp(d);
    r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
    r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
    double s = f * r;
    s = __builtin_fma(__builtin_fma(-d, s, f), r, s);
    const double z = s * s, w = z * z;
    const double t1 = w * __builtin_fma(w, __builtin_fma(w, 1.531383769920937332e-01, 2.222219843214978396e-01),
                                        3.999999999940941908e-01);
    const double t2 = z * __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, 1.479819860511658591e-01,
                                                                          1.818357216161805012e-01),
                                                         2.857142874366239149e-01),
                                        6.666666666666735130e-01);
    const double R = t2 + t1;
    const double hfsq = 0.5 * f * f;
    const double lnm = f - (hfsq - s * (hfsq + R));
    const double kd = (double)k;
    return __builtin_fma(kd, 3.01029995663611771306e-01,
                         __builtin_fma(kd, 3.69423907715893078616e-13, lnm * 4.34294481903251816668e-01));
}

// SPL() with the Python-2 minval Intensity(-30) = 10**-13 (psychoac.py:15-42)
__device__ __forceinline__ double pac_spl(double I) {
    if (I < 1e-13) I = 1e-13;
    double s = 96.0 + 10.0 * pac_log10_pos(I);
    return s < -30.0 ? -30.0 : s;
}

// a non-temporal 16-byte store (streamed past the L2's normal allocation)
__device__ __forceinline__ void nt_store(double2* p, double2 v) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store((d2v){v.x, v.y}, reinterpret_cast<d2v*>(p));
}

// SMR terms without a logarithm per line.  SPL is 96 + 10 log10 of the
// intensity clamped below at 10^-12.6 (its -30 dB floor), so with thresholds
// kept as intensities I (k_master_thr, k_origin_front: every threshold lies
// above the threshold in quiet, far above the floor)
//   SPL(P) - SPL(I) = 10 log10(max(P, 10^-12.6) / I)
// and the band maximum of the SMRs (psychoac.py calcStereoSMR / CalcSMRs) is
// 10 log10 of the band maximum of those ratios: one log10 per band instead of
// two per line.  Rounding of the same class as the reference's difference of
// two SPLs (a few ulp of ~100 dB).
#define PAC_SPL_IMIN 2.51188643150958e-13       // 10^(-126/10): SPL = -30 dB
// max(P, IMIN) / I for a positive normal I: v_rcp_f64 + two Newton steps
// (about 1 ulp; the division's IEEE sequence is twice as long)
__device__ __forceinline__ double pac_spl_ratio(double P, double I) {
    double r = __builtin_amdgcn_rcp(I);
    r = __builtin_fma(__builtin_fma(-I, r, 1.0), r, r);
    r = __builtin_fma(__builtin_fma(-I, r, 1.0), r, r);
    return (P > PAC_SPL_IMIN ? P : PAC_SPL_IMIN) * r;
}
// the SMR of a band maximum q of pac_spl_ratio
__device__ __forceinline__ double pac_ratio_db(double q) { return 10.0 * pac_log10_pos(q); }
// MLD thresholds (psychoac.py:582-583, MLD_* = BTHR_*_MLD * mld in dB) as the
// intensity of that SPL, 10^((mld SPL(I) - 96)/10), so that the M/S
// combination max(BTHR_M, min(BTHR_S, MLD_S)) (monotone in SPL) runs on
// intensities
__device__ __forceinline__ double pac_mld_intensity(double I, double mld) {
    return pac_exp2_v((__dmul_rn(pac_spl(I), mld) - 96.0) * 0.33219280948873624);   // log2(10)/10
}

// QuantizeUniform (quantize.py:40-64) for |a|, R <= 31 bits: the code is below
// 2^(R-1) <= 2^30, so 32-bit integers carry it (one v_cvt_u32_f64; the
// float64 -> uint64 conversion is a ~10-instruction sequence)
__device__ __forceinline__ uint32_t pac_quant_abs32(double a, int R) {
    const uint32_t sbm = 1u << (R - 1);
    if (a >= 1.0) return sbm - 1;
    const double largest = (double)(2u * sbm - 1u);
    return (uint32_t)(__dadd_rn(__dmul_rn(largest, a), 1.0) * 0.5);    // / 2.0, exact
}
__device__ __forceinline__ uint64_t pac_quant_abs(double a, int R) { return pac_quant_abs32(a, R); }

// ScaleFactor (quantize.py:148-177) with nScaleBits = 4: the leading zeros of
// the R-bit code (q << 1 < 2^R), capped at 15 -- by count-leading-zeros
// instead of the reference's shift loop (the same value)
__device__ __forceinline__ int pac_scale_factor(double a, int nMantBits) {
    if (nMantBits <= 0) return 0;
    const int R = nMantBits + 15;
    const uint32_t q = pac_quant_abs32(fabs(a), R) << 1;
    const int lz = q ? __builtin_clz(q) - (32 - R) : R;
    return lz < 15 ? lz : 15;
}

// vMantissa (quantize.py:315-342) for one line, nScaleBits = 4:
// (code << (scale + 1)) >> (R - nMantBits + 1) = code >> (15 - scale) for
// scale <= 15 (the code is below 2^30: no bits pass bit 31)
__device__ __forceinline__ uint32_t pac_mantissa(double x, int scale, int nMantBits) {
    const bool sign = __builtin_signbit(x);
    const uint32_t code = pac_quant_abs32(sign ? -x : x, nMantBits + 15);
    uint32_t m = code >> (15 - scale);
    if (sign) m += 1u << (nMantBits - 1);
    return m;
}

// pcmfile.py:89-98 + quantize.py:120-145: +-2|c|/65535, -32768 -> +0.0.
// Branch-free; the quotient is RN(2|c|/65535) exactly: q0 = 2|c| * RN(1/65535)
// corrected once by its fma residual (checked for every |c| <= 32768).
// Rounding to nearest is odd-symmetric, so the signed code goes through the
// same three operations (-32768 -> 0 first): RN(-x) = -RN(x), and 0 stays +0.0
// (bit-identical to the sign-magnitude form for all 65536 codes).
__device__ __forceinline__ double pac_pcm_to_float(int c) {
    const double n = (double)(2 * (c == -32768 ? 0 : c));
    const double r = 1.0 / 65535.0;
    const double q = n * r;
    return __builtin_fma(__builtin_fma(-q, 65535.0, n), r, q);
}

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(__dsub_rn(__dmul_rn(a.x, b.x), __dmul_rn(a.y, b.y)),
                        __dadd_rn(__dmul_rn(a.x, b.y), __dmul_rn(a.y, b.x)));
}
// a * b with two fused multiply-adds (4 VALU instead of 6): the side kernel's
// paired FFTs (rounding of the same class, not bit-identical to cmul)
__device__ __forceinline__ double2 cmul_fma(double2 a, double2 b) {
    return make_double2(__builtin_fma(a.x, b.x, -(a.y * b.y)), __builtin_fma(a.x, b.y, a.y * b.x));
}
