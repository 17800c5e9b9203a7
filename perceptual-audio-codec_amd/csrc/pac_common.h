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

// Constant tables, generated on the host in float64 with libm following the
// reference's numpy expressions (see pac_abi.hip build_tables) and uploaded once
// per sample rate.  Read-only in every kernel.
struct PacTables {
    double sine[PAC_N];           // window.py:27-39
    double hann[PAC_N];           // window.py:41-53
    double2 mdct_pre[PAC_HALFN / 2];   // exp(-i pi (q+1/4)/M)   (DCT-IV fold, M=1024)
    double2 mdct_post[PAC_HALFN / 2];  // exp(-i pi q / M)
    double2 fft_tw[PAC_HALFN / 2];     // exp(-2 pi i k / 1024), k < 512
    double2 rfft_tw[PAC_HALFN];        // exp(-2 pi i k / 2048), k < 1024
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
    int32_t pad_;
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

// 2^y for y in about [-300, 60]: y = n + f, |f| <= 1/2, degree-11 Chebyshev fit
// of 2^f (max rel err 2.7e-17 before rounding), then ldexp.  ~1 ulp.
__device__ __forceinline__ double pac_exp2(double y) {
    double n = __builtin_rint(y);
    double f = y - n;
    double p = 4.456051696773062e-10;
    p = __builtin_fma(p, f, 7.074198612412512e-09);
    p = __builtin_fma(p, f, 1.0178055564858192e-07);
    p = __builtin_fma(p, f, 1.3215432509674393e-06);
    p = __builtin_fma(p, f, 1.5252733845316332e-05);
    p = __builtin_fma(p, f, 0.00015403530463783927);
    p = __builtin_fma(p, f, 0.0013333558146402102);
    p = __builtin_fma(p, f, 0.009618129107587194);
    p = __builtin_fma(p, f, 0.05550410866482165);
    p = __builtin_fma(p, f, 0.2402265069591016);
    p = __builtin_fma(p, f, 0.6931471805599453);
    p = __builtin_fma(p, f, 1.0);
    return __builtin_ldexp(p, (int)n);
}

// SPL() with the Python-2 minval Intensity(-30) = 10**-13 (psychoac.py:15-42)
__device__ __forceinline__ double pac_spl(double I) {
    if (I < 1e-13) I = 1e-13;
    double s = 96.0 + 10.0 * log10(I);
    return s < -30.0 ? -30.0 : s;
}

// QuantizeUniform (quantize.py:40-64) for |a|, R bits
__device__ __forceinline__ uint64_t pac_quant_abs(double a, int R) {
    uint64_t sbm = 1ull << (R - 1);
    double largest = (double)(sbm << 1) - 1.0;
    if (a >= 1.0) return sbm - 1;
    return (uint64_t)(__dadd_rn(__dmul_rn(largest, a), 1.0) / 2.0);
}

// ScaleFactor (quantize.py:148-177) with nScaleBits = 4
__device__ __forceinline__ int pac_scale_factor(double a, int nMantBits) {
    if (nMantBits <= 0) return 0;
    const int largestScale = 15;
    int R = nMantBits + largestScale;
    uint64_t q = pac_quant_abs(fabs(a), R) << 1;
    // leading zeros of the R-bit code, capped at 15
    int scale = 0;
    uint64_t zmask = 1ull << (R - 1);
    while (scale < largestScale && (zmask & q) == 0) { q <<= 1; scale++; }
    return scale;
}

// vMantissa (quantize.py:315-342) for one line, nScaleBits = 4
__device__ __forceinline__ uint32_t pac_mantissa(double x, int scale, int nMantBits) {
    const int R = nMantBits + 15;
    bool sign = __builtin_signbit(x);
    double a = sign ? -x : x;
    uint64_t sbm = 1ull << (R - 1);
    double largest = (double)(sbm << 1) - 1.0;
    uint64_t code = (a < 1.0) ? (uint64_t)(__dadd_rn(__dmul_rn(a, largest), 1.0) / 2.0) : sbm - 1;
    uint64_t m = (code << (scale + 1)) >> (R - nMantBits + 1);
    if (sign) m += 1ull << (nMantBits - 1);
    return (uint32_t)m;
}

// pcmfile.py:89-98 + quantize.py:120-145: +-2|c|/65535, -32768 -> +0.0
__device__ __forceinline__ double pac_pcm_to_float(int c) {
    if (c >= 0) return (2.0 * (double)c) / 65535.0;
    if (c == -32768) return 0.0;
    return -((2.0 * (double)(-c)) / 65535.0);
}

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(__dsub_rn(__dmul_rn(a.x, b.x), __dmul_rn(a.y, b.y)),
                        __dadd_rn(__dmul_rn(a.x, b.y), __dmul_rn(a.y, b.x)));
}
