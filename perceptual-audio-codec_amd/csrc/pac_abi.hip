// pac_abi.hip -- host side of libpacgpu.so: the C-ABI declared in
// include/pac_gpu.h, constant-table generation and kernel orchestration.
//
// One translation unit (kernels included) so hipcc emits one gfx950 code
// object.  Host tables are generated in float64 with libm following the
// reference's numpy expressions, then uploaded once per sample rate.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <unordered_map>
#include <vector>

#include "../../include/pac_gpu.h"
#include "pac_kernels.hip"
#include "pac_master.hip"
#include "pac_decode.hip"
#include "pac_wav.hip"

#define PAC_VERSION 100

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------

static thread_local char g_err[512];

static int set_err(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

#define HIPCHK(x)                                                                         \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess)                                                             \
            return set_err(PAC_E_HIP, "%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), \
                           __FILE__, __LINE__);                                           \
    } while (0)

extern "C" const char* pac_last_error(void) { return g_err; }
extern "C" int pac_version(void) { return PAC_VERSION; }

// ---------------------------------------------------------------------------
// constant tables (host, float64, libm)
// ---------------------------------------------------------------------------

static const double kCbFreqLimits[PAC_NB] = {  // psychoac.py:122
    100.0, 200.0, 300.0, 400.0, 510.0, 630.0, 770.0, 920.0, 1080.0, 1270.0,
    1480.0, 1720.0, 2000.0, 2320.0, 2700.0, 3150.0, 3700.0, 4400.0, 5300.0,
    6400.0, 7700.0, 9500.0, 12000.0, 15500.0, 24000.0};

static double host_bark(double f) {  // psychoac.py:56-64
    double khz = f / 1000.0;
    double t2 = khz / 7.5;
    return 13.0 * atan(khz * 0.76) + 3.5 * atan(t2 * t2);
}

static double host_thresh(double f) {  // psychoac.py:44-54
    if (f < 10.0) f = 10.0;
    double khz = f / 1000.0;
    double d = khz - 3.3;
    return 3.64 * pow(khz, -0.8) + -6.5 * exp(-0.6 * (d * d)) + 0.001 * pow(khz, 4.0);
}

// AssignMDCTLinesFromFreqLimits(1024, fs) psychoac.py:124-156
static void host_band_layout(int fs, int32_t* out) {
    double lower = 0.0, upper = 0.0;
    for (int b = 0; b < PAC_NB; b++) {
        double limit = kCbFreqLimits[b];
        upper = (limit >= fs / 2.0) ? fs / 2.0 : limit;
        int cnt = 0;
        for (int k = 0; k < PAC_HALFN; k++) {
            double f = (k + 0.5) / PAC_HALFN * (double)(fs / 2);  // Py2 int sampleRate/2
            if (f <= upper && f > lower) cnt++;
        }
        out[b] = cnt;
        lower = upper;
    }
}

// KBDWindow (window.py:56-78), alpha = 4: the Kaiser kernel over t = 0..N/2,
// w[n] = sqrt(cumsum(kaiser[:-1]^2)[n] / sum(kaiser^2)), mirrored.  Evaluated
// in long double (I0 by its power series) and rounded once: Princen-Bradley
// w[n]^2 + w[n+N/2]^2 = 1 holds to the last bit of the rounding.
static long double bessel_i0(long double x) {
    long double sum = 1.0L, term = 1.0L;
    const long double q = x * x / 4.0L;
    for (int k = 1; k < 500; k++) {
        term *= q / ((long double)k * (long double)k);
        sum += term;
        if (term < sum * 1e-22L) break;
    }
    return sum;
}
static void kbd_window(int n, double alpha, double* w) {
    const int h = n / 2;
    std::vector<long double> k2(h + 1);
    const long double pa = (long double)M_PI * (long double)alpha, norm = bessel_i0(pa);
    long double den = 0.0L;
    for (int t = 0; t <= h; t++) {
        const long double r = 4.0L * t / n - 1.0L;
        const long double kv = bessel_i0(pa * sqrtl(fmaxl(0.0L, 1.0L - r * r))) / norm;
        k2[t] = kv * kv;
        den += k2[t];
    }
    long double cum = 0.0L;
    for (int t = 0; t < h; t++) {
        cum += k2[t];
        w[t] = (double)sqrtl(cum / den);
        w[n - 1 - t] = w[t];
    }
}

static void build_tables(int fs, int window, PacTables* t) {
    memset(t, 0, sizeof(*t));
    t->sample_rate = fs;
    host_band_layout(fs, t->nlines);
    int acc = 0;
    for (int b = 0; b < PAC_NB; b++) {
        t->lower[b] = acc;
        for (int l = acc; l < acc + t->nlines[b]; l++) t->band_of_line[l] = b;
        acc += t->nlines[b];
    }
    for (int l = acc; l < PAC_HALFN; l++) t->band_of_line[l] = PAC_NB - 1;  // unreachable
    for (int l = 0; l < PAC_HALFN; l++) {
        const int b = t->band_of_line[l];
        t->band_span[l] = t->lower[b] | ((t->lower[b] + t->nlines[b] - 1) << 10) | (b << 20);
    }
    for (int n = 0; n < PAC_N; n++) {
        double tt = (double)n;
        t->sine[n] = sin((tt + 0.5) * M_PI / (double)PAC_N);
        t->hann[n] = 0.5 * (1 - cos(2.0 * (tt + 0.5) * M_PI / (double)PAC_N));
    }
    if (window == PAC_WINDOW_KBD) kbd_window(PAC_N, 4.0, t->sine);   // the MDCT window of every kernel
    const double M = PAC_HALFN;
    for (int q = 0; q < PAC_HALFN / 2; q++) {
        double a = -M_PI * (q + 0.25) / M;
        t->mdct_pre[q] = make_double2(cos(a), sin(a));
        double b = -M_PI * q / M;
        t->mdct_post[q] = make_double2(cos(b), sin(b));
    }
    for (int k = 0; k < PAC_HALFN; k++) {
        double c = -2.0 * M_PI * k / 1024.0;
        t->fft_tw[k] = make_double2(cos(c), sin(c));
    }
    static_assert(offsetof(PacTables, fft_tw4) == offsetof(PacTables, fft_tw) + PAC_HALFN * sizeof(double2),
                  "tw4_of addresses the stage table from fft_tw");
    for (int Ns = 4, b = 0; Ns <= 256; b += Ns, Ns *= 4)
        for (int k = 0; k < Ns; k++)
            for (int r = 1; r <= 3; r++) t->fft_tw4[3 * (b + k) + r - 1] = t->fft_tw[r * k * (256 / Ns)];
    for (int k = 0; k < PAC_HALFN; k++) {
        double a = -2.0 * M_PI * k / 2048.0;
        t->rfft_tw[k] = make_double2(cos(a), sin(a));
    }
    for (int k = 0; k < PAC_HALFN; k++) t->rfft_tw2[k] = make_double2(0.5 * t->rfft_tw[k].x, 0.5 * t->rfft_tw[k].y);
    t->sine_win = window == PAC_WINDOW_SINE;
    for (int k = 0; k < PAC_HALFN; k++) {
        // sin(pi (n + 1/2)/N) = (e^{i pi (n+1/2)/N} - e^{-i pi (n+1/2)/N}) / 2i turns the
        // MDCT's odd-frequency sum of x*w into (c X[k] - conj(c) X[k+1]) / 2i, c = e^{i pi/2N}
        const long double pi = 3.141592653589793238462643383279502884L;
        const long double th = 2.0L * pi * 512.5L * ((long double)k + 0.5L) / 2048.0L;
        const long double a = th - pi / 4096.0L, b = th + pi / 4096.0L;
        t->mdct_tw2[k] = make_double4((double)(cosl(a) / 2048.0L), (double)(sinl(a) / 2048.0L),
                                      (double)(cosl(b) / 2048.0L), (double)(sinl(b) / 2048.0L));
    }
    {   // mdct.py:355 post-twiddle angle, evaluated as numpy does
        double c1 = (-2.0 * M_PI) / (double)PAC_N;
        double c2 = c1 * 512.5;
        for (int k = 0; k < PAC_HALFN; k++) {
            double ph = c2 * (k + 0.5);
            t->mdct_zero_neg[k] = (cos(ph) < 0.0 && sin(ph) >= 0.0) ? 1 : 0;
        }
    }
    {   // findpeaks floor: largest m with 10*log10(m) <= -30, squared
        double m = 1e-3;
        while (10.0 * log10(m) > -30.0) m = nextafter(m, 0.0);
        while (10.0 * log10(nextafter(m, 1.0)) <= -30.0) m = nextafter(m, 1.0);
        t->peak_floor2 = m * m;
    }
    for (int i = 1; i < 64; i++) t->inv_int[i] = 1.0 / (double)i;
    for (int d = 0; d < 64; d++) {
        if (d > 40) { t->mom_eps[d] = INFINITY; continue; }     // PAC_MOM_DMAX
        // ln remainder = eps + (d+1) ln eps - lgamma(d+2), increasing in eps
        const long double lim = -57.0L * logl(2.0L), lg = lgammal((long double)d + 2.0L);
        long double lo = 0.0L, hi = 64.0L;
        for (int it = 0; it < 200; it++) {
            const long double mid = 0.5L * (lo + hi);
            if (mid + ((long double)d + 1.0L) * logl(mid) - lg <= lim) lo = mid; else hi = mid;
        }
        t->mom_eps[d] = (double)(lo * (1.0L - 1e-12L));          // conservative
    }
    {   // numpy pairwise-sum leaves (loops_utils.h.src) of every band, in order
        int nl = 0;
        struct Rec {
            static void go(PacTables* t, int& nl, int b, int e0, int n) {
                if (n <= 128) {
                    if (nl < 64) {
                        t->lr_leaf_band[nl] = (int16_t)b;
                        t->lr_leaf_e0[nl] = (int16_t)e0;
                        t->lr_leaf_n[nl] = (int16_t)n;
                    }
                    nl++;
                    return;
                }
                int n2 = n / 2;
                n2 -= n2 % 8;
                go(t, nl, b, e0, n2);
                go(t, nl, b, e0 + n2 / 2, n - n2);
            }
        };
        for (int b = 0; b < PAC_NB; b++) {
            t->lr_first_leaf[b] = nl;
            Rec::go(t, nl, b, 0, 2 * t->nlines[b]);
        }
        t->lr_nleaf = nl;     // <= 64 for any layout of 1024 lines (checked in get_tables)
    }
    const int step = fs / PAC_N;  // Py2 integer division, psychoac.py:188
    double mx = -1.0;
    for (int k = 0; k < PAC_HALFN; k++) {
        double f = fs / 2.0 / (double)PAC_HALFN * ((double)k + 0.5);  // psychoac.py:434
        t->bark_line[k] = host_bark(f);
        t->tiq[k] = pow(10.0, (host_thresh(f) - 96.0) / 10.0);
        t->bark_bin[k] = host_bark((double)(k * step));
        double f2 = (((double)k + 0.5) / (double)PAC_HALFN) * (fs / 2.0);  // psychoac.py:570
        double fm = f2 < 3000. ? f2 : 3000.;
        double v = pow(10.0, 1.25 * (1 - cos(M_PI * (fm / 3000.))) - 2.5);
        t->mld[k] = v;
        if (v > mx) mx = v;
    }
    for (int k = 0; k < PAC_HALFN; k++) t->mld[k] = t->mld[k] / mx;
    {
        const long double kl = (long double)(-27.0 * 0.33219280948873624);   // PAC_KL, double-rounded
        for (int l = 0; l < PAC_HALFN; l++) {
            const long double e = kl * (long double)t->bark_line[l];
            t->pow_kl[l] = (double)exp2l(e);
            t->pow_mkl[l] = (double)exp2l(-e);
            const long double zb = (long double)t->bark_bin[l];
            t->pow_pl[l] = (double)exp2l(kl * (zb - 0.5L));
            t->pow_pu[l] = (double)exp2l(-kl * (zb + 0.5L));
        }
    }
    {   // block-switching extension tables (pac_bs.h), the same formulas at N = 512
        for (int n = 0; n < 512; n++) {
            t->sine_s[n] = sin(((double)n + 0.5) * M_PI / 512.0);
            t->hann_s[n] = 0.5 * (1 - cos(2.0 * ((double)n + 0.5) * M_PI / 512.0));
        }
        if (window == PAC_WINDOW_KBD) kbd_window(512, 4.0, t->sine_s);
        for (int q = 0; q < 128; q++) {
            const double a = -M_PI * (q + 0.25) / 256.0, b = -M_PI * q / 256.0;
            t->mdct_pre_s[q] = make_double2(cos(a), sin(a));
            t->mdct_post_s[q] = make_double2(cos(b), sin(b));
        }
        const int step_s = fs / 512;
        double mxs = -1.0;
        for (int k = 0; k < 256; k++) {
            const double f = fs / 2.0 / 256.0 * ((double)k + 0.5);
            t->bark_line_s[k] = host_bark(f);
            t->tiq_s[k] = pow(10.0, (host_thresh(f) - 96.0) / 10.0);
            t->bark_bin_s[k] = host_bark((double)(k * step_s));
            const double f2 = (((double)k + 0.5) / 256.0) * (fs / 2.0);
            const double fm = f2 < 3000. ? f2 : 3000.;
            const double v = pow(10.0, 1.25 * (1 - cos(M_PI * (fm / 3000.))) - 2.5);
            t->mld_s[k] = v;
            if (v > mxs) mxs = v;
        }
        for (int k = 0; k < 256; k++) t->mld_s[k] = t->mld_s[k] / mxs;
        const long double kl = (long double)(-27.0 * 0.33219280948873624);   // PAC_KL, double-rounded
        for (int l = 0; l < 256; l++) {
            const long double e = kl * (long double)t->bark_line_s[l];
            t->pow_kl_s[l] = (double)exp2l(e);
            t->pow_mkl_s[l] = (double)exp2l(-e);
        }
    }
    for (int l = 0, ku = 0, kv = 0; l < PAC_HALFN; l++) {   // bark_line ascending in l
        const double zl = t->bark_line[l];
        while (ku < PAC_HALFN - 1 && zl - t->bark_bin[ku] > 0.5) ku++;
        while (kv < PAC_HALFN - 1 && zl - t->bark_bin[kv] >= -0.5) kv++;
        t->mask_ku[l] = (int16_t)ku;
        t->mask_kv[l] = (int16_t)kv;
    }
}

extern "C" int pac_band_layout(int32_t sample_rate, int32_t n_lines_out[25]) {
    if (sample_rate <= 0 || !n_lines_out) return set_err(PAC_E_ARG, "bad sample rate / pointer");
    host_band_layout(sample_rate, n_lines_out);
    return PAC_OK;
}

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    int ensure(size_t want) {
        if (want <= n) return PAC_OK;
        if (p) hipFree(p);
        p = nullptr;
        n = 0;
        size_t cap = want + want / 4 + 64;
        if (hipMalloc((void**)&p, cap * sizeof(T)) != hipSuccess)
            return set_err(PAC_E_NOMEM, "hipMalloc(%zu bytes) failed", cap * sizeof(T));
        n = cap;
        return PAC_OK;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        n = 0;
    }
};

struct pac_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::map<int, PacTables*> tables;  // device tables per sample rate
    PacHuffTables* huff = nullptr;     // device
    DevBuf<uint32_t> hscore;           // [PAC_HSC_N][PAC_HSC_W] per-(ba, symbol) costs of the ten tables (k_master_tail)
    bool have_huff = false;
    // work
    DevBuf<double> smr, bandpeak;
    DevBuf<long long> prof;                // PAC_DEBUG_FLAGS & 16: phase clocks
    DevBuf<uint8_t> overall, ba, sf;
    DevBuf<int32_t> nbytes;
    DevBuf<int64_t> off, tile_sums, grand_total, frame_off, blk_off, stream_off;
    DevBuf<int16_t> pcm_stage;
    DevBuf<int32_t> lead;                   // per-stream prior-hop frames (PAC_STREAM_HAS_PRIOR)
    DevBuf<uint8_t> out_stage;
    DevBuf<double> fsrc;
    // master
    DevBuf<double> m_thr, m_lines, m_smr, m_peak;
    DevBuf<double2> m_spec;               // [chunk][2][PAC_SPEC_LD] k_master_spec -> k_master_thr
    DevBuf<double> m_mdct;                // [2][chunk][2][1024] side kernel -> k_master_front<true>
    DevBuf<uint8_t> m_lrms, m_overall, m_ba, m_sf, m_tid;
    DevBuf<uint32_t> m_rowm;                // [nblocks] k_master_lrms -> k_master_thr row masks
    DevBuf<uint32_t> m_msm;                 // [nblocks] k_master_lrms -> k_master_front LRMS band masks
    DevBuf<uint32_t> m_mldm;                // [nblocks] the MLD rows that exist (k_master_lrms, k_master_thr -> front)
    DevBuf<uint16_t> m_codes;               // master: signed mantissa codes per line (tail -> pack; pack path only)
    DevBuf<uint16_t> m_ccodes;              // master: the chunk's codes, tail-internal (emission path)
    DevBuf<uint8_t> m_stg;                  // master: channel-blocks emitted by the tail (staging)
    DevBuf<int64_t> m_stoff;                // master: staging offset per channel-block
    DevBuf<unsigned long long> m_stg_next;  // master: staging bump allocator
    DevBuf<uint64_t> hcode;                 // [10][PAC_NSYM] (code length << 32) | code bits, 0: escape
    DevBuf<int64_t> st_extra, st_deposit;
    DevBuf<int32_t> m_perm;                 // master: streams by length within their group (run_master)
    std::vector<int32_t> h_perm;            // its host copy (lives until the async upload has run)
    DevBuf<uint32_t> dbg_mant;              // per-block API: per-line mantissas and Huffman codes
    DevBuf<uint64_t> dbg_code;
    DevBuf<uint8_t> dbg_len;
    DevBuf<uint8_t> bs_att, bs_fl;          // block switching: attack / PAC_BS_* flags per block
    DevBuf<uint8_t> dec_bsf;                // decoder: the short-frame bit per channel-block
    hipStream_t stream2 = nullptr;          // master: the reservoir tail, overlapping the next chunk
    hipStream_t stream3 = nullptr;          // master: the next chunk's LRMS decisions and spectra
    hipStream_t stream4 = nullptr;          // master: the bitstream emission of the previous chunk
    // PAC_TAIL_MODE=serial: every master kernel on `stream` in order (nothing
    // co-runs) -- the measurement baseline of run_master's pipelined placement
    bool tail_serial = false;
    int tail_wide = -1;                    // PAC_TAIL_WIDE: 0 one-lane tail only, 1 wave-per-stream only, auto
    bool side_fused = true;                // PAC_SIDE_FUSED=0: LRMS and spectra as two kernels (A/B switch)
    bool front_fast = true;                // PAC_FRONT_FAST=0: the front computes its own MDCTs (A/B switch)
    bool side_coded = true;                // PAC_SIDE_CODED=0: the front forms the coded lines (k_master_front<false>)
    bool side_early = false;               // PAC_SIDE_EARLY=1: side(i+2) beside thr(i+1), spectra double-buffered
    bool tail_early = false;               // PAC_TAIL_EARLY=1: tail(i) right after front(i) (A/B switch)
    bool mld_skip = true;                  // PAC_MLD_SKIP=0: every MLD row, the pairs in three workgroups per block
    bool front_late = false;               // PAC_FRONT_LATE=1: front(i) on s2 after side(i+1), beside thr(i+1)
                                           // (thresholds double-buffered; measured slower: thr +135 ms for a
                                           // side window -100 ms); default: on s0 beside side(i+1)
    int64_t stg_bias = 0;                  // PAC_DEBUG_STG_BIAS: staging starts this many bytes in (tests of >4 GB offsets)
    int64_t stg_cap_max = 0;               // PAC_DEBUG_STG_CAP: staging capacity cap (tests of the pack fallback)
    hipEvent_t evs[5] = {};                 // master: front/tail hand-off events (no timing)
    // decoder
    DevBuf<uint32_t> hdec_tab;              // two-level Huffman decoding tables (device)
    PacHuffDec hdec = {};
    DevBuf<uint8_t> dec_data, dec_ba, dec_sf, dec_ov, dec_lrms;
    DevBuf<uint16_t> dec_codes;
    DevBuf<int64_t> dec_so, dec_cnt, dec_cbbase, dec_cboff, dec_nblk, dec_segbase, dec_fo;
    DevBuf<int> dec_err;
    // WAV ingest / egress
    DevBuf<uint8_t> wav_blob, wav_pcm, wav_out;
    DevBuf<int64_t> wav_foff, wav_fo, wav_segb, wav_ns, wav_wo;
    DevBuf<PacWavInfo> wav_info;
    DevBuf<int16_t> dec_pcm;
    DevBuf<double> dec_fpcm;
    int64_t chunk_blocks = 0;              // blocks per pass-1 chunk; 0: run_master's default
    int dbg = 0;                           // PAC_DEBUG_FLAGS (diagnostic builds of the timing only)
    // timing
    bool timing = false;
    hipEvent_t ev[5] = {};
    std::vector<hipEvent_t> evpool;         // master: events of every chunk, read after the call
    pac_timing last = {};
    hipEvent_t pool_event(size_t i) {
        while (evpool.size() <= i) {
            hipEvent_t e = nullptr;
            hipEventCreate(&e);
            evpool.push_back(e);
        }
        return evpool[i];
    }
};

extern "C" int pac_ctx_create(int device, pac_ctx** out) {
    if (!out) return set_err(PAC_E_ARG, "null out");
    int n = 0;
    HIPCHK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return set_err(PAC_E_ARG, "device %d out of range (%d)", device, n);
    HIPCHK(hipSetDevice(device));
    pac_ctx* c = new pac_ctx();
    c->device = device;
    if (const char* f = getenv("PAC_TAIL_MODE")) c->tail_serial = !strcmp(f, "serial");
    if (const char* f = getenv("PAC_TAIL_WIDE")) c->tail_wide = atoi(f) != 0;
    if (const char* f = getenv("PAC_SIDE_FUSED")) c->side_fused = atoi(f) != 0;
    if (const char* f = getenv("PAC_FRONT_FAST")) c->front_fast = atoi(f) != 0;
    if (const char* f = getenv("PAC_SIDE_CODED")) c->side_coded = atoi(f) != 0;
    if (const char* f = getenv("PAC_SIDE_EARLY")) c->side_early = atoi(f) != 0;
    if (const char* f = getenv("PAC_TAIL_EARLY")) c->tail_early = atoi(f) != 0;
    if (const char* f = getenv("PAC_FRONT_LATE")) c->front_late = atoi(f) != 0;
    if (const char* f = getenv("PAC_MLD_SKIP")) c->mld_skip = atoi(f) != 0;
    if (const char* f = getenv("PAC_CHUNK_BLOCKS")) c->chunk_blocks = atoll(f);
    if (const char* f = getenv("PAC_DEBUG_STG_BIAS")) c->stg_bias = std::max<long long>(0, atoll(f)) & ~15ll;
    if (const char* f = getenv("PAC_DEBUG_STG_CAP")) c->stg_cap_max = std::max<long long>(0, atoll(f));
    // PAC_STREAM_PRIO (experiment): four digits, one per stream (thr/front, tail,
    // side, emit): 0 = the device's greatest priority, 1 = normal, 2 = least
    int prio[4] = {1, 1, 1, 1};
    if (const char* f = getenv("PAC_STREAM_PRIO"))
        for (int k = 0; k < 4 && f[k]; ++k) prio[k] = std::min(2, std::max(0, f[k] - '0'));
    int plo = 0, phi = 0;
    if (hipDeviceGetStreamPriorityRange(&plo, &phi) != hipSuccess) plo = phi = 0;
    auto mk_stream = [&](hipStream_t* s, int k) {
        return hipStreamCreateWithPriority(s, hipStreamNonBlocking, phi + (plo - phi) * prio[k] / 2) == hipSuccess;
    };
    const bool ok = mk_stream(&c->stream, 0) && mk_stream(&c->stream2, 1) && mk_stream(&c->stream3, 2) &&
                    mk_stream(&c->stream4, 3);
    if (!ok) {
        delete c;
        return set_err(PAC_E_HIP, "hipStreamCreate failed");
    }
    for (auto& e : c->ev) hipEventCreate(&e);
    for (auto& e : c->evs) hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (const char* f = getenv("PAC_DEBUG_FLAGS")) c->dbg = atoi(f);
    *out = c;
    return PAC_OK;
}

extern "C" void pac_ctx_destroy(pac_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    hipStreamSynchronize(c->stream2);
    hipStreamSynchronize(c->stream3);
    hipStreamSynchronize(c->stream4);
    for (auto& kv : c->tables) hipFree(kv.second);
    c->hscore.release(); c->hcode.release(); c->m_ccodes.release(); c->m_stg.release(); c->m_stoff.release();
    c->m_stg_next.release();
    c->bs_att.release(); c->bs_fl.release(); c->dec_bsf.release(); c->m_codes.release();
    if (c->huff) hipFree(c->huff);
    c->m_thr.release(); c->m_lines.release(); c->m_smr.release(); c->m_peak.release(); c->m_spec.release(); c->m_mdct.release();
    c->m_lrms.release(); c->m_rowm.release(); c->m_msm.release(); c->m_mldm.release(); c->m_overall.release(); c->m_ba.release(); c->m_sf.release();
    c->m_tid.release(); c->st_extra.release(); c->st_deposit.release(); c->m_perm.release();
    c->dbg_mant.release(); c->dbg_code.release(); c->dbg_len.release();
    c->hdec_tab.release(); c->dec_data.release(); c->dec_ba.release(); c->dec_sf.release();
    c->dec_ov.release(); c->dec_lrms.release(); c->dec_codes.release(); c->dec_so.release();
    c->dec_cnt.release(); c->dec_cbbase.release(); c->dec_cboff.release(); c->dec_nblk.release();
    c->dec_segbase.release(); c->dec_fo.release(); c->dec_err.release();
    c->wav_blob.release(); c->wav_pcm.release(); c->wav_out.release(); c->wav_foff.release();
    c->wav_fo.release(); c->wav_segb.release(); c->wav_ns.release(); c->wav_wo.release(); c->wav_info.release(); c->dec_pcm.release(); c->dec_fpcm.release();
    c->smr.release(); c->bandpeak.release(); c->overall.release(); c->ba.release(); c->prof.release();
    c->sf.release(); c->nbytes.release(); c->off.release(); c->tile_sums.release();
    c->grand_total.release(); c->frame_off.release(); c->blk_off.release();
    c->stream_off.release(); c->lead.release(); c->pcm_stage.release(); c->out_stage.release(); c->fsrc.release();
    for (auto& e : c->ev) hipEventDestroy(e);
    for (auto& e : c->evpool) hipEventDestroy(e);
    for (auto& e : c->evs) hipEventDestroy(e);
    hipStreamDestroy(c->stream);
    hipStreamDestroy(c->stream2);
    hipStreamDestroy(c->stream3);
    hipStreamDestroy(c->stream4);
    delete c;
}

static int get_tables(pac_ctx* c, int fs, int window, PacTables** out) {
    const int key = fs * 4 + window;
    auto it = c->tables.find(key);
    if (it != c->tables.end()) {
        *out = it->second;
        return PAC_OK;
    }
    PacTables* h = (PacTables*)malloc(sizeof(PacTables));
    if (!h) return set_err(PAC_E_NOMEM, "host tables");
    build_tables(fs, window, h);
    if (h->lr_nleaf > 64) {
        free(h);
        return set_err(PAC_E_UNSUPPORTED, "band layout of %d Hz needs more than 64 pairwise-sum leaves", fs);
    }
    PacTables* d = nullptr;
    if (hipMalloc((void**)&d, sizeof(PacTables)) != hipSuccess) {
        free(h);
        return set_err(PAC_E_NOMEM, "device tables");
    }
    hipError_t e = hipMemcpy(d, h, sizeof(PacTables), hipMemcpyHostToDevice);
    free(h);
    if (e != hipSuccess) return set_err(PAC_E_HIP, "table upload: %s", hipGetErrorString(e));
    c->tables[key] = d;
    *out = d;
    return PAC_OK;
}

extern "C" int pac_huffman_load(pac_ctx* c, const uint8_t* buf, int64_t len) {
    if (!c || !buf) return set_err(PAC_E_ARG, "null argument");
    if (len < 12 || memcmp(buf, "PACHUF01", 8) != 0) return set_err(PAC_E_TABLES, "not a PACHUF01 image");
    uint32_t n;
    memcpy(&n, buf + 8, 4);
    if (n != PAC_NTAB) return set_err(PAC_E_TABLES, "expected %d tables, image has %u", PAC_NTAB, n);
    PacHuffTables* h = (PacHuffTables*)calloc(1, sizeof(PacHuffTables));
    if (!h) return set_err(PAC_E_NOMEM, "host huffman tables");
    int64_t o = 12;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t hdr[4];
        if (o + 16 > len) { free(h); return set_err(PAC_E_TABLES, "truncated image"); }
        memcpy(hdr, buf + o, 16);
        o += 16;
        uint32_t tid = hdr[0];
        if (tid < 1 || tid > PAC_NTAB || hdr[2] < 1 || hdr[2] > 32) {
            free(h);
            return set_err(PAC_E_TABLES, "bad table header");
        }
        h->esc_len[tid - 1] = (int32_t)hdr[2];
        h->esc_bits[tid - 1] = hdr[3];
        for (uint32_t e = 0; e < hdr[1]; e++) {
            int32_t sym;
            uint32_t l, b;
            if (o + 12 > len) { free(h); return set_err(PAC_E_TABLES, "truncated image"); }
            memcpy(&sym, buf + o, 4);
            memcpy(&l, buf + o + 4, 4);
            memcpy(&b, buf + o + 8, 4);
            o += 12;
            if (sym < 0 || sym >= PAC_NSYM || l < 1 || l > 32) {
                free(h);
                return set_err(PAC_E_TABLES, "bad table entry");
            }
            h->len[tid - 1][sym] = (uint8_t)l;
            h->bits[tid - 1][sym] = b;
        }
    }
    for (int sym = 0; sym < PAC_NSYM; sym++)
        for (int t = 0; t < PAC_NTAB; t++)
            if (h->len[t][sym] > 30) {     // the pack's 64-bit bit windows and the 16-bit scoring sums assume it
                free(h);
                return set_err(PAC_E_TABLES, "code longer than 30 bits");
            }
    // the tail's scoring table: for each ba = 2..16 and symbol < 2^(ba-1), the
    // ten tables' code lengths, or escape length + ba (Huffman.py:284-300)
    std::vector<uint32_t> hs((size_t)PAC_HSC_N * PAC_HSC_W, 0u);
    for (int ba = 2; ba <= 16; ba++)
        for (int sym = 0; sym < (1 << (ba - 1)); sym++) {
            uint32_t* ent = hs.data() + (size_t)(((1 << (ba - 1)) - 2) + sym) * PAC_HSC_W;
            for (int t = 0; t < PAC_NTAB; t++) {
                const uint32_t cost = h->len[t][sym] ? h->len[t][sym] : (uint32_t)(h->esc_len[t] + ba);
                ent[t >> 1] |= cost << (16 * (t & 1));
            }
        }
    HIPCHK(hipSetDevice(c->device));
    int rc3;
    if ((rc3 = c->hscore.ensure(hs.size()))) { free(h); return rc3; }
    if (hipMemcpy(c->hscore.p, hs.data(), hs.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
        free(h);
        return set_err(PAC_E_HIP, "huffman scoring table upload");
    }
    std::vector<uint64_t> hc((size_t)PAC_NTAB * PAC_NSYM, 0ull);
    for (int t = 0; t < PAC_NTAB; t++)
        for (int sym = 0; sym < PAC_NSYM; sym++)
            if (h->len[t][sym]) hc[(size_t)t * PAC_NSYM + sym] = ((uint64_t)h->len[t][sym] << 32) | h->bits[t][sym];
    if ((rc3 = c->hcode.ensure(hc.size()))) { free(h); return rc3; }
    if (hipMemcpy(c->hcode.p, hc.data(), hc.size() * sizeof(uint64_t), hipMemcpyHostToDevice) != hipSuccess) {
        free(h);
        return set_err(PAC_E_HIP, "huffman code table upload");
    }
    if (!c->huff && hipMalloc((void**)&c->huff, sizeof(PacHuffTables)) != hipSuccess) {
        free(h);
        return set_err(PAC_E_NOMEM, "device huffman tables");
    }
    int rc2;
    hipError_t e = hipMemcpy(c->huff, h, sizeof(PacHuffTables), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        free(h);
        return set_err(PAC_E_HIP, "huffman upload: %s", hipGetErrorString(e));
    }
    // decoding tables (Huffman.decodeData, Huffman.py:321-344): level 1 on the
    // first min(11, maxlen) bits, level 2 for longer codes
    std::vector<uint32_t> tab;
    for (int t = 0; t < PAC_NTAB; t++) {
        int ml = h->esc_len[t];
        for (int sym = 0; sym < PAC_NSYM; sym++) ml = std::max(ml, (int)h->len[t][sym]);
        if (ml > 30) {
            free(h);
            return set_err(PAC_E_TABLES, "code longer than 30 bits");
        }
        const int l1 = std::min(ml, 11), l2 = ml - l1;
        const size_t base = tab.size();
        tab.resize(base + ((size_t)1 << l1), 0u);
        for (int sym = -1; sym < PAC_NSYM; sym++) {
            const int len = sym < 0 ? h->esc_len[t] : h->len[t][sym];
            if (!len) continue;
            const uint32_t code = sym < 0 ? h->esc_bits[t] : h->bits[t][sym];
            const uint32_t ent = ((uint32_t)len << 16) | (sym < 0 ? 0xffffu : (uint32_t)sym);
            if (len <= l1) {
                const uint32_t first = code << (l1 - len), n = 1u << (l1 - len);
                for (uint32_t i = 0; i < n; i++) tab[base + first + i] = ent;
            } else {
                const uint32_t top = code >> (len - l1);
                uint32_t& slot = tab[base + top];
                if (!(slot >> 31)) {
                    const size_t sub = tab.size();
                    tab.resize(sub + ((size_t)1 << l2), 0u);
                    tab[base + top] = 0x80000000u | (uint32_t)sub;
                }
                const size_t sub = tab[base + top] & 0x7fffffffu;
                const uint32_t rest = code & ((1u << (len - l1)) - 1u);
                const uint32_t first = rest << (ml - len), n = 1u << (ml - len);
                for (uint32_t i = 0; i < n; i++) tab[sub + first + i] = ent;
            }
        }
        c->hdec.base[t] = (int32_t)base;
        c->hdec.maxlen[t] = ml;
        c->hdec.l1[t] = l1;
    }
    // the short-code table (PacHuffDec.sbase): every code of at most
    // PAC_DEC_SBITS bits over all its PAC_DEC_SBITS-bit extensions
    c->hdec.sbase = (int32_t)tab.size();
    tab.resize(tab.size() + ((size_t)PAC_NTAB << PAC_DEC_SBITS), 0x80000000u);
    for (int t = 0; t < PAC_NTAB; t++)
        for (int sym = -1; sym < PAC_NSYM; sym++) {
            const int len = sym < 0 ? h->esc_len[t] : h->len[t][sym];
            if (!len || len > PAC_DEC_SBITS) continue;
            const uint32_t code = sym < 0 ? h->esc_bits[t] : h->bits[t][sym];
            const uint32_t ent = ((uint32_t)len << 16) | (sym < 0 ? 0xffffu : (uint32_t)sym);
            const uint32_t first = code << (PAC_DEC_SBITS - len), n = 1u << (PAC_DEC_SBITS - len);
            for (uint32_t i = 0; i < n; i++) tab[c->hdec.sbase + ((size_t)t << PAC_DEC_SBITS) + first + i] = ent;
        }
    free(h);
    if ((rc2 = c->hdec_tab.ensure(tab.size()))) return rc2;
    HIPCHK(hipMemcpy(c->hdec_tab.p, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    c->have_huff = true;
    return PAC_OK;
}

static int check_params(const pac_params* p) {
    if (!p) return set_err(PAC_E_ARG, "null params");
    if (p->n_mdct_lines != 1024 || p->n_scale_bits != 4 || p->n_mant_size_bits != 4)
        return set_err(PAC_E_UNSUPPORTED,
                       "only nMDCTLines=1024, nScaleBits=4, nMantSizeBits=4 (pacfile.py:452-454)");
    if (p->sample_rate < PAC_N || p->sample_rate > 400000)
        return set_err(PAC_E_UNSUPPORTED, "sample rate %d", p->sample_rate);
    if (p->profile == PAC_PROFILE_ORIGIN) {
        if (p->n_channels < 1 || p->n_channels > 8) return set_err(PAC_E_ARG, "n_channels %d", p->n_channels);
    } else if (p->profile == PAC_PROFILE_MASTER) {
        // the reference's master coder is stereo only (codec.py:46-47,98); one
        // channel is this build's extension (LRMS all 0, parity unpinned)
        if (p->n_channels != 2 && p->n_channels != 1)
            return set_err(PAC_E_UNSUPPORTED, "master coder: 1 or 2 channels (codec.py:46-47,98)");
        if (p->n_table_id_bits != 4) return set_err(PAC_E_UNSUPPORTED, "nTableIDBits must be 4");
    } else {
        return set_err(PAC_E_ARG, "unknown profile %d", p->profile);
    }
    if (!(p->target_bits_per_sample > 0.0)) return set_err(PAC_E_ARG, "targetBitsPerSample");
    if (p->window != PAC_WINDOW_SINE && p->window != PAC_WINDOW_KBD) return set_err(PAC_E_ARG, "window %d", p->window);
    if (p->block_switch != 0 && p->block_switch != 1) return set_err(PAC_E_ARG, "block_switch %d", p->block_switch);
    if (p->block_switch && p->profile != PAC_PROFILE_MASTER)
        return set_err(PAC_E_UNSUPPORTED, "block switching is built for the master profile");
    return PAC_OK;
}

// bitBudget as codec.py:223-227 / Origin codec.py:86-88 compute it, same op order
static double bit_budget(const pac_params* p) {
    double b = p->target_bits_per_sample * 1024;
    b -= p->n_scale_bits * (PAC_NB + 1);
    b -= p->n_mant_size_bits * PAC_NB;
    if (p->profile == PAC_PROFILE_MASTER) b -= p->n_table_id_bits;
    return b;
}

// worst-case bytes of one channel-block: '<L' + payload.  Origin: 4 + 25*8 +
// 16*1024 bits; master: PAC_MASTER_MAX_BITS (sign + code <= 47 bits per line)
static int64_t pac_encode_bound_per_channel_block(int profile) {
    const int64_t bits = profile == PAC_PROFILE_MASTER ? (int64_t)PAC_MASTER_MAX_BITS
                                                       : (int64_t)(4 + PAC_NB * 8 + 16 * PAC_HALFN);
    return 4 + (bits + 7) / 8;
}

extern "C" int64_t pac_encode_bound(const pac_params* p, int32_t n_streams, const int64_t* fo) {
    if (!p || !fo || n_streams < 0) return -1;
    int64_t blocks = 0;
    for (int s = 0; s < n_streams; s++) blocks += (fo[s + 1] - fo[s] + PAC_HALFN - 1) / PAC_HALFN + 1;
    return blocks * p->n_channels * pac_encode_bound_per_channel_block(p->profile);
}

__global__ void k_stream_offsets(const int64_t* __restrict__ off, const int64_t* __restrict__ blk_off,
                                 int n_streams, int nch, const int64_t* __restrict__ total,
                                 int64_t* __restrict__ so) {
    int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n_streams) so[s] = off[blk_off[s] * nch];
    if (s == n_streams) so[s] = *total;
}

// diagnostic: mean shader-clock cycles per phase of k_origin_front over the
// sampled workgroups (per wave, and the spread between a workgroup's waves)
static int report_phase_clocks(pac_ctx* c, hipStream_t s, int64_t n) {
    std::vector<long long> h(n);
    HIPCHK(hipMemcpyAsync(h.data(), c->prof.p, n * sizeof(long long), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    double mean[PAC_PROF_MARKS] = {0}, spread[PAC_PROF_MARKS] = {0};
    int64_t cnt = 0;
    for (int64_t g = 0; g < PAC_PROF_WG; g++) {
        const long long* t = &h[g * 4 * PAC_PROF_MARKS];
        if (!t[0]) continue;
        cnt++;
        for (int k = 1; k < 9; k++) {
            long long mx = 0, mn = 0;
            for (int w = 0; w < 4; w++) {
                long long d = t[w * PAC_PROF_MARKS + k] - t[w * PAC_PROF_MARKS + k - 1];
                mean[k] += d / 4.0;
                if (w == 0 || d > mx) mx = d;
                if (w == 0 || d < mn) mn = d;
            }
            spread[k] += (double)(mx - mn);
        }
    }
    if (!cnt) return PAC_OK;
    fprintf(stderr, "PAC_PROF %lld workgroups, mean cycles per phase (wave mean / max-min spread):\n",
            (long long)cnt);
    for (int k = 1; k < 9; k++)
        fprintf(stderr, "  phase %d: %10.0f  %10.0f\n", k, mean[k] / cnt, spread[k] / cnt);
    // masking rows: wave w, i-th row (end of previous row or mark 5 to mark 10+i)
    double row[4][4] = {{0}};
    for (int64_t g = 0; g < PAC_PROF_WG; g++) {
        const long long* t = &h[g * 4 * PAC_PROF_MARKS];
        if (!t[0]) continue;
        for (int w = 0; w < 4; w++)
            for (int i = 0; i < 4; i++)
                row[w][i] += (double)(t[w * PAC_PROF_MARKS + 10 + i] -
                                      t[w * PAC_PROF_MARKS + (i ? 9 + i : 5)]);
    }
    for (int w = 0; w < 4; w++)
        fprintf(stderr, "  wave %d rows: %9.0f %9.0f %9.0f %9.0f\n", w, row[w][0] / cnt, row[w][1] / cnt,
                row[w][2] / cnt, row[w][3] / cnt);
    return PAC_OK;
}

// diagnostic build (-DPAC_ROWPROF): masking-row statistics of the last call
static int report_rowprof(pac_ctx* c, hipStream_t s) {
#ifdef PAC_ROWPROF
    std::vector<unsigned long long> all(1024 * 16);
    unsigned long long rp[16] = {0};
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipMemcpyFromSymbol(all.data(), HIP_SYMBOL(pac_rowprof), all.size() * 8));
    for (int i = 0; i < 1024 * 16; i++) rp[i % 16] += all[i];
    const double n = (double)(rp[0] ? rp[0] : 1);
    fprintf(stderr, "ROWPROF rows %llu  cyc zones %.0f skip %.0f mom %.0f direct+rag %.0f | nm %.1f nloud %.1f "
            "momrows %.3f D %.2f mom_n %.1f rag %.1f m0 %.1f umax %.1f\n",
            rp[0], rp[1] / n, rp[2] / n, rp[3] / n, rp[4] / n, rp[5] / n, rp[6] / n, rp[7] / n,
            rp[8] / (double)(rp[7] ? rp[7] : 1), rp[9] / n, rp[10] / n, rp[11] / n, rp[12] / n);
    std::fill(all.begin(), all.end(), 0ull);
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(pac_rowprof), all.data(), all.size() * 8));
#else
    (void)c;
    (void)s;
#endif
    return PAC_OK;
}

static int run_origin(pac_ctx* c, const pac_params* p, PacTables* T, PacSource src, int64_t G,
                      uint8_t* out_dev, int64_t out_cap, int64_t* out_total, int64_t** off_dev) {
    int rc;
    if ((rc = c->smr.ensure(PAC_NB * G)) || (rc = c->bandpeak.ensure(PAC_NB * G)) ||
        (rc = c->overall.ensure(G)) || (rc = c->ba.ensure(PAC_NB * G)) || (rc = c->sf.ensure(PAC_NB * G)) ||
        (rc = c->nbytes.ensure(G)) || (rc = c->off.ensure(G + 1)) ||
        (rc = c->tile_sums.ensure((G + SCAN_TILE - 1) / SCAN_TILE + 1)) || (rc = c->grand_total.ensure(1)))
        return rc;
    PacOriginWork W{c->smr.p, c->bandpeak.p, c->overall.p, c->ba.p, c->sf.p, c->nbytes.p};
    hipStream_t s = c->stream;
    if (c->timing) HIPCHK(hipEventRecord(c->ev[0], s));
    const int64_t nprof = (int64_t)PAC_PROF_WG * 4 * PAC_PROF_MARKS;
    if (c->dbg & 16) {
        if ((rc = c->prof.ensure(nprof))) return rc;
        HIPCHK(hipMemsetAsync(c->prof.p, 0, nprof * sizeof(long long), s));
        src.prof = c->prof.p;
    }
    hipLaunchKernelGGL(k_origin_front, dim3((unsigned)G), dim3(FRONT_NT), 0, s, src, T, W, G);
    HIPCHK(hipGetLastError());
    if (c->dbg & 16) report_phase_clocks(c, s, nprof);
    if (c->timing) HIPCHK(hipEventRecord(c->ev[1], s));
    hipLaunchKernelGGL(k_origin_alloc, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, s, T, W, G,
                       bit_budget(p), 16);
    HIPCHK(hipGetLastError());
    if (c->timing) HIPCHK(hipEventRecord(c->ev[2], s));
    int64_t ntiles = (G + SCAN_TILE - 1) / SCAN_TILE;
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)ntiles), dim3(256), 0, s, c->nbytes.p, G, c->tile_sums.p);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(256), 0, s, c->tile_sums.p, ntiles, c->grand_total.p);
    hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)ntiles), dim3(256), 0, s, c->nbytes.p, G, c->tile_sums.p,
                       c->off.p);
    HIPCHK(hipGetLastError());
    if (c->timing) HIPCHK(hipEventRecord(c->ev[3], s));
    // no host round trip inside the pipeline: the pack kernel skips any
    // channel-block that would end past out_cap, the caller checks the total
    // (c->grand_total) after the call and reports PAC_E_CAPACITY
    hipLaunchKernelGGL(k_origin_pack, dim3((unsigned)G), dim3(FRONT_NT), 0, s, src, T, W, G, c->off.p, out_dev,
                       out_cap);
    HIPCHK(hipGetLastError());
    if (c->timing) HIPCHK(hipEventRecord(c->ev[4], s));
    HIPCHK(hipMemcpyAsync(out_total, c->grand_total.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    *off_dev = c->off.p;
    return PAC_OK;
}

static void finish_timing(pac_ctx* c, int64_t G, int64_t bytes) {
    if (!c->timing) return;
    c->last.thr_ms = 0.f;
    c->last.lrms_ms = 0.f;
    c->last.thr_short_ms = 0.f;
    c->last.spec_ms = 0.f;
    c->last.emit_ms = 0.f;
    hipEventSynchronize(c->ev[4]);
    hipEventElapsedTime(&c->last.front_ms, c->ev[0], c->ev[1]);
    hipEventElapsedTime(&c->last.alloc_ms, c->ev[1], c->ev[2]);
    hipEventElapsedTime(&c->last.scan_ms, c->ev[2], c->ev[3]);
    hipEventElapsedTime(&c->last.pack_ms, c->ev[3], c->ev[4]);
    hipEventElapsedTime(&c->last.total_ms, c->ev[0], c->ev[4]);
    c->last.n_channel_blocks = G;
    c->last.out_bytes = bytes;
}

// --- master: two passes, chunks of whole-block ranges ---------------------

// Runs the master pipeline over global blocks [0, nblocks).  States (device
// st_extra / st_deposit, per stream) must be initialised by the caller on
// c->stream.  Pass 1: streams in groups of at most chunk_blocks, each group
// swept in time slices of S blocks per stream (S * streams <= chunk_blocks)
// so every stream's serial reservoir chain advances in parallel; thresholds +
// front on c->stream, the tail of the same chunk on c->stream2 while the next
// chunk's thresholds run (chunk outputs double-buffered, ordered by events).
// Pass 2: exclusive scan of the channel-block byte counts (file order) ->
// final offsets, then k_master_pack writes every channel-block in place.
// No host synchronisation inside the pipeline.  Leaves the offsets in c->off
// and the total (async) in *out_total.
// pack = false: the tail emits every channel-block into the staging buffer
// and k_master_place copies them to their offsets; *stg_need (host, async)
// receives the staging bytes it used -- more than *stg_cap means some were
// not emitted and the caller re-runs with pack = true.  pack = true (and the
// per-block API's debug codes): the tail stores the mantissa codes of every
// channel-block and k_master_pack packs them.
static int run_master(pac_ctx* c, const pac_params* p, PacTables* T, PacSource src,
                      const std::vector<int64_t>& blk, uint8_t* out_dev, int64_t out_cap,
                      int64_t* out_total, bool dbg_codes, bool pack = true, uint64_t* stg_need = nullptr,
                      int64_t* stg_cap = nullptr) {
    int rc;
    const int n_streams = src.n_streams;
    const int64_t nblocks = blk[n_streams];
    const int nch = src.n_ch;                          // 2, or 1 (mono master extension)
    const int64_t G = nch * nblocks;
    const int nvar = nch == 2 ? 6 : 1;                 // threshold variants per block
    // blocks per chunk: PAC_CHUNK_BLOCKS / pac_set_chunk_blocks, else 32768 (65536 with
    // block switching) -- measured: configs[2] 6.88 -> 6.97 M blocks/s and configs[3]
    // 6.27 -> 6.59 M against 65536; configs[4] 5.39 M at 65536 against 5.30 M
    const int64_t CB = c->chunk_blocks > 0 ? c->chunk_blocks : p->block_switch ? 65536 : 32768;
    if (CB > PAC_CHUNK_MAX) return set_err(PAC_E_ARG, "chunk_blocks (PAC_CHUNK_BLOCKS) above PAC_CHUNK_MAX (131071)");
    // chunk geometry: groups [g0, g1) of at most CB streams, each ordered by
    // length (longest first, perm); chunk = blocks t0 .. t0+S-1 of the
    // group's streams still running at t0 (a prefix of that order), S =
    // CB / (running streams) -- ragged stream sets keep their chunks full
    std::vector<int32_t>& perm = c->h_perm;
    perm.assign(n_streams, 0);
    struct Chunk { PacMasterChunk ck; int64_t B; int n_s; };
    std::vector<Chunk> chunks;
    int64_t cbmax = 1;
    for (int g0 = 0; g0 < n_streams;) {
        const int g1 = (int)std::min<int64_t>(n_streams, g0 + CB);
        for (int k = g0; k < g1; k++) perm[k] = k;
        std::stable_sort(perm.begin() + g0, perm.begin() + g1,
                         [&](int a, int b) { return blk[a + 1] - blk[a] > blk[b + 1] - blk[b]; });
        const int64_t gmax = std::max<int64_t>(1, blk[perm[g0] + 1] - blk[perm[g0]]);
        int n_act = g1 - g0;
        for (int64_t t0 = 0; t0 < gmax;) {
            while (n_act > 1 && blk[perm[g0 + n_act - 1] + 1] - blk[perm[g0 + n_act - 1]] <= t0) n_act--;
            const int S = (int)std::max<int64_t>(1, std::min<int64_t>(CB / n_act, gmax - t0));
            chunks.push_back({PacMasterChunk{g0, n_act, t0, S, nch, nullptr}, (int64_t)n_act * S, n_act});
            cbmax = std::max<int64_t>(cbmax, (int64_t)n_act * S);
            t0 += S;
        }
        g0 = g1;
    }
    if ((rc = c->m_perm.ensure(n_streams + 1))) return rc;
    HIPCHK(hipMemcpyAsync(c->m_perm.p, perm.data(), n_streams * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    for (Chunk& q : chunks) q.ck.perm = c->m_perm.p;
    // the MLD skip, pipelined (k_master_thr mode 1): the threshold launch of
    // chunk i also runs chunk i-1's MLD rows, the front of chunk i-1 follows it;
    // thresholds and spectra double-, MDCT lines triple-buffered
    const bool pipe = c->mld_skip && nch == 2 && !c->side_early && !c->front_late && !c->tail_serial;
    if ((rc = c->m_lrms.ensure(nblocks * PAC_NB + 1)) || (rc = c->m_rowm.ensure(nblocks + 1)) || (rc = c->m_msm.ensure(nblocks + 1)) || (rc = c->m_mldm.ensure(nblocks + 1)) || (rc = c->m_overall.ensure(G + 1)) ||
        (rc = c->m_ba.ensure(G * PAC_NB + 1)) || (rc = c->m_sf.ensure(G * PAC_NB + 1)) ||
        (rc = c->m_tid.ensure(G + 1)) || (rc = c->nbytes.ensure(G + 1)) || (rc = c->off.ensure(G + 1)) ||
        (rc = c->tile_sums.ensure((G + SCAN_TILE - 1) / SCAN_TILE + 1)) || (rc = c->grand_total.ensure(1)) ||
        (rc = c->m_thr.ensure((c->front_late || pipe ? 2 : 1) * cbmax * 6 * PAC_HALFN)) || (rc = c->m_spec.ensure((c->side_early || pipe ? 2 : 1) * cbmax * 2 * PAC_SPEC_LD)) || (rc = c->m_lines.ensure(3 * cbmax * 2 * PAC_HALFN)) ||
        (rc = c->m_smr.ensure(3 * cbmax * 2 * PAC_NB)) || (rc = c->m_peak.ensure(3 * cbmax * 2 * PAC_NB)))
        return rc;
    pack = pack || dbg_codes;
    PacMasterFields F{c->m_lrms.p, c->m_overall.p, c->m_ba.p, c->m_sf.p, c->m_tid.p, c->nbytes.p,
                      nullptr, nullptr, nullptr, nullptr, nullptr, c->m_rowm.p, nullptr, nullptr, nullptr, 0,
                      c->m_msm.p, c->m_mldm.p};
    if (pack) {
        if ((rc = c->m_codes.ensure(G * PAC_HALFN))) return rc;   // 2 KB per channel-block: tail -> pack
        F.codes = c->m_codes.p;
    } else {
        // staging: the output's capacity (at most a 1.5 KB average per
        // channel-block -- the bit budget gives ~300 B) + the burst
        // padding per channel-block (k_master_emit); a larger need is detected after the call
        int64_t cap = std::min<int64_t>(out_cap, G * 1536) + 4 * PAC_EMIT_WORDS * G + 64 + c->stg_bias;
        if (c->stg_cap_max > 0) cap = std::min<int64_t>(cap, c->stg_bias + c->stg_cap_max);
        if ((rc = c->m_ccodes.ensure(2 * cbmax * 2 * PAC_HALFN)) || (rc = c->m_stg.ensure(cap)) ||
            (rc = c->m_stoff.ensure(G + 1)) || (rc = c->m_stg_next.ensure(1)))
            return rc;
        F.stg = c->m_stg.p;
        F.stoff = c->m_stoff.p;
        F.stg_next = c->m_stg_next.p;
        F.stg_cap = cap;
        const unsigned long long bias = (unsigned long long)c->stg_bias;
        HIPCHK(hipMemcpyAsync(c->m_stg_next.p, &bias, sizeof(bias), hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));   // `bias` is a stack value
        if (stg_cap) *stg_cap = cap;
    }
    if (p->block_switch) {     // pac_bs.h: attack flags, then each block's PAC_BS_* flags
        if ((rc = c->bs_att.ensure(nblocks + 1)) || (rc = c->bs_fl.ensure(nblocks + 1))) return rc;
        hipLaunchKernelGGL(k_bs_attack, dim3((unsigned)((nblocks + 1) / 2)), dim3(64), 0, c->stream, src, nblocks,
                           c->bs_att.p);
        hipLaunchKernelGGL(k_bs_flags, dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, c->stream,
                           src.blk_off, n_streams, nblocks, c->bs_att.p, c->bs_fl.p);
        HIPCHK(hipGetLastError());
        F.bsf = c->bs_fl.p;
    }
    // the MDCT lines from the side kernel's LRMS spectra (mdct_from_dft): sine
    // window, stereo.  Without block switching the side kernel forms the coded
    // lines themselves (k_master_lrms_spec<true>: K.lines, with the overall
    // scale factors) and k_master_front<true> reads them and stores none
    // (front_fast); otherwise k_master_front<false> reads the side kernel's
    // MDCT lines (K.mdct; with block switching those of the plain long
    // frames) and transforms the others itself
    const bool side_mdct = c->front_fast && nch == 2 && p->window == PAC_WINDOW_SINE && c->side_fused;
    const bool front_fast = side_mdct && !F.bsf && c->side_coded;
    const bool side_md = side_mdct && !front_fast;
    if (side_md && (rc = c->m_mdct.ensure((pipe ? 3 : 2) * cbmax * 2 * PAC_HALFN))) return rc;
    if (dbg_codes) {
        if ((rc = c->dbg_mant.ensure(G * PAC_HALFN)) || (rc = c->dbg_code.ensure(G * PAC_HALFN)) ||
            (rc = c->dbg_len.ensure(G * PAC_HALFN)))
            return rc;
        F.dbg_mant = c->dbg_mant.p;
        F.dbg_code = c->dbg_code.p;
        F.dbg_len = c->dbg_len.p;
    }
    // Streams: s0 the thresholds and the front (the critical path), s2 the
    // LRMS decisions and spectra of the NEXT chunk, s1 the reservoir tail.
    // Per chunk i (buffer set k = i % 3 of the front -> tail outputs):
    //   s0: thr(i) -> front(i) -> [wait spec(i+1)] -> thr(i+1) ...
    //   s2: [wait thr(i): the spectrum buffer is free] lrms(i+1) -> spec(i+1)
    //   s1: [wait front(i), spec(i+1)] tail(i), beside thr(i+1)
    // lrms/spec of the next chunk thus co-run with front(i) (three
    // latency-bound kernels filling each other's issue gaps), and the tail
    // (<= 96 VGPRs, one wave per workgroup) takes the fifth wave slot of a
    // SIMD next to 4 threshold waves (104 VGPRs each) without displacing one.
    // PAC_TAIL_MODE=serial: every kernel on s0 in order (the baseline).
    const bool serial = c->tail_serial;
    hipStream_t s0 = c->stream, s1 = serial ? c->stream : c->stream2, s2 = serial ? c->stream : c->stream3;
    hipStream_t s3 = serial ? c->stream : c->stream4;
    const double budget = bit_budget(p);
    // timing: events recorded around every launch on its own stream, read
    // once after the call; mk[k] = (pool event, phase) of stream k, phase -1
    // opens an interval, phase >= 0 closes one
    std::vector<std::pair<size_t, int>> mk[4];
    size_t nev = 0;
    auto mark = [&](int k, int phase) -> int {
        if (!c->timing) return PAC_OK;
        const hipEvent_t e = c->pool_event(nev);
        mk[k].emplace_back(nev++, phase);
        HIPCHK(hipEventRecord(e, k == 3 ? s3 : k == 2 ? s2 : (k ? s1 : s0)));
        return PAC_OK;
    };
    // a fresh ordering event (no timing); a failed record would only show as a
    // wrong order, so the first failure is kept and the call fails with it
    hipError_t ev_err = hipSuccess;
    auto event_on = [&](hipStream_t st) -> hipEvent_t {
        const hipEvent_t e = c->pool_event(nev++);
        const hipError_t r = hipEventRecord(e, st);
        if (r != hipSuccess && ev_err == hipSuccess) ev_err = r;
        return e;
    };
    // mono: the LRMS flags are all 0 (L/R coding; the 25 bits are still written)
    if (nch == 1) HIPCHK(hipMemsetAsync(c->m_lrms.p, 0, nblocks * PAC_NB, s0));
    {
        const hipEvent_t e = event_on(s0);            // states and tables are on s0
        HIPCHK(hipStreamWaitEvent(s1, e, 0));
        HIPCHK(hipStreamWaitEvent(s2, e, 0));
        HIPCHK(hipStreamWaitEvent(s3, e, 0));
    }
    const int64_t nck = (int64_t)chunks.size();
    c->last.chunks = (int32_t)nck;
    // front(i) after side(i+1) on s2, beside thr(i+1) (thresholds double-buffered):
    // the window between two threshold launches is the side kernel alone
    const bool late = c->front_late && !c->side_early && !serial;
    auto bufset = [&](int64_t i) {
        const int64_t k = i % 3;
        return PacMasterChunkBuf{c->m_thr.p + (late || pipe ? (i & 1) * cbmax * 6 * PAC_HALFN : 0),
                                 c->m_lines.p + k * cbmax * 2 * PAC_HALFN,
                                 c->m_smr.p + k * cbmax * 2 * PAC_NB, c->m_peak.p + k * cbmax * 2 * PAC_NB,
                                 c->m_spec.p + (c->side_early || pipe ? (i & 1) * cbmax * 2 * PAC_SPEC_LD : 0),
                                 c->m_ccodes.p + (i & 1) * cbmax * 2 * PAC_HALFN,
                                 side_md ? c->m_mdct.p + (pipe ? i % 3 : i & 1) * cbmax * 2 * PAC_HALFN : nullptr};
    };
    // PAC_DEBUG_FLAGS 32: phase clocks of the fused LRMS + spectra kernel, 64: of the front
    // 128: of the thresholds
    PacSource src_side = src, src_front = src, src_thr = src;
    const int64_t nprof = (int64_t)PAC_PROF_WG * 4 * PAC_PROF_MARKS;
    if (c->dbg & (32 | 64 | 128)) {
        if ((rc = c->prof.ensure(nprof))) return rc;
        HIPCHK(hipMemsetAsync(c->prof.p, 0, nprof * sizeof(long long), s0));
        HIPCHK(hipStreamWaitEvent(s2, event_on(s0), 0));
        if (c->dbg & 32) src_side.prof = c->prof.p;
        else if (c->dbg & 64) src_front.prof = c->prof.p;
        else src_thr.prof = c->prof.p;
    }
    std::vector<hipEvent_t> tail_done(nck, nullptr), emit_done(nck, nullptr), spec_ev(nck + 1, nullptr);
    auto launch_side = [&](int64_t i) -> int {         // lrms(i), spec(i) on s2
        int rc2;
        const Chunk& q = chunks[i];
        const PacMasterChunkBuf K = bufset(i);
        // front_fast: the side kernel writes line set i % 3, whose last reader
        // was the tail of chunk i - 3 (recorded before this launch in every
        // schedule; it ran beside an earlier threshold launch).  A schedule
        // that launches the side kernel first would race on K.lines: refused.
        if (front_fast && i >= 3) {
            if (!tail_done[i - 3])
                return set_err(PAC_E_HIP, "internal: side kernel of chunk %lld before the tail of chunk %lld",
                               (long long)i, (long long)(i - 3));
            HIPCHK(hipStreamWaitEvent(s2, tail_done[i - 3], 0));
        }
        if ((rc2 = mark(2, -1))) return rc2;
        if (c->side_fused) {          // timed as the spectra phase (spec_ms), lrms_ms = 0
            if (front_fast)
                hipLaunchKernelGGL(k_master_lrms_spec<true>, dim3((unsigned)q.B), dim3(256), 0, s2, src_side, T, K, F,
                                   q.ck);
            else
                hipLaunchKernelGGL(k_master_lrms_spec<false>, dim3((unsigned)q.B), dim3(256), 0, s2, src_side, T, K, F,
                                   q.ck);
            HIPCHK(hipGetLastError());
            return mark(2, 7);
        }
        if (nch == 2) hipLaunchKernelGGL(k_master_lrms, dim3((unsigned)q.B), dim3(256), 0, s2, src, T, F, q.ck);
        if ((rc2 = mark(2, 5))) return rc2;
        hipLaunchKernelGGL(k_master_spec, dim3((unsigned)q.B), dim3(256), 0, s2, src, T, K, F, q.ck);
        HIPCHK(hipGetLastError());
        if ((rc2 = mark(2, 7))) return rc2;
        return PAC_OK;
    };
    const bool early = c->side_early && !serial;
    if ((rc = launch_side(0))) return rc;
    hipEvent_t spec_ready = event_on(s2);
    spec_ev[0] = spec_ready;
    if (early && nck > 1) {       // side(i+1) runs beside thr(i): spectra and MDCT lines double-buffered
        if ((rc = launch_side(1))) return rc;
        spec_ev[1] = event_on(s2);
    }
    // iteration i: the thresholds of chunk i (pipe: and chunk i-1's MLD rows),
    // then the front, tail and emission of chunk f = i (pipe: i - 1)
    const int64_t d = pipe ? 1 : 0;
    for (int64_t i = 0; i < nck + d; ++i) {
        const bool hasA = i < nck;
        const int64_t f = i - d;
        if (hasA) {
            if (early) spec_ready = spec_ev[i];
            HIPCHK(hipStreamWaitEvent(s0, spec_ready, 0));
        }
        if (f >= 3 && !late) HIPCHK(hipStreamWaitEvent(s0, tail_done[f - 3], 0));   // set f % 3's last reader
        if ((rc = mark(0, -1))) return rc;
        if (pipe) {    // mode 1: pairs {0,1}, {2,3} of chunk i, the MLD pair of chunk i - 1
            const int64_t bA = hasA ? chunks[i].B : 0, bB = i >= 1 ? chunks[i - 1].B : 0;
            const int64_t ia = hasA ? i : i - 1, ib = i >= 1 ? i - 1 : i;
            hipLaunchKernelGGL(k_master_thr, dim3((unsigned)(3 * std::max(bA, bB))), dim3(FRONT_NT), 0, s0, src_thr,
                               T, bufset(ia), F, chunks[ia].ck, bufset(ib), chunks[ib].ck, bA, bB, 1);
        } else {
            const PacMasterChunkBuf K = bufset(i);
            hipLaunchKernelGGL(k_master_thr, dim3((unsigned)(chunks[i].B * (nch == 2 ? 3 : 1))), dim3(FRONT_NT), 0,
                               s0, src_thr, T, K, F, chunks[i].ck, K, chunks[i].ck, chunks[i].B, (int64_t)0, 0);
        }
        if ((rc = mark(0, 0))) return rc;
        if (F.bsf && hasA) {   // the short frames' thresholds (the long kernel skips them)
            hipLaunchKernelGGL(k_master_thr_short, dim3((unsigned)(chunks[i].B * nvar)), dim3(256), 0, s0, src, T,
                               bufset(i), F, chunks[i].ck);
            if ((rc = mark(0, 6))) return rc;
        }
        const hipEvent_t thr_done = event_on(s0);
        if (!early && i + 1 < nck) {                  // the next chunk's LRMS + spectra, beside this front
            HIPCHK(hipStreamWaitEvent(s2, thr_done, 0));
            if ((rc = launch_side(i + 1))) return rc;
            spec_ready = event_on(s2);
        }
        if (f < 0) continue;                          // pipe: chunk 0's MLD rows come with chunk 1's launch
        const Chunk& q = chunks[f];
        const PacMasterChunkBuf K = bufset(f);
        const hipStream_t sf = late ? s2 : s0;       // the front's stream
        if (late) {
            if (i + 1 >= nck) HIPCHK(hipStreamWaitEvent(s2, thr_done, 0));      // no side(i+1) before it
            if (i >= 3) HIPCHK(hipStreamWaitEvent(s2, tail_done[i - 3], 0));   // set k's last reader
        }
        if ((rc = mark(late ? 2 : 0, -1))) return rc;
        if (front_fast)
            hipLaunchKernelGGL(k_master_front<true>, dim3((unsigned)q.B), dim3(256), 0, sf, src_front, T, K, F, q.ck);
        else
            hipLaunchKernelGGL(k_master_front<false>, dim3((unsigned)q.B), dim3(256), 0, sf, src_front, T, K, F, q.ck);
        HIPCHK(hipGetLastError());
        if ((rc = mark(late ? 2 : 0, 1))) return rc;
        const hipEvent_t front_done = event_on(sf);
        if (early && i + 2 < nck) {                   // buffer set i & 1 is free once front(i) is done
            HIPCHK(hipStreamWaitEvent(s2, front_done, 0));
            if ((rc = launch_side(i + 2))) return rc;
            spec_ev[i + 2] = event_on(s2);
        }
        // the tail of this chunk once the next chunk's spectra are ready too,
        // i.e. beside the next chunk's thresholds
        HIPCHK(hipStreamWaitEvent(s1, front_done, 0));
        if (i + 1 < nck && !c->tail_early) HIPCHK(hipStreamWaitEvent(s1, early ? spec_ev[i + 1] : spec_ready, 0));
        if (!pack && f >= 2) HIPCHK(hipStreamWaitEvent(s1, emit_done[f - 2], 0));   // its codes buffer is free
        if ((rc = mark(1, -1))) return rc;
        // few streams: a wave per stream (the one-lane chain's latency would
        // bound the call), else a lane per stream (fewest VALU instructions)
        if (c->tail_wide == 1 || (c->tail_wide < 0 && q.n_s <= PAC_WIDE_MAX))
            hipLaunchKernelGGL(k_master_tail_wide, dim3((unsigned)q.n_s), dim3(WAVE), 0, s1, T, c->hscore.p, K, F,
                               c->blk_off.p, q.ck, c->st_extra.p, c->st_deposit.p, budget);
        else
            hipLaunchKernelGGL(k_master_tail, dim3((unsigned)((q.n_s + WAVE - 1) / WAVE)), dim3(PAC_TAIL_Q * WAVE), PAC_TAIL_LDS,
                               s1, T, c->hscore.p, K, F, c->blk_off.p, q.ck, c->st_extra.p, c->st_deposit.p, budget);
        HIPCHK(hipGetLastError());
        if ((rc = mark(1, 2))) return rc;
        tail_done[f] = event_on(s1);
        if (!pack) {                                  // this chunk's bitstream, beside the next chunk's tail
            HIPCHK(hipStreamWaitEvent(s3, tail_done[f], 0));
            if ((rc = mark(3, -1))) return rc;
            hipLaunchKernelGGL(k_master_emit, dim3((unsigned)((q.B * nch + WAVE - 1) / WAVE)), dim3(WAVE), 0, s3, T,
                               c->huff, c->hcode.p, K, F, c->blk_off.p, q.ck);
            HIPCHK(hipGetLastError());
            if ((rc = mark(3, 8))) return rc;
            emit_done[f] = event_on(s3);
        }
    }
    HIPCHK(hipStreamWaitEvent(s0, event_on(s1), 0));
    HIPCHK(hipStreamWaitEvent(s0, event_on(s3), 0));
    HIPCHK(ev_err);
    if (c->dbg & (32 | 64 | 128)) {
        HIPCHK(hipStreamWaitEvent(s0, event_on(s2), 0));
        if ((rc = report_phase_clocks(c, s0, nprof))) return rc;
    }
    // pass 2: byte offsets in file order, then the packing
    if ((rc = mark(0, -1))) return rc;
    const int64_t ntiles = (G + SCAN_TILE - 1) / SCAN_TILE;
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)ntiles), dim3(256), 0, s0, c->nbytes.p, G, c->tile_sums.p);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(256), 0, s0, c->tile_sums.p, ntiles, c->grand_total.p);
    hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)ntiles), dim3(256), 0, s0, c->nbytes.p, G, c->tile_sums.p,
                       c->off.p);
    HIPCHK(hipGetLastError());
    if ((rc = mark(0, 4))) return rc;
    if (pack) {
        hipLaunchKernelGGL(k_master_pack, dim3((unsigned)nblocks), dim3(256), 0, s0, T, c->huff, F, nch, nblocks,
                           c->off.p, out_dev, out_cap);
    } else {
        hipLaunchKernelGGL(k_master_place, dim3((unsigned)((G + 3) / 4)), dim3(256), 0, s0, F, G, c->off.p, out_dev,
                           out_cap);
        if (stg_need) HIPCHK(hipMemcpyAsync(stg_need, c->m_stg_next.p, sizeof(uint64_t), hipMemcpyDeviceToHost, s0));
    }
    HIPCHK(hipGetLastError());
    if ((rc = mark(0, 3))) return rc;
    HIPCHK(hipMemcpyAsync(out_total, c->grand_total.p, sizeof(int64_t), hipMemcpyDeviceToHost, s0));
    if (c->timing) {
        HIPCHK(hipStreamSynchronize(s0));
        float ph[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int k = 0; k < 4; k++)
            for (size_t j = 1; j < mk[k].size(); j++) {
                if (mk[k][j].second < 0) continue;
                float ms = 0.f;
                HIPCHK(hipEventElapsedTime(&ms, c->evpool[mk[k][j - 1].first], c->evpool[mk[k][j].first]));
                ph[mk[k][j].second] += ms;
            }
        c->last.thr_ms = ph[0];
        c->last.front_ms = ph[1];
        c->last.alloc_ms = ph[2];
        c->last.pack_ms = ph[3];
        c->last.scan_ms = ph[4];
        c->last.lrms_ms = ph[5];
        c->last.thr_short_ms = ph[6];
        c->last.spec_ms = ph[7];
        c->last.emit_ms = ph[8];
        c->last.total_ms = ph[0] + ph[1] + ph[3] + ph[4] + ph[5] + ph[6] + ph[7];   // the tail overlaps the next chunk
        c->last.n_channel_blocks = G;
        c->last.out_bytes = 0;
    }
    return PAC_OK;
}

extern "C" int pac_encode_streams(pac_ctx* c, const pac_params* p, int32_t n_streams, const int16_t* pcm,
                                  const int64_t* frame_offsets, int32_t pcm_is_device, uint8_t* out,
                                  int64_t out_capacity, int32_t out_is_device, int64_t* stream_byte_offsets,
                                  pac_stream_state* states) {
    int rc;
    if (!c || !frame_offsets || !out || !stream_byte_offsets || n_streams < 1)
        return set_err(PAC_E_ARG, "null argument or n_streams < 1");
    if ((rc = check_params(p))) return rc;
    const bool master = p->profile == PAC_PROFILE_MASTER;
    if (master && !c->have_huff) return set_err(PAC_E_TABLES, "master profile needs pac_huffman_load()");
    if (frame_offsets[0] != 0) return set_err(PAC_E_ARG, "frame_offsets[0] must be 0");
    c->last = pac_timing{};        // this call's timing, chunk count and repack flag only
    for (int s = 0; s < n_streams; s++)
        if (frame_offsets[s + 1] < frame_offsets[s])
            return set_err(PAC_E_ARG, "frame_offsets must be non-decreasing");
    HIPCHK(hipSetDevice(c->device));
    PacTables* T;
    if ((rc = get_tables(c, p->sample_rate, p->window, &T))) return rc;
    const int nch = p->n_channels;
    // blocks per stream: every hop after the (optional) carried priorBlock, plus
    // the Close() flush block unless the stream continues in a later call
    std::vector<int64_t> blk(n_streams + 1);
    std::vector<int32_t> lead(n_streams, 0);
    bool any_lead = false;
    blk[0] = 0;
    for (int s = 0; s < n_streams; s++) {
        const int32_t fl = states ? states[s].flags : 0;
        if (fl & ~(PAC_STREAM_HAS_PRIOR | PAC_STREAM_NO_FLUSH)) return set_err(PAC_E_ARG, "stream %d: flags", s);
        if (fl && p->block_switch)        // a frame's window depends on the next frame's hop
            return set_err(PAC_E_UNSUPPORTED, "block switching encodes whole streams (no continuation flags)");
        int64_t n = frame_offsets[s + 1] - frame_offsets[s];
        if (fl & PAC_STREAM_HAS_PRIOR) {   // a short prior is zero-padded, as the last hop (pcmfile.py:77-79)
            lead[s] = PAC_HALFN;
            any_lead = true;
            n = n > PAC_HALFN ? n - PAC_HALFN : 0;
        }
        blk[s + 1] = blk[s] + (n + PAC_HALFN - 1) / PAC_HALFN + ((fl & PAC_STREAM_NO_FLUSH) ? 0 : 1);
    }
    const int64_t nblocks = blk[n_streams];
    const int64_t G = nblocks * nch;
    if (G > 0x7fffffffLL) return set_err(PAC_E_ARG, "too many channel-blocks in one call");
    const int64_t nframes = frame_offsets[n_streams];
    hipStream_t s = c->stream;
    if ((rc = c->frame_off.ensure(n_streams + 1)) || (rc = c->blk_off.ensure(n_streams + 1)) ||
        (rc = c->stream_off.ensure(n_streams + 1)))
        return rc;
    HIPCHK(hipMemcpyAsync(c->frame_off.p, frame_offsets, (n_streams + 1) * sizeof(int64_t),
                          hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->blk_off.p, blk.data(), (n_streams + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    if (any_lead) {
        if ((rc = c->lead.ensure(n_streams))) return rc;
        HIPCHK(hipMemcpyAsync(c->lead.p, lead.data(), n_streams * sizeof(int32_t), hipMemcpyHostToDevice, s));
    }
    if (nblocks == 0) {       // nothing to encode (every stream continues, no new hop)
        for (int k = 0; k <= n_streams; k++) stream_byte_offsets[k] = 0;
        HIPCHK(hipStreamSynchronize(s));
        return PAC_OK;
    }
    const int16_t* pcm_dev = pcm;
    if (!pcm_is_device) {
        if ((rc = c->pcm_stage.ensure(nframes * nch + 1))) return rc;
        if (nframes) HIPCHK(hipMemcpyAsync(c->pcm_stage.p, pcm, nframes * nch * sizeof(int16_t),
                                           hipMemcpyHostToDevice, s));
        pcm_dev = c->pcm_stage.p;
    }
    uint8_t* out_dev = out;
    if (!out_is_device) {
        int64_t bound = pac_encode_bound(p, n_streams, frame_offsets);
        int64_t want = bound < out_capacity ? bound : out_capacity;
        if ((rc = c->out_stage.ensure(want))) return rc;
        out_dev = c->out_stage.p;
    }
    PacSource src{pcm_dev, c->frame_off.p, c->blk_off.p, nullptr, n_streams, nch, c->dbg, nullptr,
                  any_lead ? c->lead.p : nullptr};
    int64_t total = 0;
    if (master) {
        if ((rc = c->st_extra.ensure(n_streams)) || (rc = c->st_deposit.ensure(n_streams))) return rc;
        std::vector<int64_t> ex(n_streams, 0), dp(n_streams, 0);
        if (states)
            for (int i = 0; i < n_streams; i++) { ex[i] = states[i].extra_bits; dp[i] = states[i].bit_deposit; }
        HIPCHK(hipMemcpyAsync(c->st_extra.p, ex.data(), n_streams * sizeof(int64_t), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(c->st_deposit.p, dp.data(), n_streams * sizeof(int64_t), hipMemcpyHostToDevice, s));
        uint64_t need = 0;
        int64_t scap = 0;
        if ((rc = run_master(c, p, T, src, blk, out_dev, out_capacity, &total, false, false, &need, &scap))) return rc;
        HIPCHK(hipStreamSynchronize(s));
        c->last.repacked = 0;
        if ((int64_t)need > scap && total > out_capacity)    // no second pass for an output that cannot fit
            return set_err(PAC_E_CAPACITY, "output needs %lld bytes, capacity %lld", (long long)total,
                           (long long)out_capacity);
        if ((int64_t)need > scap) {   // the staging overflowed (> 1.5 KB per channel-block): again, packing
            c->last.repacked = 1;
            HIPCHK(hipMemcpyAsync(c->st_extra.p, ex.data(), n_streams * sizeof(int64_t), hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(c->st_deposit.p, dp.data(), n_streams * sizeof(int64_t), hipMemcpyHostToDevice, s));
            if ((rc = run_master(c, p, T, src, blk, out_dev, out_capacity, &total, false, true))) return rc;
        }
        hipLaunchKernelGGL(k_stream_offsets, dim3((n_streams + 1 + 255) / 256), dim3(256), 0, s, c->off.p,
                           c->blk_off.p, n_streams, nch, c->grand_total.p, c->stream_off.p);
        HIPCHK(hipGetLastError());
        if (states) {
            HIPCHK(hipMemcpyAsync(ex.data(), c->st_extra.p, n_streams * sizeof(int64_t), hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(dp.data(), c->st_deposit.p, n_streams * sizeof(int64_t), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            for (int i = 0; i < n_streams; i++) { states[i].extra_bits = ex[i]; states[i].bit_deposit = dp[i]; }
        }
    } else {
        int64_t* off_dev = nullptr;
        if ((rc = run_origin(c, p, T, src, G, out_dev, out_capacity, &total, &off_dev))) return rc;
        hipLaunchKernelGGL(k_stream_offsets, dim3((n_streams + 1 + 255) / 256), dim3(256), 0, s, off_dev,
                           c->blk_off.p, n_streams, nch, c->grand_total.p, c->stream_off.p);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipMemcpyAsync(stream_byte_offsets, c->stream_off.p, (n_streams + 1) * sizeof(int64_t),
                          hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (total > out_capacity)
        return set_err(PAC_E_CAPACITY, "output needs %lld bytes, capacity %lld", (long long)total,
                       (long long)out_capacity);
    if (!out_is_device && total) {
        HIPCHK(hipMemcpyAsync(out, out_dev, total, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    if (!master) finish_timing(c, G, total);
    return report_rowprof(c, s);
}

// --- per-block API ----------------------------------------------------------

struct BitReader {
    const uint8_t* p;
    int64_t bit;
    uint32_t get(int n) {
        uint32_t v = 0;
        for (int i = 0; i < n; i++, bit++) v = (v << 1) | ((p[bit >> 3] >> (7 - (bit & 7))) & 1u);
        return v;
    }
};

extern "C" int pac_encode_block(pac_ctx* c, const pac_params* p, const double* full_block,
                                pac_stream_state* state, uint8_t* out, int64_t out_capacity, int64_t* out_bytes,
                                pac_block_fields* fields) {
    int rc;
    if (!c || !full_block || !out || !out_bytes) return set_err(PAC_E_ARG, "null argument");
    if ((rc = check_params(p))) return rc;
    if (p->block_switch)      // a frame's window depends on its neighbours' hops
        return set_err(PAC_E_UNSUPPORTED, "block switching needs whole streams (pac_encode_streams)");
    const bool master = p->profile == PAC_PROFILE_MASTER;
    if (master && !c->have_huff) return set_err(PAC_E_TABLES, "master profile needs pac_huffman_load()");
    HIPCHK(hipSetDevice(c->device));
    PacTables* T;
    if ((rc = get_tables(c, p->sample_rate, p->window, &T))) return rc;
    const int nch = p->n_channels;
    const int64_t G = nch;
    hipStream_t s = c->stream;
    if ((rc = c->fsrc.ensure(G * PAC_N)) || (rc = c->out_stage.ensure(G * 8400)) ||
        (rc = c->blk_off.ensure(2)) || (rc = c->stream_off.ensure(2)))
        return rc;
    HIPCHK(hipMemcpyAsync(c->fsrc.p, full_block, G * PAC_N * sizeof(double), hipMemcpyHostToDevice, s));
    PacSource src{nullptr, nullptr, c->blk_off.p, c->fsrc.p, 1, nch, 0, nullptr, nullptr};
    int64_t total = 0;
    std::vector<double> smr(PAC_NB * G);
    int32_t lrms[PAC_NB] = {0};
    std::vector<uint32_t> dbg_mant;
    std::vector<uint64_t> dbg_code;
    std::vector<uint8_t> dbg_len;
    if (master) {
        std::vector<int64_t> blk = {0, 1};
        HIPCHK(hipMemcpyAsync(c->blk_off.p, blk.data(), 2 * sizeof(int64_t), hipMemcpyHostToDevice, s));
        if ((rc = c->st_extra.ensure(1)) || (rc = c->st_deposit.ensure(1))) return rc;
        int64_t ex = state ? state->extra_bits : 0, dp = state ? state->bit_deposit : 0;
        HIPCHK(hipMemcpyAsync(c->st_extra.p, &ex, sizeof(int64_t), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(c->st_deposit.p, &dp, sizeof(int64_t), hipMemcpyHostToDevice, s));
        if ((rc = run_master(c, p, T, src, blk, c->out_stage.p, c->out_stage.n, &total, fields != nullptr)))
            return rc;
        if (fields) {   // per-line mantissas and Huffman codes as the pack kernel emitted them
            dbg_mant.resize(G * PAC_HALFN);
            dbg_code.resize(G * PAC_HALFN);
            dbg_len.resize(G * PAC_HALFN);
            HIPCHK(hipMemcpyAsync(dbg_mant.data(), c->dbg_mant.p, G * PAC_HALFN * sizeof(uint32_t),
                                  hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(dbg_code.data(), c->dbg_code.p, G * PAC_HALFN * sizeof(uint64_t),
                                  hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(dbg_len.data(), c->dbg_len.p, G * PAC_HALFN, hipMemcpyDeviceToHost, s));
        }
        HIPCHK(hipMemcpyAsync(&ex, c->st_extra.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(&dp, c->st_deposit.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(smr.data(), c->m_smr.p, smr.size() * sizeof(double), hipMemcpyDeviceToHost, s));
        uint8_t lr[PAC_NB];
        HIPCHK(hipMemcpyAsync(lr, c->m_lrms.p, PAC_NB, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        for (int b = 0; b < PAC_NB; b++) lrms[b] = lr[b];
        if (state) { state->extra_bits = ex; state->bit_deposit = dp; }
    } else {
        int64_t* off_dev = nullptr;
        if ((rc = run_origin(c, p, T, src, G, c->out_stage.p, c->out_stage.n, &total, &off_dev))) return rc;
        HIPCHK(hipMemcpyAsync(smr.data(), c->smr.p, smr.size() * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        finish_timing(c, G, total);
    }
    if (total > out_capacity) return set_err(PAC_E_CAPACITY, "block needs %lld bytes", (long long)total);
    HIPCHK(hipMemcpyAsync(out, c->out_stage.p, total, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    *out_bytes = total;
    if (fields) {
        // the codec.Encode() tuple: side info read back from the GPU-written
        // channel-blocks, mantissas (origin: raw codes in the bitstream;
        // master: as the pack kernel emitted them, with their Huffman codes)
        memset(fields, 0, sizeof(*fields));
        fields->n_channels = nch;
        int32_t nl[PAC_NB];
        host_band_layout(p->sample_rate, nl);
        int64_t o = 0;
        for (int ch = 0; ch < nch; ch++) {
            uint32_t nb = out[o] | (out[o + 1] << 8) | (out[o + 2] << 16) | ((uint32_t)out[o + 3] << 24);
            fields->nbytes[ch] = (int32_t)nb;
            BitReader br{out + o + 4, 0};
            fields->overall[ch] = (int32_t)br.get(4);
            int tid = master ? (int)br.get(4) : 0;
            fields->table_id[ch] = tid;
            int line = 0;
            for (int b = 0; b < PAC_NB; b++) {
                int ba = (int)br.get(4);
                if (ba) ba++;
                fields->ba[ch][b] = ba;
                fields->sf[ch][b] = (int32_t)br.get(4);
                fields->smr[ch][b] = smr[ch * PAC_NB + b];
                if (!master) {
                    for (int l = 0; l < nl[b]; l++) fields->mant[ch][line + l] = ba ? (int32_t)br.get(ba) : 0;
                } else if (ba) {      // skip the band's sign bits and codes in the bitstream
                    br.bit += nl[b];
                    for (int l = line; l < line + nl[b]; l++) {
                        fields->mant[ch][l] = (int32_t)dbg_mant[ch * PAC_HALFN + l];
                        fields->huff_code[ch][l] = dbg_code[ch * PAC_HALFN + l];
                        fields->huff_len[ch][l] = (int32_t)dbg_len[ch * PAC_HALFN + l];
                        br.bit += dbg_len[ch * PAC_HALFN + l];
                    }
                }
                line += nl[b];
            }
            o += 4 + nb;
        }
        for (int b = 0; b < PAC_NB; b++) fields->lrms[b] = lrms[b];
    }
    return PAC_OK;
}

// --- device buffers / sync / timing -----------------------------------------

extern "C" int pac_device_alloc(pac_ctx* c, int64_t bytes, void** ptr) {
    if (!c || !ptr || bytes < 0) return set_err(PAC_E_ARG, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    if (hipMalloc(ptr, bytes ? bytes : 1) != hipSuccess) return set_err(PAC_E_NOMEM, "hipMalloc(%lld)", (long long)bytes);
    return PAC_OK;
}
extern "C" int pac_device_free(pac_ctx* c, void* ptr) {
    if (!c) return set_err(PAC_E_ARG, "null ctx");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipFree(ptr));
    return PAC_OK;
}
extern "C" int pac_copy_to_device(pac_ctx* c, void* dst, const void* src, int64_t bytes) {
    if (!c) return set_err(PAC_E_ARG, "null ctx");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return PAC_OK;
}
extern "C" int pac_copy_to_host(pac_ctx* c, void* dst, const void* src, int64_t bytes) {
    if (!c) return set_err(PAC_E_ARG, "null ctx");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return PAC_OK;
}
extern "C" int pac_synth_white(pac_ctx* c, int16_t* dev_pcm, int64_t n, uint64_t seed) {
    if (!c || !dev_pcm || n < 0) return set_err(PAC_E_ARG, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    hipLaunchKernelGGL(k_synth_white, dim3(4096), dim3(256), 0, c->stream, dev_pcm, n, seed);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return PAC_OK;
}
extern "C" int pac_synth_pink_tones(pac_ctx* c, int16_t* dev_pcm, int64_t n_frames, int32_t sample_rate,
                                    uint64_t seed) {
    if (!c || !dev_pcm || n_frames < 0 || sample_rate <= 0) return set_err(PAC_E_ARG, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    hipLaunchKernelGGL(k_synth_pink_tones, dim3(4096), dim3(256), 0, c->stream, dev_pcm, n_frames,
                       (double)sample_rate, seed);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return PAC_OK;
}

extern "C" int pac_synth_bursts(pac_ctx* c, int16_t* dev_pcm, int64_t n_frames, int64_t period, uint64_t seed) {
    if (!c || !dev_pcm || n_frames < 0 || period < 4096) return set_err(PAC_E_ARG, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    hipLaunchKernelGGL(k_synth_bursts, dim3(4096), dim3(256), 0, c->stream, dev_pcm, n_frames, period, seed);
    HIPCHK(hipGetLastError());
    return PAC_OK;
}
extern "C" int pac_sync(pac_ctx* c) {
    if (!c) return set_err(PAC_E_ARG, "null ctx");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    return PAC_OK;
}
extern "C" int pac_set_timing(pac_ctx* c, int32_t enable) {
    if (!c) return set_err(PAC_E_ARG, "null ctx");
    c->timing = enable != 0;
    return PAC_OK;
}
extern "C" int pac_debug_threshold(pac_ctx* c, int32_t sample_rate, int32_t n, const double* data,
                                   int32_t no_drop, double* thr, int32_t* npeaks) {
    int rc;
    if (!c || !data || !thr || !npeaks || n < 1) return set_err(PAC_E_ARG, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    PacTables* T;
    if ((rc = get_tables(c, sample_rate, PAC_WINDOW_SINE, &T))) return rc;
    double *dd = nullptr, *dt = nullptr;
    int32_t* dp = nullptr;
    HIPCHK(hipMalloc((void**)&dd, (size_t)n * PAC_N * sizeof(double)));
    HIPCHK(hipMalloc((void**)&dt, (size_t)n * PAC_HALFN * sizeof(double)));
    HIPCHK(hipMalloc((void**)&dp, (size_t)n * sizeof(int32_t)));
    HIPCHK(hipMemcpy(dd, data, (size_t)n * PAC_N * sizeof(double), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_debug_threshold, dim3(n), dim3(64), 0, c->stream, T, dd, no_drop, dt, dp);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(thr, dt, (size_t)n * PAC_HALFN * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(npeaks, dp, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost));
    hipFree(dd); hipFree(dt); hipFree(dp);
    return PAC_OK;
}

extern "C" int pac_debug_mdct(pac_ctx* c, int32_t n, const double* data, double* X) {
    if (!c || !data || !X || n < 1) return set_err(PAC_E_ARG, "bad argument");
    int rc;
    HIPCHK(hipSetDevice(c->device));
    PacTables* T;
    if ((rc = get_tables(c, 48000, PAC_WINDOW_SINE, &T))) return rc;
    double *dd = nullptr, *dx = nullptr;
    HIPCHK(hipMalloc((void**)&dd, (size_t)n * PAC_N * sizeof(double)));
    HIPCHK(hipMalloc((void**)&dx, (size_t)n * PAC_HALFN * sizeof(double)));
    HIPCHK(hipMemcpy(dd, data, (size_t)n * PAC_N * sizeof(double), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_debug_mdct, dim3(n), dim3(64), 0, c->stream, T, dd, dx);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(X, dx, (size_t)n * PAC_HALFN * sizeof(double), hipMemcpyDeviceToHost));
    hipFree(dd); hipFree(dx);
    return PAC_OK;
}

extern "C" int pac_debug_mdct_dft(pac_ctx* c, int32_t n, const double* data, double* X) {
    if (!c || !data || !X || n < 1) return set_err(PAC_E_ARG, "bad argument");
    int rc;
    HIPCHK(hipSetDevice(c->device));
    PacTables* T;
    if ((rc = get_tables(c, 48000, PAC_WINDOW_SINE, &T))) return rc;
    double *dd = nullptr, *dx = nullptr;
    HIPCHK(hipMalloc((void**)&dd, (size_t)n * PAC_N * sizeof(double)));
    HIPCHK(hipMalloc((void**)&dx, (size_t)n * PAC_HALFN * sizeof(double)));
    HIPCHK(hipMemcpy(dd, data, (size_t)n * PAC_N * sizeof(double), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_debug_mdct_dft, dim3((unsigned)((n + 1) / 2)), dim3(256), 0, c->stream, T, dd, n, dx);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(X, dx, (size_t)n * PAC_HALFN * sizeof(double), hipMemcpyDeviceToHost));
    hipFree(dd); hipFree(dx);
    return PAC_OK;
}

extern "C" int pac_set_chunk_blocks(pac_ctx* c, int64_t blocks) {
    if (!c || blocks < 1) return set_err(PAC_E_ARG, "bad argument");
    if (blocks > PAC_CHUNK_MAX) return set_err(PAC_E_ARG, "chunk_blocks above PAC_CHUNK_MAX (131071)");
    c->chunk_blocks = blocks;
    return PAC_OK;
}
extern "C" int pac_last_timing(pac_ctx* c, pac_timing* out) {
    if (!c || !out) return set_err(PAC_E_ARG, "null argument");
    *out = c->last;
    return PAC_OK;
}

// ---------------------------------------------------------------------------
// decoder
// ---------------------------------------------------------------------------

// host-side layout of n data sections held in host memory: the output frame
// offsets pac_decode_streams will produce (no device work, no staging)
extern "C" int pac_decode_layout(const pac_params* p, int32_t n_streams, const uint8_t* data,
                                 const int64_t* so, int32_t preroll, int64_t* frame_offsets) {
    if (!p || !data || !so || !frame_offsets || n_streams < 1) return set_err(PAC_E_ARG, "null argument");
    const int nch = p->n_channels;
    if (nch < 1) return set_err(PAC_E_ARG, "n_channels %d", nch);
    int64_t frames = 0;
    for (int k = 0; k < n_streams; k++) {
        int64_t pos = so[k], cnt = 0;
        const int64_t end = so[k + 1];
        while (pos + 4 <= end) {
            const uint8_t* q = data + pos;
            const uint32_t nb = q[0] | (q[1] << 8) | (q[2] << 16) | ((uint32_t)q[3] << 24);
            pos += 4 + (int64_t)nb;
            cnt++;
        }
        if (pos != end || cnt % nch)
            return set_err(PAC_E_ARG, "stream %d: malformed data section (channel-blocks %lld, %d channels)", k,
                           (long long)cnt, nch);
        frame_offsets[k] = frames;
        frames += (cnt / nch + (preroll ? 1 : 0)) * PAC_HALFN;
    }
    frame_offsets[n_streams] = frames;
    return PAC_OK;
}

extern "C" int pac_decode_streams(pac_ctx* c, const pac_params* p, int32_t n_streams, const uint8_t* data,
                                  const int64_t* stream_byte_offsets, int32_t data_is_device, int32_t preroll,
                                  int16_t* pcm_out, int64_t pcm_capacity_frames, int32_t pcm_is_device,
                                  double* float_out, int64_t* frame_offsets) {
    int rc;
    if (!c || !p || !stream_byte_offsets || !frame_offsets || n_streams < 1)
        return set_err(PAC_E_ARG, "null argument or n_streams < 1");
    if ((rc = check_params(p))) return rc;
    const bool master = p->profile == PAC_PROFILE_MASTER;
    const int nch = p->n_channels;
    if (master && !c->have_huff) return set_err(PAC_E_TABLES, "master profile needs pac_huffman_load()");
    if (stream_byte_offsets[0] != 0) return set_err(PAC_E_ARG, "stream_byte_offsets[0] must be 0");
    for (int s = 0; s < n_streams; s++)
        if (stream_byte_offsets[s + 1] < stream_byte_offsets[s])
            return set_err(PAC_E_ARG, "stream_byte_offsets must be non-decreasing");
    HIPCHK(hipSetDevice(c->device));
    PacTables* T;
    if ((rc = get_tables(c, p->sample_rate, p->window, &T))) return rc;
    hipStream_t s = c->stream;
    const int64_t nbytes = stream_byte_offsets[n_streams];
    const uint8_t* ddev = data;
    if (!data_is_device) {
        if ((rc = c->dec_data.ensure(nbytes + 8))) return rc;
        if (nbytes) HIPCHK(hipMemcpyAsync(c->dec_data.p, data, nbytes, hipMemcpyHostToDevice, s));
        ddev = c->dec_data.p;
    }
    if ((rc = c->dec_so.ensure(n_streams + 1)) || (rc = c->dec_cnt.ensure(n_streams)) ||
        (rc = c->dec_cbbase.ensure(n_streams + 1)) || (rc = c->dec_nblk.ensure(n_streams)) ||
        (rc = c->dec_segbase.ensure(n_streams + 1)) || (rc = c->dec_fo.ensure(n_streams + 1)))
        return rc;
    HIPCHK(hipMemcpyAsync(c->dec_so.p, stream_byte_offsets, (n_streams + 1) * sizeof(int64_t),
                          hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_dec_count, dim3((n_streams + 255) / 256), dim3(256), 0, s, ddev, c->dec_so.p, n_streams,
                       c->dec_cnt.p);
    HIPCHK(hipGetLastError());
    std::vector<int64_t> cnt(n_streams), cbb(n_streams + 1), nb(n_streams), segb(n_streams + 1);
    HIPCHK(hipMemcpyAsync(cnt.data(), c->dec_cnt.p, n_streams * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    int64_t G = 0, segs = 0, frames = 0;
    for (int k = 0; k < n_streams; k++) {
        if (cnt[k] < 0 || cnt[k] % nch)
            return set_err(PAC_E_ARG, "stream %d: malformed data section (channel-blocks %lld, %d channels)", k,
                           (long long)cnt[k], nch);
        cbb[k] = G;
        G += cnt[k];
        nb[k] = cnt[k] / nch;
        segb[k] = segs;
        segs += (nb[k] + DEC_SEG - 1) / DEC_SEG;
        frame_offsets[k] = frames;
        frames += (nb[k] + (preroll ? 1 : 0)) * PAC_HALFN;
    }
    cbb[n_streams] = G;
    segb[n_streams] = segs;
    frame_offsets[n_streams] = frames;
    if (!pcm_out || pcm_capacity_frames < frames)
        return set_err(PAC_E_CAPACITY, "decoded output needs %lld frames, capacity %lld", (long long)frames,
                       (long long)pcm_capacity_frames);
    if (G > 0x7fffffffLL) return set_err(PAC_E_ARG, "too many channel-blocks in one call");
    const int64_t G1 = G > 0 ? G : 1;
    if ((rc = c->dec_cboff.ensure(G1)) || (rc = c->dec_codes.ensure(((G1 + DEC_PARSE_NT - 1) / DEC_PARSE_NT) * DEC_PARSE_NT * PAC_HALFN)) ||
        (rc = c->dec_ba.ensure(G1 * DEC_NBP * 2)) ||
        (rc = c->dec_ov.ensure(G1)) || (rc = c->dec_lrms.ensure(G1 * DEC_NBP)) || (rc = c->dec_err.ensure(1)) ||
        (p->block_switch && (rc = c->dec_bsf.ensure(G1))))
        return rc;
    HIPCHK(hipMemsetAsync(c->dec_err.p, 0, sizeof(int), s));
    HIPCHK(hipMemcpyAsync(c->dec_cbbase.p, cbb.data(), (n_streams + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->dec_nblk.p, nb.data(), n_streams * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->dec_segbase.p, segb.data(), (n_streams + 1) * sizeof(int64_t), hipMemcpyHostToDevice,
                          s));
    HIPCHK(hipMemcpyAsync(c->dec_fo.p, frame_offsets, (n_streams + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    int16_t* pdev = pcm_out;
    if (!pcm_is_device) {
        if ((rc = c->dec_pcm.ensure(frames * nch + 1))) return rc;
        pdev = c->dec_pcm.p;
    }
    double* fdev = nullptr;
    if (float_out) {
        if ((rc = c->dec_fpcm.ensure(frames * nch + 1))) return rc;
        fdev = c->dec_fpcm.p;
    }
    // an empty data section still yields the one all-zero ReadDataBlock result with preroll
    if (preroll)
        for (int k = 0; k < n_streams; k++)
            if (!nb[k]) {
                HIPCHK(hipMemsetAsync(pdev + frame_offsets[k] * nch, 0, PAC_HALFN * nch * sizeof(int16_t), s));
                if (fdev) HIPCHK(hipMemsetAsync(fdev + frame_offsets[k] * nch, 0, PAC_HALFN * nch * sizeof(double), s));
            }
    if (c->timing) HIPCHK(hipEventRecord(c->ev[0], s));
    if (G) {
        hipLaunchKernelGGL(k_dec_index, dim3((n_streams + 255) / 256), dim3(256), 0, s, ddev, c->dec_so.p, n_streams,
                           c->dec_cbbase.p, c->dec_cboff.p);
        PacDecWork D{c->dec_codes.p, reinterpret_cast<uint16_t*>(c->dec_ba.p), c->dec_ov.p, c->dec_lrms.p, c->dec_err.p,
                     p->block_switch ? c->dec_bsf.p : nullptr};
        hipLaunchKernelGGL(k_dec_parse, dim3((unsigned)((G + DEC_PARSE_NT - 1) / DEC_PARSE_NT)), dim3(DEC_PARSE_NT), 0, s,
                           ddev, c->dec_cboff.p, G,
                           (int)master, T, master ? c->hdec_tab.p : nullptr, c->hdec, D);
        HIPCHK(hipGetLastError());
        if (c->timing) HIPCHK(hipEventRecord(c->ev[1], s));
        PacDecOut O{pdev, fdev, c->dec_fo.p, preroll ? 1 : 0};
        const int64_t grid = segs * (master ? 1 : nch);
        if (grid > 0) {     // the block-switching instantiation only when the stream has the flags
            if (D.bsf)
                hipLaunchKernelGGL(k_dec_synth<true>, dim3((unsigned)grid), dim3(256), 0, s, T, D, c->dec_cbbase.p,
                                   c->dec_nblk.p, c->dec_segbase.p, n_streams, nch, (int)master, O);
            else
                hipLaunchKernelGGL(k_dec_synth<false>, dim3((unsigned)grid), dim3(256), 0, s, T, D, c->dec_cbbase.p,
                                   c->dec_nblk.p, c->dec_segbase.p, n_streams, nch, (int)master, O);
        }
        HIPCHK(hipGetLastError());
    } else if (c->timing) {
        HIPCHK(hipEventRecord(c->ev[1], s));
    }
    if (c->timing) HIPCHK(hipEventRecord(c->ev[2], s));
    if (!pcm_is_device && frames)
        HIPCHK(hipMemcpyAsync(pcm_out, pdev, frames * nch * sizeof(int16_t), hipMemcpyDeviceToHost, s));
    if (float_out && frames)
        HIPCHK(hipMemcpyAsync(float_out, fdev, frames * nch * sizeof(double), hipMemcpyDeviceToHost, s));
    int derr = 0;
    HIPCHK(hipMemcpyAsync(&derr, c->dec_err.p, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (derr)
        return set_err(PAC_E_ARG, "malformed data section: a channel-block's fields run past its nBytes");
    if (c->timing) {
        hipEventElapsedTime(&c->last.front_ms, c->ev[0], c->ev[1]);    // parse
        hipEventElapsedTime(&c->last.pack_ms, c->ev[1], c->ev[2]);     // synthesis
        c->last.alloc_ms = 0;
        c->last.scan_ms = 0;
        hipEventElapsedTime(&c->last.total_ms, c->ev[0], c->ev[2]);
        c->last.n_channel_blocks = G;
        c->last.out_bytes = frames * nch * 2;
    }
    return PAC_OK;
}

// ---------------------------------------------------------------------------
// WAV ingest / egress on the device
// ---------------------------------------------------------------------------

static_assert(sizeof(PacWavInfo) == sizeof(pac_wav_info), "pac_wav_info layout");

static const char* wav_status_msg(int st) {     // the reference's raises (pcmfile.py:36-51)
    switch (st) {
        case PAC_WAV_NOT_RIFF: return "File opened for PCMFile is not a RIFF file!";
        case PAC_WAV_NO_FMT: return "Didn't find WAV file 'fmt ' chunk following RIFF file header";
        case PAC_WAV_NOT_PCM: return "Opened a non-PCM WAV file as a PCMFile";
        case PAC_WAV_NOT_16BIT: return "PCMFile was not 16-bits per sample";
        case PAC_WAV_NO_DATA: return "Didn't find WAV file 'data' chunk following 'fmt ' chunk";
        default: return "malformed WAV file";
    }
}

// stage (if host) and scan n files; the blob's device pointer in *dev
static int wav_scan_dev(pac_ctx* c, int32_t n, const uint8_t* blob, const int64_t* foff, int32_t blob_is_device,
                        const uint8_t** dev, pac_wav_info* info) {
    int rc;
    if (!c || !blob || !foff || !info || n < 1) return set_err(PAC_E_ARG, "null argument or n_files < 1");
    if (foff[0] != 0) return set_err(PAC_E_ARG, "file_offsets[0] must be 0");
    for (int i = 0; i < n; i++)
        if (foff[i + 1] < foff[i]) return set_err(PAC_E_ARG, "file_offsets must be non-decreasing");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const int64_t bytes = foff[n];
    const uint8_t* d = blob;
    if (!blob_is_device) {
        if ((rc = c->wav_blob.ensure(bytes + 1))) return rc;
        if (bytes) HIPCHK(hipMemcpyAsync(c->wav_blob.p, blob, bytes, hipMemcpyHostToDevice, s));
        d = c->wav_blob.p;
    }
    if ((rc = c->wav_foff.ensure(n + 1)) || (rc = c->wav_info.ensure(n))) return rc;
    HIPCHK(hipMemcpyAsync(c->wav_foff.p, foff, (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_wav_scan, dim3((n + 63) / 64), dim3(64), 0, s, d, c->wav_foff.p, n, c->wav_info.p,
                       (int)PAC_HALFN);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(info, c->wav_info.p, n * sizeof(pac_wav_info), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    *dev = d;
    return PAC_OK;
}

extern "C" int pac_wav_scan(pac_ctx* c, int32_t n_files, const uint8_t* blob, const int64_t* file_offsets,
                            int32_t blob_is_device, pac_wav_info* info) {
    const uint8_t* d;
    return wav_scan_dev(c, n_files, blob, file_offsets, blob_is_device, &d, info);
}

extern "C" int pac_encode_wav(pac_ctx* c, const pac_params* p, int32_t n_files, const uint8_t* blob,
                              const int64_t* file_offsets, int32_t blob_is_device, uint8_t* out,
                              int64_t out_capacity, int32_t out_is_device, int64_t* stream_byte_offsets,
                              pac_stream_state* states, pac_wav_info* info_out) {
    int rc;
    if ((rc = check_params(p))) return rc;
    std::vector<pac_wav_info> info(n_files > 0 ? n_files : 1);
    const uint8_t* d = nullptr;
    if ((rc = wav_scan_dev(c, n_files, blob, file_offsets, blob_is_device, &d, info.data()))) return rc;
    if (info_out) memcpy(info_out, info.data(), n_files * sizeof(pac_wav_info));
    const int nch = p->n_channels;
    std::vector<int64_t> fo(n_files + 1, 0), segb(n_files + 1, 0);
    for (int i = 0; i < n_files; i++) {
        if (info[i].status) return set_err(PAC_E_ARG, "file %d: %s", i, wav_status_msg(info[i].status));
        if (info[i].sample_rate != p->sample_rate || info[i].n_channels != nch)
            return set_err(PAC_E_ARG, "file %d: %d Hz x %d channels, the call is %d Hz x %d", i,
                           info[i].sample_rate, info[i].n_channels, p->sample_rate, nch);
        fo[i + 1] = fo[i] + info[i].frames;
        segb[i + 1] = segb[i] + (info[i].frames * nch * 2 + PAC_WAV_SEG - 1) / PAC_WAV_SEG;
    }
    hipStream_t s = c->stream;
    if ((rc = c->wav_pcm.ensure(fo[n_files] * nch * 2 + 2)) || (rc = c->wav_fo.ensure(n_files + 1)) ||
        (rc = c->wav_segb.ensure(n_files + 1)))
        return rc;
    HIPCHK(hipMemcpyAsync(c->wav_fo.p, fo.data(), (n_files + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->wav_segb.p, segb.data(), (n_files + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    if (segb[n_files] > 0) {
        hipLaunchKernelGGL(k_wav_gather, dim3((unsigned)segb[n_files]), dim3(256), 0, s, d, c->wav_foff.p,
                           c->wav_info.p, c->wav_fo.p, c->wav_segb.p, n_files, nch, c->wav_pcm.p);
        HIPCHK(hipGetLastError());
    }
    return pac_encode_streams(c, p, n_files, reinterpret_cast<const int16_t*>(c->wav_pcm.p), fo.data(), 1, out,
                              out_capacity, out_is_device, stream_byte_offsets, states);
}

extern "C" int pac_decode_wav(pac_ctx* c, const pac_params* p, int32_t n_streams, const uint8_t* data,
                              const int64_t* stream_byte_offsets, int32_t data_is_device,
                              const int64_t* num_samples, uint8_t* out, int64_t out_capacity, int32_t out_is_device,
                              int64_t* wav_offsets) {
    int rc;
    if (!c || !p || !data || !stream_byte_offsets || !num_samples || !wav_offsets || n_streams < 1)
        return set_err(PAC_E_ARG, "null argument or n_streams < 1");
    if ((rc = check_params(p))) return rc;
    const int nch = p->n_channels;
    std::vector<int64_t> fo(n_streams + 1, 0), segb(n_streams + 1, 0);
    if (data_is_device) {           // frame offsets from the device data: size query
        rc = pac_decode_streams(c, p, n_streams, data, stream_byte_offsets, 1, 0, nullptr, 0, 1, nullptr, fo.data());
        if (rc != PAC_OK && rc != PAC_E_CAPACITY) return rc;
    } else if ((rc = pac_decode_layout(p, n_streams, data, stream_byte_offsets, 0, fo.data()))) {
        return rc;
    }
    const int64_t frames = fo[n_streams];
    if ((rc = c->wav_pcm.ensure(frames * nch * 2 + 2))) return rc;
    if ((rc = pac_decode_streams(c, p, n_streams, data, stream_byte_offsets, data_is_device, 0,
                                 reinterpret_cast<int16_t*>(c->wav_pcm.p), frames, 1, nullptr, fo.data())))
        return rc;
    wav_offsets[0] = 0;
    for (int k = 0; k < n_streams; k++) {
        wav_offsets[k + 1] = wav_offsets[k] + 44 + (fo[k + 1] - fo[k]) * nch * 2;
        segb[k + 1] = segb[k] + (44 + (fo[k + 1] - fo[k]) * nch * 2 + PAC_WAV_SEG - 1) / PAC_WAV_SEG;
    }
    const int64_t total = wav_offsets[n_streams];
    if (total > out_capacity)
        return set_err(PAC_E_CAPACITY, "WAV output needs %lld bytes, capacity %lld", (long long)total,
                       (long long)out_capacity);
    hipStream_t s = c->stream;
    if ((rc = c->wav_fo.ensure(n_streams + 1)) || (rc = c->wav_segb.ensure(n_streams + 1)) ||
        (rc = c->wav_ns.ensure(n_streams)) || (rc = c->wav_wo.ensure(n_streams + 1)))
        return rc;
    uint8_t* od = out;
    if (!out_is_device) {
        if ((rc = c->wav_out.ensure(total + 1))) return rc;
        od = c->wav_out.p;
    }
    HIPCHK(hipMemcpyAsync(c->wav_fo.p, fo.data(), (n_streams + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->wav_segb.p, segb.data(), (n_streams + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->wav_ns.p, num_samples, n_streams * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->wav_wo.p, wav_offsets, (n_streams + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_wav_write, dim3((unsigned)segb[n_streams]), dim3(256), 0, s, c->wav_pcm.p, c->wav_fo.p,
                       c->wav_ns.p, c->wav_wo.p, c->wav_segb.p, n_streams, nch, p->sample_rate, od);
    HIPCHK(hipGetLastError());
    if (!out_is_device) HIPCHK(hipMemcpyAsync(out, od, total, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return PAC_OK;
}
