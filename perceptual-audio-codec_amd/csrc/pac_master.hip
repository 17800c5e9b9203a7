// pac_master.hip -- gfx950 kernels of the master (.wak) profile: codec/ of the
// reference (M/S decision, six masking thresholds, bit reservoir, Huffman).
//
// Two passes over the call's blocks (file order: stream, block, channel).
// Pass 1 sweeps time slices (chunk = blocks t0..t0+S-1 of every stream of a
// stream group, PacMasterChunk) so the serial reservoir chain of every stream
// advances in parallel; pass 2 packs every channel-block at its final offset:
//   k_master_lrms   one workgroup per block: LRMS decision (codec.py:94-102)
//                   and the 64-line rows each coding mode's bands use
//   k_master_spec   one workgroup per block: FFT(a), FFT(b) of the windowed
//                   channels (the first in-place chains of calcBTHR)
//   k_master_thr    one workgroup per (block, variant pair): the six calcBTHR()
//                   calls of getStereoMaskThreshold (psychoac.py:540-562), each
//                   variant's spectrum derived from FFT(a), FFT(b) (M/S and the
//                   in-place Hann multiplies in the frequency domain) -> chunk
//                   thr[j][v][1024], only the rows the variant's bands use;
//                   the MLD pair one launch later, only the rows the M/S
//                   combination can select (+inf elsewhere)
//   k_master_front  one workgroup per block: MDCT L/R + overall scale
//                   (codec.py:237-246), M/S lines, MLD combination and per-band
//                   SMR selection (psychoac.py:533-682)
//   k_master_tail   one lane per STREAM of the chunk, its blocks in order:
//                   withdrawBits, the two BitAlloc calls with the extraBits carry
//                   (codec.py:222-260, bitalloc.py:129-184), scale factors,
//                   mantissas, 10-table Huffman length scoring, depositBits
//                   (codec.py:111-124) and the channel-block's byte count
//   (k_scan_* over the byte counts -> final offsets, as the origin profile)
//   k_master_pack   one workgroup per block (pass 2): from the tail's stored
//                   mantissa codes, sign bits, Huffman codes and LRMS packed
//                   MSB-first (pacfile.py:288-351) straight to the final offset.
// The LRMS + spectra of chunk i+1 run beside the front of chunk i, the tail of
// chunk i beside the thresholds of chunk i+1 (HIP streams, run_master).  With
// the MLD skip the threshold launch of chunk i carries chunk i-1's MLD rows
// and the front of chunk i-1 follows it.

#include "pac_bs.h"

// diagnostic (PAC_DEBUG_FLAGS 32 / 64, run_master): shader clock at phase mark
// k of every wave of the first PAC_PROF_WG workgroups of a launch
#define MPROF(k)                                                                                     \
    do {                                                                                             \
        if (src.prof && blockIdx.x < PAC_PROF_WG && (threadIdx.x & (WAVE - 1)) == 0)                 \
            src.prof[((int64_t)blockIdx.x * 4 + threadIdx.x / WAVE) * PAC_PROF_MARKS + (k)] =        \
                (long long)__builtin_amdgcn_s_memtime();                                             \
    } while (0)

// chunk-local scratch, local block j (thr and spec single-buffered, ordered by
// events in run_master; lines / smr / bandpeak triple-buffered between the
// front of chunk i and its tail, which runs beside chunk i+1's thresholds)
struct PacMasterChunkBuf {
    double* thr;        // [Bc][6][1024]
    double* lines;      // [Bc][2][1024]  LRMSmdctLines
    double* smr;        // [Bc][2][25]
    double* bandpeak;   // [Bc][2][25]    max |line| per band
    double2* spec;      // [Bc][2][PAC_SPEC_LD] FFT bins -2..1026 of a and b (k_master_spec)
    uint16_t* codes;    // [Bc][2][1024] signed mantissa codes, tail-internal (F.codes when the pack runs)
    // [Bc][2][1024] the MDCT lines of L and R (sine window, plain long frames,
    // stereo), computed by the side kernel from the LRMS spectra and read by the
    // front (k_master_front<true>); null: the front transforms the block itself
    double* mdct;
};
#define PAC_SPEC_LD 1040    // double2 per spectrum: bins -2..1026 at [bin + 2], padded to 256 B

// per-call fields; channel-block g = nch gb + ch (gb = global block, file order)
struct PacMasterFields {
    uint8_t* lrms;      // [nblocks][25]
    uint8_t* overall;   // [G]
    uint8_t* ba;        // [G][25]
    uint8_t* sf;        // [G][25]
    uint8_t* tid;       // [G]
    int32_t* nbytes;    // [G]  '<L' + payload bytes
    // per-block API only (else null): per MDCT line of g, the signed mantissa
    // code, its Huffman code (escape code ++ ba raw bits for an escape) and length
    uint32_t* dbg_mant;  // [G][1024]
    uint64_t* dbg_code;  // [G][1024]
    uint8_t* dbg_len;    // [G][1024]
    uint16_t* codes;     // [G][1024] signed mantissa codes (tail -> pack; 0 where ba == 0)
    const uint8_t* bsf;  // [nblocks] PAC_BS_* flags (block-switching extension), or null: off
    uint32_t* rowm;      // [nblocks] 64-line rows of L/R-coded bands (bits 0-15), M/S-coded (16-31), k_master_lrms
    // the tail's bitstream emission (null: k_master_pack packs from `codes`):
    // each channel-block's '<L' nBytes + payload at stg + stoff[g] (16-byte
    // aligned, padded to a whole LaneBits16 burst), placed at its file offset by k_master_place
    uint8_t* stg;
    int64_t* stoff;      // [G]
    unsigned long long* stg_next;   // bump allocator of stg
    int64_t stg_cap;
    uint32_t* msm;       // [nblocks] the LRMS flags as a band mask (bit b: band b M/S), k_master_lrms
    // [nblocks] the 64-line rows whose MLD_M (bits 0-15) / MLD_S (16-31) thresholds
    // exist: all ones from k_master_lrms, narrowed by k_master_thr's MLD skip; the
    // front reads no other MLD row (the others are +inf: min(., +inf) = .)
    uint32_t* mldm;
};

// A time slice of a stream group: blocks t0 .. t0+S-1 of the streams
// perm[s_first .. s_first+n_s-1]; local block j = k * S + (t - t0) for the
// stream perm[s_first + k].  run_master orders each group's streams by length
// (longest first) and lists only the streams still running at t0, choosing
// S per chunk, so the chunks of ragged stream sets stay full.
struct PacMasterChunk {
    int s_first, n_s;
    int64_t t0;
    int S;
    int nch;        // 2, or 1 for the mono master extension (no LRMS, one threshold)
    const int32_t* perm;
};

// global block id of local block j (and its stream, index in the stream),
// false if that stream has ended
struct ChunkPos { int64_t gb, t; int s; };
__device__ __forceinline__ bool chunk_block(const int64_t* __restrict__ blk_off, const PacMasterChunk& ck,
                                            int64_t j, ChunkPos* cp) {
    const int s = ck.perm[ck.s_first + (int)(j / ck.S)];
    const int64_t t = ck.t0 + j % ck.S;
    const int64_t b0 = blk_off[s];
    if (t >= blk_off[s + 1] - b0) return false;
    cp->gb = b0 + t;
    cp->t = t;
    cp->s = s;
    return true;
}

// LRMS-variant signals: the in-place window chains of EncodeDualChannel and
// getStereoMaskThreshold.  a = (x_L*sine)*hann, b = (x_R*sine)*hann;
// M = (a+b)/2, S = (a-b)/2; v2 = M*hann, v3 = S*hann, v4 = (M*hann)*hann, ...
// fl: block-switching flags of a long frame (the MDCT window's start / stop
// shapes, pac_bs.h), 0 = the plain window
__device__ __forceinline__ double variant_sample(const BlockPcm& rL, const BlockPcm& rR,
                                                 const PacTables* __restrict__ T, int v, int i, int fl) {
    const double h = T->hann[i];
    const double w = fl ? bs_long_win(T, fl, i) : T->sine[i];
    if (v == 1) return __dmul_rn(__dmul_rn(rR(i), w), h);
    const double a = __dmul_rn(__dmul_rn(rL(i), w), h);
    if (v == 0) return a;
    const double b = __dmul_rn(__dmul_rn(rR(i), w), h);
    double ms = ((v & 1) == 0) ? __dadd_rn(a, b) / 2.0 : __dsub_rn(a, b) / 2.0;
    ms = __dmul_rn(ms, h);
    if (v >= 4) ms = __dmul_rn(ms, h);
    return ms;
}

// The six variants' spectra from A = FFT(a), B = FFT(b) (bins 0..1024,
// X[-k] = conj X[k], X[2048-k] = conj X[k] for the real blocks): the M/S
// signals are (a +- b)/2 and an in-place Hann multiply (window.py:41-53,
// h[n] = (1 - cos(2 pi (n + 1/2)/N))/2) is, on the spectrum, the 3-tap
//   FFT(x h)[k] = X[k]/2 - e^{i pi/N} X[k-1]/4 - e^{-i pi/N} X[k+1]/4
// (v2 = M h, v3 = S h: one tap; v4 = M h h, v5 = S h h: two).  The same
// values as a direct FFT of the windowed signal up to rounding of the
// FFT's own order (bins within ~1e-16 of the spectrum's maximum).
#define PAC_HANN_C 0.9999988234517019      // cos(pi / 2048)
#define PAC_HANN_S 0.0015339801862847655   // sin(pi / 2048)
__device__ __forceinline__ double2 hann_tap(double2 xm, double2 x0, double2 xp) {
    // e^{i pi/N} xm + e^{-i pi/N} xp, then x0/2 - that/4
    const double sx = xm.x + xp.x, dy = xm.y - xp.y, sy = xm.y + xp.y, dx = xm.x - xp.x;
    const double re = __builtin_fma(PAC_HANN_C, sx, -(PAC_HANN_S * dy));
    const double im = __builtin_fma(PAC_HANN_C, sy, PAC_HANN_S * dx);
    return make_double2(__builtin_fma(-0.25, re, 0.5 * x0.x), __builtin_fma(-0.25, im, 0.5 * x0.y));
}
// ((double*)buf)[k] = |V_v[k]|^2 (dense), k < 1024; S = the block's spectra
// (bin k of A at S[k + 2], of B at S[PAC_SPEC_LD + k + 2], k = -2..1026).
// Each thread owns 4 consecutive bins (8 loads of the neighbourhood instead
// of 5 per bin) and stores them as two 16-byte halves, lanes 4-7 of every 8
// the second half first: each ds_write_b128 then covers 8 distinct 16-byte
// bank slots (the 4 consecutive doubles at a 32-byte lane stride would be a
// 2-way conflict, the old double2 .x layout an 8-way one).
template <int NT>
__device__ __forceinline__ void grp_variant_pow_regs(const double2* __restrict__ S, int v, int tid, double (&p)[4]) {
    static_assert(NT * 4 == 1024, "4 bins per thread");
    const int k0 = 4 * tid;
    double2 X[4];
    if (v < 2) {
        const double2* P = S + (v ? PAC_SPEC_LD : 0) + 2 + k0;
#pragma unroll
        for (int i = 0; i < 4; ++i) X[i] = P[i];
    } else {
        const double sg = (v & 1) ? -1.0 : 1.0;      // M = (a + b)/2, S = (a - b)/2
        auto ms = [&](int o) {                       // bin k0 + o - 2 of M or S
            const double2 a = S[k0 + o], b = S[PAC_SPEC_LD + k0 + o];
            return make_double2(0.5 * (a.x + sg * b.x), 0.5 * (a.y + sg * b.y));
        };
        double2 m[8];                                // bins k0 - 2 .. k0 + 5
        // the thread's own four bins from memory, the two on each side from the
        // neighbouring lanes (DPP wave shifts; the same values): half the loads;
        // a wave's edge lanes load theirs -- right after the own bins' loads,
        // in one branch, so that one round trip covers both (loaded and
        // combined in two branches after the shifts, they cost the variant
        // four serial round trips)
        const int lane = tid & (WAVE - 1);
#pragma unroll
        for (int i = 2; i < 6; ++i) m[i] = ms(i);
        double2 ea = make_double2(0.0, 0.0), eb = ea, fa = ea, fb = ea;   // A, B of the two edge bins
        if (lane == 0 || lane == WAVE - 1) {
            const int o = k0 + (lane ? 6 : 0);
            ea = S[o];
            eb = S[o + 1];
            fa = S[PAC_SPEC_LD + o];
            fb = S[PAC_SPEC_LD + o + 1];
        }
        auto sh = [](double2 x, auto ctrl) {
            constexpr int C = decltype(ctrl)::value;
            return make_double2(dpp_f64<C>(x.x, x.x), dpp_f64<C>(x.y, x.y));
        };
        m[0] = sh(m[4], std::integral_constant<int, PAC_DPP_WSHR1>{});
        m[1] = sh(m[5], std::integral_constant<int, PAC_DPP_WSHR1>{});
        m[6] = sh(m[2], std::integral_constant<int, PAC_DPP_WSHL1>{});
        m[7] = sh(m[3], std::integral_constant<int, PAC_DPP_WSHL1>{});
        const double2 e0 = make_double2(0.5 * (ea.x + sg * fa.x), 0.5 * (ea.y + sg * fa.y));   // as ms()
        const double2 e1 = make_double2(0.5 * (eb.x + sg * fb.x), 0.5 * (eb.y + sg * fb.y));
        if (lane == 0) { m[0] = e0; m[1] = e1; }
        if (lane == WAVE - 1) { m[6] = e0; m[7] = e1; }
        double2 h[6];                                // M h at bins k0 - 1 .. k0 + 4
#pragma unroll
        for (int i = 0; i < 6; ++i) h[i] = hann_tap(m[i], m[i + 1], m[i + 2]);
#pragma unroll
        for (int i = 0; i < 4; ++i) X[i] = v < 4 ? h[i + 1] : hann_tap(h[i], h[i + 1], h[i + 2]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = __builtin_fma(X[i].x, X[i].x, X[i].y * X[i].y);
}
// ... stored to LDS (the thread's 4 bins as two 16-byte halves, see above)
template <int NT>
__device__ __forceinline__ void grp_variant_pow_store(const double (&p)[4], double2* buf, int tid) {
    double2* pw2 = reinterpret_cast<double2*>(buf);
    const bool sw = tid & 4;
    pw2[2 * tid + (sw ? 1 : 0)] = sw ? make_double2(p[2], p[3]) : make_double2(p[0], p[1]);
    pw2[2 * tid + (sw ? 0 : 1)] = sw ? make_double2(p[0], p[1]) : make_double2(p[2], p[3]);
    grp_sync<NT>();
}

// one threshold variant of a block (k_master_thr): |V|^2 from the block's
// spectra, maskers, the rows the variant's bands use.
// diagnostic (PAC_DEBUG_FLAGS 128): shader clock at phase mark k of every wave
// (pm = this workgroup's marks, or null)
#define TPROF(k)                                                                                     \
    do {                                                                                             \
        if (pm && (threadIdx.x & (WAVE - 1)) == 0)                                                   \
            pm[(threadIdx.x / WAVE) * PAC_PROF_MARKS + (k)] = (long long)__builtin_amdgcn_s_memtime(); \
    } while (0)
// (p: the thread's four bins of the variant's |V[k]|^2, grp_variant_pow_regs)
// The MLD rows a block needs (bits r: MLD_M, 16 + r: MLD_S), recorded by its
// M/S workgroup for the MLD workgroup of the next launch in the block's MLD_S
// row slot: each wave its own word of the row's last 16 bytes, which the MLD
// workgroup reads before it stores any row
#define MLD_NEED_AT(mld_s_row) reinterpret_cast<uint32_t*>((mld_s_row) + PAC_HALFN - 2)
// PRUNE (an MLD variant in mode 1): rows that wave_masking_row<true> finds not
// needed are not stored and their bit is cleared in the LDS word *kept
template <bool PRUNE = false>
__device__ __forceinline__ void thr_variant(const PacTables* __restrict__ T, const double (&p)[4],
                                         double* __restrict__ out, int v, int rows, double2* buf, double2* tmp,
                                         int tid, long long* pm, int mk, int* kept = nullptr) {
    const int lane = tid & (WAVE - 1);
    // wave priority: the barrier-bound list building above the barrier-free
    // masking rows, so that a workgroup's waves reach its barriers sooner
    // while the rows of the other workgroups fill the issue slots (thr −2.5 %;
    // the tail and the emission, which co-run latency-bound, at 3)
    __builtin_amdgcn_s_setprio(1);
    grp_variant_pow_store<FRONT_NT>(p, buf, tid);
    TPROF(mk);
    const MaskerLists L = masker_lists(buf, tmp);
    const int nm = grp_find_maskers<FRONT_NT>(reinterpret_cast<const double*>(buf), T, v >= 4 ? 0.0 : 15.0, tid, L);
    TPROF(mk + 1);
    // rows claimed dynamically, most expensive first (as in k_origin_front);
    // the counter was reset by grp_find_maskers before its last barrier
    int* rowctr = L.misc;
    __builtin_amdgcn_s_setprio(0);
#pragma unroll 1
    while (true) {
        int k = 0;
        if (lane == 0) k = atomicAdd(rowctr, 1);
        k = __builtin_amdgcn_readfirstlane(k);
        if (k >= 16) break;
        const int r = (int)((PAC_ROW_ORDER >> (4 * k)) & 15);
        if (!((rows >> r) & 1)) continue;                   // no line of the row uses this variant
        double t;
        if constexpr (PRUNE) {
            // the M/S rows this MLD row is min-ed with: BTHR_M, BTHR_S of the
            // block (stored by its M/S workgroup in the previous launch), below
            // `out` in the block's six rows
            const double* bt = out - (v - 2) * PAC_HALFN;
            const double bm = bt[r * WAVE + lane], bsv = bt[PAC_HALFN + r * WAVE + lane];
            int gone = 0;
            t = v == 4 ? wave_masking_row<true>(L, nm, T, lane, r, bm, bsv, &gone)
                       : wave_masking_row<true>(L, nm, T, lane, r, bsv, bm, &gone);
            gone = __builtin_amdgcn_readfirstlane(gone);
            if (gone) {                                         // scalar (SCC) branch
                if (lane == 0) atomicAnd(kept, ~(1 << (r + (v == 5 ? 16 : 0))));
                continue;
            }
        } else {
            t = wave_masking_row(L, nm, T, lane, r);
        }
        // thresholds as intensities (k_master_front takes the SMRs as ratios,
        // pac_spl_ratio); the MLD pair as the intensities of MLD_M / MLD_S =
        // BTHR_*_MLD * mld (psychoac.py:582-583), the only form the front reads
        out[r * WAVE + lane] = v >= 4 ? pac_mld_intensity(t, T->mld[r * WAVE + lane]) : t;
    }
    TPROF(mk + 2);
}

// the MLD workgroup's surviving rows (kept[0]) to F.mldm at the address
// parked in kept[2..3], once every wave's pruning is in
__device__ __forceinline__ void mld_rows_back(int* kept, int tid) {
    lds_sync();
    if (tid == 0)
        *reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(
            *(volatile __attribute__((address_space(3))) unsigned long long*)(kept + 2)) = (uint32_t)kept[0];   // LDS read, global store
}

// One workgroup per (block, variant pair) -- {0,1} = L/R, {2,3} = M/S,
// {4,5} = M/S without the drop (MLD) -- runs the pair's variants one after the
// other: a third of the dispatches and row-mask passes of one workgroup per
// variant, and the two M/S variants of a pair read the same spectrum
// neighbourhoods.  Written as two straight-line calls, not a loop: a loop
// over the variants keeps ~80 more VGPRs live (loop-invariant addresses).
//
// mode 1 (the MLD skip, pipelined): the launch for chunk i runs the pairs
// {0,1}, {2,3} of chunk i (KA, ckA, bA blocks) and the MLD pair {4,5} of
// chunk i - 1 (KB, ckB, bB blocks), whose {2,3} rows the previous launch
// wrote.  THR_M = max(BTHR_M, min(BTHR_S, MLD_S)) (psychoac.py:582-591)
// equals BTHR_M on every line where BTHR_S <= BTHR_M, whatever MLD_S is (and
// THR_S = BTHR_S where BTHR_M <= BTHR_S): a line needs at most one of MLD_M,
// MLD_S.  The MLD workgroup reads the block's BTHR_M / BTHR_S rows, computes
// an MLD row only where one of its lines needs it and records which rows
// exist (F.mldm); the front takes +inf for the others (min(., +inf) = . : its
// combination then yields BTHR_M / BTHR_S there, as the reference's does).  On correlated stereo BTHR_M >
// BTHR_S almost everywhere: most blocks need no MLD_S row and skip that
// variant entirely.  One launch, three kinds of workgroup co-running as in
// mode 0 (the skip as a separate launch, or as a chain of four variants in
// one workgroup, measured slower than no skip at all).
__global__ __launch_bounds__(FRONT_NT) void k_master_thr(PacSource src, const PacTables* __restrict__ T,
                                                         PacMasterChunkBuf KA, PacMasterFields F,
                                                         PacMasterChunk ckA, PacMasterChunkBuf KB,
                                                         PacMasterChunk ckB, int64_t bA, int64_t bB, int mode) {
    __shared__ double2 buf[1024];                              // spectrum, then masker lists (region A)
    __shared__ __attribute__((aligned(16))) double2 tmp[1024]; // masker lists (region B)
    const int tid = threadIdx.x;
    const int64_t item = xcd_item(blockIdx.x, gridDim.x);
    // (block, pair) = (item / 3, item % 3); mode 1: pair 2 is the MLD pair of the
    // previous chunk's block -- interleaved with the others, so that the three
    // kinds co-run (dispatch follows the item order)
    const int npair = ckA.nch == 2 ? 3 : 1;     // mono master: BTHR_L only
    const int64_t j = item / npair;            // block within the chunk
    const int pi = (int)(item % npair);
    const bool mld = mode == 1 && pi == 2;     // an MLD workgroup of the previous chunk
    if (j >= (mld ? bB : bA)) return;
    const PacMasterChunkBuf& K = mld ? KB : KA;
    const PacMasterChunk& ck = mld ? ckB : ckA;
    const int vb = 2 * pi;
    const double2* spec = K.spec + j * 2 * PAC_SPEC_LD;
    // the M/S pair's first variant's |V|^2 straight away: its spectrum loads
    // then overlap the block lookup and the row-mask load below (three serial
    // round trips); an M/S pair nearly always has rows on stereo input (a
    // skipped one wastes the loads; the L/R and MLD pairs, often skipped,
    // load after their row masks)
    double p[4];
    const bool early = !mld && vb == 2 && ck.nch == 2;
    if (early) grp_variant_pow_regs<FRONT_NT>(spec, 2, tid, p);
    ChunkPos cp;
    if (!chunk_block(src.blk_off, ck, j, &cp)) return;     // uniform per workgroup
    const int64_t gb = cp.gb;
    const int fl = F.bsf ? F.bsf[gb] : 0;
    if (fl & PAC_BS_SHORT) return;                          // k_master_thr_short's
    // rows whose lines' bands use the pair: L/R (v < 2) where LRMS = 0, the
    // M/S thresholds (v >= 2) where LRMS = 1 (getStereoMaskThreshold takes
    // each band's SMR from one mode, psychoac.py:662-682; k_master_lrms
    // records both masks); none: nothing to do.  Mono: every row of a band.
    int rows;
    if (ck.nch == 2) {
        const uint32_t rm = F.rowm[gb];
        rows = (int)(vb >= 2 ? rm >> 16 : rm & 0xffffu);
    } else {
        rows = (2 << ((T->lower[PAC_NB - 1] + T->nlines[PAC_NB - 1] - 1) / WAVE)) - 1;
    }
    rows = __builtin_amdgcn_readfirstlane(rows);
    if (!rows) return;
    // phase clocks (PAC_DEBUG_FLAGS 128) only in a -DPAC_THR_PROF build: their
    // pointer would cost the kernel the SGPRs that keep it at 104 VGPRs
#ifdef PAC_THR_PROF
    long long* pm = (src.prof && blockIdx.x < PAC_PROF_WG) ? src.prof + (int64_t)blockIdx.x * 4 * PAC_PROF_MARKS
                                                          : nullptr;
#else
    long long* pm = nullptr;
#endif
    TPROF(0);
    int rows2 = rows;                          // the second variant's rows
    if (mld) {
        // the MLD rows needed (bits 0-15 MLD_M, 16-31 MLD_S), recorded by the
        // block's M/S workgroup in the previous launch (its rows still in
        // registers then): the rows that exist, for the front too (which takes
        // +inf for the others: no +inf rows are stored or read)
        const uint32_t* nw = MLD_NEED_AT(K.thr + (j * 6 + 5) * PAC_HALFN);
        const uint32_t need = nw[0] | nw[1] | nw[2] | nw[3];
        rows = __builtin_amdgcn_readfirstlane((int)(need & 0xffffu) & rows);
        rows2 = __builtin_amdgcn_readfirstlane((int)(need >> 16) & rows2);
        // the rows that exist, for the front: these, less the rows the pruning
        // below finds not needed -- kept in an LDS word with the mask's
        // address until the end (in registers they would push the kernel past
        // its SGPRs), written back after the variants
        if (tid == 0) {
            int* park = masker_lists(buf, tmp).misc + 2;
            park[0] = rows | (rows2 << 16);
            *reinterpret_cast<unsigned long long*>(park + 2) = reinterpret_cast<unsigned long long>(F.mldm + gb);
        }
    }
    // the variant's |V[k]|^2 from the block's spectra of a and b (k_master_spec)
    int* kept = masker_lists(buf, tmp).misc + 2;            // the MLD workgroup's surviving rows (above)
    if (mld) {         // the MLD pair (mode 1): both variants pruned, the surviving rows written back
        double* o4 = K.thr + (j * 6 + 4) * PAC_HALFN;
        if (rows) {
            grp_variant_pow_regs<FRONT_NT>(spec, 4, tid, p);
            thr_variant<true>(T, p, o4, 4, rows, buf, tmp, tid, pm, 1, kept);
        }
        if (rows2) {
            int t2 = tid;
            asm volatile("" : "+v"(t2));
            grp_variant_pow_regs<FRONT_NT>(spec, 5, t2, p);
            lds_sync();                                     // the first variant's lists are read
            thr_variant<true>(T, p, o4 + PAC_HALFN, 5, rows2, buf, tmp, t2, pm, 5, kept);
        }
        mld_rows_back(kept, tid);
        return;
    }
    if (rows) {
        if (!early) grp_variant_pow_regs<FRONT_NT>(spec, vb, tid, p);
        thr_variant(T, p, K.thr + (j * 6 + vb) * PAC_HALFN, vb, rows, buf, tmp, tid, pm, 1);
    }
    if (ck.nch != 2 || !rows2) return;
    int t2 = tid;                // opaque copy: no per-lane address of the first call is kept live for the second
    asm volatile("" : "+v"(t2));
    // the second variant's spectrum in registers while the other waves finish
    // the first one's rows (no LDS touched), then stored after the barrier
    grp_variant_pow_regs<FRONT_NT>(spec, vb + 1, t2, p);
    lds_sync();                                             // the first variant's lists are read
    TPROF(4);
    // mode 1, M/S pair: what the MLD-need pass below uses, parked in two free
    // words of the lists' counters across the variant (kept in registers it
    // would push the kernel past its SGPRs and 104 VGPRs)
    int* park = masker_lists(buf, tmp).misc + 2;
    if (t2 == 0) {
        const bool rec = mode == 1 && vb == 2;
        *reinterpret_cast<unsigned long long*>(park) =
            rec ? reinterpret_cast<unsigned long long>(K.thr + j * 6 * PAC_HALFN) : 0ull;
        park[2] = rows2;
    }
    thr_variant(T, p, K.thr + (j * 6 + vb + 1) * PAC_HALFN, vb + 1, rows2, buf, tmp, t2, pm, 5);
    TPROF(8);
    // wave-uniform by construction; readfirstlane makes it scalar for the
    // compiler too, so that the pass below (ballots) runs under no exec mask
    typedef volatile __attribute__((address_space(3))) unsigned long long lds_u64;   // an LDS read, not a flat one
    const unsigned long long pv = *(lds_u64*)park;
    const unsigned long long pbase = ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(pv >> 32)) << 32) |
                                     (unsigned)__builtin_amdgcn_readfirstlane((int)pv);
    if (pbase) {
        // the MLD rows this block needs: THR_S (psychoac.py:582-591) needs
        // MLD_M where BTHR_M > BTHR_S, THR_M needs MLD_S where BTHR_S > BTHR_M
        // -- from the rows this workgroup just stored (its other waves' stores,
        // read past the L1 from the L2: no HBM re-read of the rows a launch
        // later); each wave a quarter of the rows.  Every wave waits for its
        // own row stores to be acknowledged by the L2 (s_waitcnt vmcnt(0):
        // gfx9 counts stores in vmcnt; a workgroup-scope release emits no such
        // wait in non-tgsplit mode, and an agent-scope one would also write
        // the whole L2 back, measured 2x slower overall) before the barrier;
        // the readers' loads are agent-scope, i.e. from the L2, after it.
        __builtin_amdgcn_s_waitcnt(0x0f70);                 // vmcnt(0); expcnt, lgkmcnt unchanged
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        lds_sync();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int lane = t2 & (WAVE - 1), w = __builtin_amdgcn_readfirstlane(t2 / WAVE);
        const int prow = __builtin_amdgcn_readfirstlane(park[2]);
        // (the parked address cast back to a global pointer: global loads and
        // stores, not flat ones -- whose waits also drain the LDS operations)
        typedef __attribute__((address_space(1))) double gdouble;
        typedef __attribute__((address_space(1))) unsigned long long gu64;
        gdouble* blk = reinterpret_cast<gdouble*>(pbase);
        gu64* tm = reinterpret_cast<gu64*>(blk + 2 * PAC_HALFN);
        // the wave's four rows loaded together (one round trip; a row this
        // workgroup did not store is read too -- in bounds, stale -- and ignored)
        constexpr int NQ = 16 / (FRONT_NT / WAVE);
        double m[NQ], sv[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int r = w + q * (FRONT_NT / WAVE);
            m[q] = __builtin_bit_cast(double, __hip_atomic_load(tm + r * WAVE + lane, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT));
            sv[q] = __builtin_bit_cast(double, __hip_atomic_load(tm + PAC_HALFN + r * WAVE + lane, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT));
        }
        uint32_t need = 0u;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int r = w + q * (FRONT_NT / WAVE);
            if (!((prow >> r) & 1)) continue;
            if (__ballot(m[q] > sv[q])) need |= 1u << r;
            if (__ballot(sv[q] > m[q])) need |= 1u << (16 + r);
        }
        if (lane == 0) reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(blk + 6 * PAC_HALFN - 2)[w] = need;   // MLD_NEED_AT
    }
}

// Block-switching extension (pac_bs.h): the thresholds of a SHORT frame.  One
// 256-thread workgroup per (block, variant), wave k = short block k: the
// variant's in-place window chain on the block's 512 samples (short window,
// Hann, M/S as variant_sample), calcBTHR at N = 512, written interleaved
// (line 4 j + k) where the long thresholds go.
__global__ __launch_bounds__(256) void k_master_thr_short(PacSource src, const PacTables* __restrict__ T,
                                                          PacMasterChunkBuf K, PacMasterFields F,
                                                          PacMasterChunk ck) {
    // per wave (8 KB): FFT buffer + scratch; then the powers in the scratch and
    // the masker lists over the whole 8 KB (wave_threshold_short)
    __shared__ double2 bufs[4][2][256];
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), k = tid / WAVE;
    double* pw = reinterpret_cast<double*>(bufs[k][1]);      // = wave region + 4096
    const int64_t item = xcd_item(blockIdx.x, gridDim.x);
    const int nvar = ck.nch == 2 ? 6 : 1;
    const int64_t j = item / nvar;
    const int v = (int)(item % nvar);
    ChunkPos cp;
    if (!chunk_block(src.blk_off, ck, j, &cp)) return;
    const int64_t gb = cp.gb;
    if (!(F.bsf[gb] & PAC_BS_SHORT)) return;
    // rows (64 short lines = 256 interleaved ones) whose bands use this variant,
    // as k_master_thr: L/R where LRMS = 0, M/S where LRMS = 1; none: the wave is done
    int rows = 0;
    {
        const int want = v >= 2 ? 1 : 0;
        const int lend = T->lower[PAC_NB - 1] + T->nlines[PAC_NB - 1];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int li = 4 * (q * WAVE + lane) + k;
            const bool need = li < lend && F.lrms[gb * PAC_NB + T->band_of_line[li]] == want;
            if (__ballot(need)) rows |= 1 << q;
        }
    }
    if (!rows) return;                                       // wave-uniform (no barriers below)
    const BlockPcm rL(locate_sb(src, cp.s, cp.t, gb, 0));
    const BlockPcm rR(locate_sb(src, cp.s, cp.t, gb, ck.nch == 2 ? 1 : 0));
    const int o = 384 + 256 * k;
    auto d = [&](int i) {
        const double h = T->hann_s[i], w = T->sine_s[i];
        if (v == 1) return __dmul_rn(__dmul_rn(rR(o + i), w), h);
        const double a = __dmul_rn(__dmul_rn(rL(o + i), w), h);
        if (v == 0) return a;
        const double b = __dmul_rn(__dmul_rn(rR(o + i), w), h);
        double ms = ((v & 1) == 0) ? __dadd_rn(a, b) / 2.0 : __dsub_rn(a, b) / 2.0;
        ms = __dmul_rn(ms, h);
        if (v >= 4) ms = __dmul_rn(ms, h);
        return ms;
    };
    wave_spectrum_pow_short(d, T, bufs[k][0], bufs[k][1], pw, lane);
    double* out = K.thr + (j * 6 + v) * PAC_HALFN;
    wave_threshold_short(reinterpret_cast<char*>(bufs[k][0]), T, v >= 4 ? 0.0 : 15.0, lane, rows,
                         [&](int l, double t) { out[4 * l + k] = v >= 4 ? pac_mld_intensity(t, T->mld_s[l]) : t; });
}

// Block switching: attack flags, one wave per two blocks.  Lane (b, c, s)
// sums the first-difference energy of segment s (128 samples) of channel c
// of block b in sample order; the lanes of the new half's segments compare
// it with the mean of the 8 segments before it (pac_bs.h).
__global__ __launch_bounds__(64) void k_bs_attack(PacSource src, int64_t nblocks, uint8_t* __restrict__ att) {
    __shared__ double E[2][2][16];
    const int lane = threadIdx.x;
    const int b2 = lane >> 5, c = (lane >> 4) & 1, sg = lane & 15;
    const int64_t gb = (int64_t)blockIdx.x * 2 + b2;
    const bool live = gb < nblocks && c < src.n_ch;
    double e = 0.0;
    if (live) {
        const BlockPcm r(locate(src, gb, c));
        double xp = sg ? r.at(128 * sg - 1) : 0.0;      // per-lane blocks: at(), not the buffer path
        for (int n = 128 * sg; n < 128 * sg + 128; ++n) {
            const double x = r.at(n);
            const double dd = n ? __dsub_rn(x, xp) : 0.0;
            e = __dadd_rn(e, __dmul_rn(dd, dd));
            xp = x;
        }
    }
    E[b2][c][sg] = e;
    wave_sync();
    bool a = false;
    if (live && sg >= 8) {
        double m = 0.0;
        for (int q = sg - 8; q < sg; ++q) m = __dadd_rn(m, E[b2][c][q]);
        a = e > PAC_BS_RATIO * (m / 8.0) && e > PAC_BS_EMIN;
    }
    const unsigned long long bal = __ballot(a);
    if (gb < nblocks && (lane & 31) == 0) att[gb] = ((bal >> (32 * b2)) & 0xffffffffull) ? 1 : 0;
}

// Block switching: per block PAC_BS_* from the attack flags of its stream
// (short: an attack in it or the block before; PREV / NEXT: the neighbour's)
__global__ void k_bs_flags(const int64_t* __restrict__ blk_off, int n_streams, int64_t nblocks,
                           const uint8_t* __restrict__ att, uint8_t* __restrict__ fl) {
    const int64_t gb = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gb >= nblocks) return;
    int lo = 0, hi = n_streams;                 // stream: last s with blk_off[s] <= gb
    while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (blk_off[mid] <= gb) lo = mid; else hi = mid; }
    const int64_t t = gb - blk_off[lo], len = blk_off[lo + 1] - blk_off[lo];
    const bool sh = att[gb] || (t > 0 && att[gb - 1]);
    const bool pv = t > 0 && (att[gb - 1] || (t > 1 && att[gb - 2]));
    const bool nx = t + 1 < len && (att[gb + 1] || att[gb]);
    fl[gb] = (uint8_t)((sh ? PAC_BS_SHORT : 0) | (pv ? PAC_BS_PREV : 0) | (nx ? PAC_BS_NEXT : 0));
}

// --- numpy pairwise summation of a complex vector (loops_utils.h.src) -------
// np.sum over a band's complex values (n = 2 * count doubles): below 8
// doubles a plain loop, up to 128 an 8-accumulator block, above that the sum
// of the two halves split at (n/2) rounded down to a multiple of 8.  The
// leaves of that recursion (PacTables::lr_leaf_*, host-built per band
// layout) are summed one per lane; one lane per band then adds them in the
// recursion's order.

// leaf: doubles [0, n) of f(e0 + k), k < n/2
template <class F>
__device__ __forceinline__ double2 np_csum_leaf(const F& f, int e0, int n) {
    if (n < 8) {
        double sr = 0., si = 0.;
        for (int i = 0; i < n; i += 2) { const double2 z = f(e0 + i / 2); sr += z.x; si += z.y; }
        return make_double2(sr, si);
    }
    double r[8];
    double2 z0 = f(e0), z1 = f(e0 + 1), z2 = f(e0 + 2), z3 = f(e0 + 3);
    r[0] = z0.x; r[1] = z0.y; r[2] = z1.x; r[3] = z1.y;
    r[4] = z2.x; r[5] = z2.y; r[6] = z3.x; r[7] = z3.y;
    int i;
    for (i = 8; i < n - (n % 8); i += 8) {
        const int e = e0 + i / 2;
        z0 = f(e); z1 = f(e + 1); z2 = f(e + 2); z3 = f(e + 3);
        r[0] += z0.x; r[1] += z0.y; r[2] += z1.x; r[3] += z1.y;
        r[4] += z2.x; r[5] += z2.y; r[6] += z3.x; r[7] += z3.y;
    }
    double sr = ((r[0] + r[2]) + (r[4] + r[6]));
    double si = ((r[1] + r[3]) + (r[5] + r[7]));
    for (; i < n; i += 2) { const double2 z = f(e0 + i / 2); sr += z.x; si += z.y; }
    return make_double2(sr, si);
}

// the recursion's combine step over precomputed leaf sums (in leaf order)
template <int D>
__device__ double2 np_csum_combine(const double2* leaf, int& idx, int n) {
    if (D == 0 || n <= 128) return leaf[idx++];
    int n2 = n / 2;
    n2 -= n2 % 8;
    const double2 a = np_csum_combine<(D > 0 ? D - 1 : 0)>(leaf, idx, n2);
    const double2 b = np_csum_combine<(D > 0 ? D - 1 : 0)>(leaf, idx, n - n2);
    return make_double2(a.x + b.x, a.y + b.y);
}

// complex spectrum X[k], k < 1024, of a real 2048-block d, all in buf: the
// sample pairs staged, the one-buffer Stockham FFT, the real split in place
// (thread p reads and writes its own bin pair p, 1024 - p)
template <int NT, class DS>
__device__ __forceinline__ void grp_spectrum_cplx(const DS& d, const PacTables* __restrict__ T, double2* buf,
                                                  int tid) {
#pragma unroll 4
    for (int n0 = 0; n0 < 1024; n0 += NT) {
        const int n = n0 + tid;
        buf[n] = make_double2(d(2 * n), d(2 * n + 1));
    }
    grp_fft_stockham_1buf<10, NT>(buf, T->fft_tw, tid);
    const double2* Z = buf;
#pragma unroll
    for (int p0 = 0; p0 < 512; p0 += NT) {
        const int p = p0 + tid;
        int kk[2];
        kk[0] = p;
        kk[1] = p ? 1024 - p : 512;
        double2 X[2];
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const double2 A = Z[kk[side]];
            const double2 Bc = Z[(1024 - kk[side]) & 1023];
            const double2 e = make_double2(0.5 * (A.x + Bc.x), 0.5 * (A.y - Bc.y));
            const double2 o = make_double2(0.5 * (A.x - Bc.x), 0.5 * (A.y + Bc.y));
            const double2 wo = cmul(T->rfft_tw[kk[side]], o);
            X[side] = make_double2(e.x + wo.y, e.y - wo.x);
        }
        buf[kk[0]] = X[0];
        buf[kk[1]] = X[1];
    }
    grp_sync<NT>();
}

// the complex spectra of two real 2048-blocks dA, dB at once (as
// grp_spectrum_cplx on each: bit-identical), both FFTs stage by stage together
// (d4(n) = (dA(2n), dA(2n+1), dB(2n), dB(2n+1)): the staged pairs of both, fed
// straight into the first stage).  The real split hands every bin to
// put(u, k, X[k]) (u = 0: A, 1: B; k < 1024, and the real Nyquist bin k = 1024
// = sum_even - sum_odd); thread p computes its own bin pair p, 1024 - p from
// the pair's two FFT values only, so put may write them back in place.
template <int NT, class D4, class PUT>
__device__ __forceinline__ void grp_spectrum_cplx2p_put(const D4& d4, const PacTables* __restrict__ T,
                                                        double2* bufA, double2* bufB, int tid, const PUT& put) {
    grp_fft_stockham_1buf_x2<10, NT>(bufA, bufB, T->fft_tw, tid, d4);
#pragma unroll
    for (int p0 = 0; p0 < 512; p0 += NT) {
        const int p = p0 + tid;
        int kk[2];
        kk[0] = p;
        kk[1] = p ? 1024 - p : 512;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const double2* Z = u ? bufB : bufA;
            // X[k] = (Z[k] + conj Z[-k])/2 - i W^k (Z[k] - conj Z[-k])/2: the halves folded into
            // rfft_tw2 and the final fused multiply-adds
            const double2 A0 = Z[kk[0]], A1 = Z[kk[1]];
            const double2 B0 = p ? A1 : A0, B1 = p ? A0 : A1;        // Z[(1024 - k) & 1023]
            double2 X[2];
#pragma unroll
            for (int side = 0; side < 2; ++side) {
                const double2 A = side ? A1 : A0, Bc = side ? B1 : B0;
                const double2 wo = cmul_fma(T->rfft_tw2[kk[side]], make_double2(A.x - Bc.x, A.y + Bc.y));
                X[side] = make_double2(__builtin_fma(0.5, A.x + Bc.x, wo.y), __builtin_fma(0.5, A.y - Bc.y, -wo.x));
            }
            if (p == 0) put(u, 1024, make_double2(A0.x - A0.y, 0.0));
            put(u, kk[0], X[0]);
            put(u, kk[1], X[1]);
        }
    }
}
// ... with the spectra left in place in bufA, bufB (bins 0..1023)
template <int NT, class D4>
__device__ __forceinline__ void grp_spectrum_cplx2p(const D4& d4, const PacTables* __restrict__ T,
                                                    double2* bufA, double2* bufB, int tid) {
    grp_spectrum_cplx2p_put<NT>(d4, T, bufA, bufB, tid, [&](int u, int k, double2 X) {
        if (k < 1024) (u ? bufB : bufA)[k] = X;
    });
    grp_sync<NT>();
}

// One 256-thread workgroup per stereo block: the LRMS decision (codec.py:94-102)
// |sum(L^2 - R^2)| < 0.8 |sum(L^2 + R^2)| per band, over the complex FFT bins
// of the raw (unwindowed) blocks, with numpy's pairwise sums.  It runs first so
// that k_master_thr computes only the thresholds a band's coding mode uses.
// MDCT line k (mdct.py:49-82, N = 2048, n0 = 512.5, 2/N forward) of the
// sine-windowed block from the raw block's DFT X (the LRMS spectra): with
// w[n] = sin(pi (n + 1/2)/N) = (e^{i pi (n+1/2)/N} - e^{-i pi (n+1/2)/N}) / 2i the
// odd-frequency sum sum_n x w e^{-2 pi i n (k+1/2)/N} is (c X[k] - conj(c) X[k+1]) / 2i,
// c = e^{i pi/2N}, so X_mdct[k] = Im(e^{-ia} X[k] - e^{-ib} X[k+1]) / N,
// a, b = 2 pi n0 (k + 1/2)/N -+ pi/2N (T->mdct_tw2).  Mathematically the
// reference's transform; rounding of the same class as an FFT's (the terms
// are bounded by the raw spectrum's bins).  Exactly-zero lines take the
// reference's signed zero.
// (tw = T->mdct_tw2[k], zn = T->mdct_zero_neg[k]: the caller may load them
// ahead; the exact-zero sign applied by a select -- under "r == 0" its load
// was a branch of its own, which kept the next line's loads behind it)
__device__ __forceinline__ double mdct_from_dft_tw(double2 x0, double2 x1, double4 tw, int zn) {
    double r = x0.y * tw.x;
    r = __builtin_fma(-x0.x, tw.y, r);
    r = __builtin_fma(-x1.y, tw.z, r);
    r = __builtin_fma(x1.x, tw.w, r);
    return r == 0.0 ? __longlong_as_double((long long)(zn != 0) << 63) : r;
}
__device__ __forceinline__ double mdct_from_dft(double2 x0, double2 x1, const PacTables* __restrict__ T, int k) {
    return mdct_from_dft_tw(x0, x1, T->mdct_tw2[k], T->mdct_zero_neg[k]);
}

// parity probe (pac_debug_mdct_dft): blocks 2 i, 2 i + 1 of `data` (n blocks
// of 2048 raw samples) as the L and R of one block, the MDCT lines of both
// exactly as lrms_block derives them (same FFT, same split, mdct_from_dft)
__global__ __launch_bounds__(256) void k_debug_mdct_dft(const PacTables* __restrict__ T,
                                                        const double* __restrict__ data, int n,
                                                        double* __restrict__ X) {
    __shared__ double2 bufA[1024], bufB[1024];
    const int tid = threadIdx.x;
    const int64_t b0 = 2 * (int64_t)blockIdx.x;
    const double* dA = data + b0 * PAC_N;
    const double* dB = b0 + 1 < n ? dA + PAC_N : nullptr;
    double nyA = 0.0, nyB = 0.0;
    grp_spectrum_cplx2p_put<256>([&](int q) {
        return make_double4(dA[2 * q], dA[2 * q + 1], dB ? dB[2 * q] : 0.0, dB ? dB[2 * q + 1] : 0.0);
    }, T, bufA, bufB, tid, [&](int u, int k, double2 Z) {
        if (k < 1024) (u ? bufB : bufA)[k] = Z;
        else if (u) nyB = Z.x;
        else nyA = Z.x;
    });
    lds_sync();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = 1023 - 256 * i - tid;
        const double2 a1 = k == 1023 ? make_double2(nyA, 0.0) : bufA[k + 1];
        const double2 b1 = k == 1023 ? make_double2(nyB, 0.0) : bufB[k + 1];
        X[b0 * PAC_HALFN + k] = mdct_from_dft(bufA[k], a1, T, k);
        if (dB) X[(b0 + 1) * PAC_HALFN + k] = mdct_from_dft(bufB[k], b1, T, k);
    }
}

// CODED (a stereo sine-window call without block switching, whose front reads
// its lines from here): `mdct` receives the block's final coded lines instead
// of the MDCT lines -- each channel scaled by 2^(overall scale factor)
// (codec.py:237-246, the scale from the block maximum of its MDCT lines), and
// M = (L + R)/2, S = (L - R)/2 of the scaled channels in the bands the LRMS
// decision codes M/S (psychoac.py:551-555, codec.py:94-102) -- exactly the
// front's expressions; the overall scale factors go to F.overall.  The lines
// stay in registers across the decision (the front then stores no lines: 16 KB
// per block less in the side/front window).
template <bool CODED>
__device__ __forceinline__ void lrms_block(const PacSource& src, const PacTables* __restrict__ T,
                                           const PacMasterFields& F, const ChunkPos& cp, double2* bufA,
                                           double2* bufB, double* __restrict__ mdct,
                                           const BlockRef* pre = nullptr) {
    const int tid = threadIdx.x;
    const int64_t gb = cp.gb;
    // the block's PCM references: from the caller when it has them (the fused
    // kernel locates the block once for both of its stages)
    const BlockRef bL = pre ? pre[0] : locate_sb(src, cp.s, cp.t, gb, 0);
    const BlockPcm rL(bL);
    const BlockPcm rR(pre ? pre[1] : locate_sb(src, cp.s, cp.t, gb, 1));
    // the leaf and band tables, loaded before the FFTs (their round trips
    // overlap the transform instead of following it)
    const int lf = tid >> 2, sub = tid & 3;
    const bool has = lf < T->lr_nleaf;
    int e0 = 0, n = 0, lo = 0;
    if (has) {
        e0 = T->lr_leaf_e0[lf];
        n = T->lr_leaf_n[lf];
        lo = T->lower[T->lr_leaf_band[lf]];
    }
    int fl0 = 0, nlb = 0, lob = 0;
    if (tid < PAC_NB) {
        fl0 = T->lr_first_leaf[tid];
        nlb = T->nlines[tid];
        lob = T->lower[tid];
    }
    MPROF(0);
    // bins 0..1023 in place; the real Nyquist bins (thread 0) kept for the MDCT
    double nyA = 0.0, nyB = 0.0;
    auto put = [&](int u, int k, double2 X) {
        if (k < 1024) (u ? bufB : bufA)[k] = X;
        else if (u) nyB = X.x;
        else nyA = X.x;
    };
    if (!rL.f) {
        const StereoFrames sf(bL);
        grp_spectrum_cplx2p_put<256>([&](int n) {      // frames 2n, 2n+1: (L0, R0), (L1, R1)
            const double2 f0 = sf(2 * n), f1 = sf(2 * n + 1);
            return make_double4(f0.x, f1.x, f0.y, f1.y);
        }, T, bufA, bufB, tid, put);
    } else {
        grp_spectrum_cplx2p_put<256>([&](int n) {
            return make_double4(rL(2 * n), rL(2 * n + 1), rR(2 * n), rR(2 * n + 1));
        }, T, bufA, bufB, tid, put);
    }
    lds_sync();
    MPROF(1);
    // (the spectra and MDCT lines are stored non-temporally: a chunk's 1.6 GB
    // are read back from HBM by the next kernels anyway, and streaming them
    // through the L2 evicted the PCM block the spectra stage reads again:
    // configs[2] +1.3 %, same-box A/B)
    double cl[4], cr[4];                           // CODED: the lines until the decision is in
    double mL = 0.0, mR = 0.0;
    // the front's MDCT lines from these spectra; thread 0 owns line 1023 (CODED:
    // after the leaf sums below, so that the lines and the sums are not live
    // together: the kernel's 5 waves per SIMD need <= 96 VGPRs)
    auto mdct_lines = [&]() {
        // each line's twiddles loaded one line ahead: the next line's round
        // trip overlaps this line's arithmetic (one exposed round trip, not four)
        double4 twn = T->mdct_tw2[1023 - tid];
        int znn = T->mdct_zero_neg[1023 - tid];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = 1023 - 256 * i - tid;
            const double4 tw = twn;
            const int zn = znn;
            if (i < 3) {
                twn = T->mdct_tw2[k - 256];
                znn = T->mdct_zero_neg[k - 256];
            }
            const double2 a0 = bufA[k], b0 = bufB[k];
            const double2 a1 = k == 1023 ? make_double2(nyA, 0.0) : bufA[k + 1];
            const double2 b1 = k == 1023 ? make_double2(nyB, 0.0) : bufB[k + 1];
            const double xl = mdct_from_dft_tw(a0, a1, tw, zn), xr = mdct_from_dft_tw(b0, b1, tw, zn);
            if constexpr (CODED) {
                cl[i] = xl;
                cr[i] = xr;
                mL = fmax(mL, fabs(xl));
                mR = fmax(mR, fabs(xr));
            } else {
                __builtin_nontemporal_store(xl, mdct + k);
                __builtin_nontemporal_store(xr, mdct + PAC_HALFN + k);
            }
        }
    };
    if (!CODED && mdct) mdct_lines();
    auto sq = [](double2 z) {   // np.power(z, 2) == z*z (npy_cpow n == 2)
        return make_double2(__dsub_rn(__dmul_rn(z.x, z.x), __dmul_rn(z.y, z.y)),
                            __dadd_rn(__dmul_rn(z.x, z.y), __dmul_rn(z.y, z.x)));
    };
    // leaf sums (np_csum_leaf) of both sums -- sum(L^2 - R^2) and sum(L^2 + R^2) --
    // by the four lanes of a quad per leaf: lane `sub` runs numpy's accumulators
    // r[2 sub], r[2 sub + 1] (complex elements e0 + 4 k + sub) in order, the
    // quad then combines ((r0 + r2) + (r4 + r6)) by DPP, lane 0 adds the tail
    // elements: numpy's exact operation order
    auto zz = [&](int e, double2& d, double2& sm) {
        const double2 a = sq(bufA[lo + e]), c = sq(bufB[lo + e]);
        d = make_double2(__dsub_rn(a.x, c.x), __dsub_rn(a.y, c.y));
        sm = make_double2(__dadd_rn(a.x, c.x), __dadd_rn(a.y, c.y));
    };
    const int nfull = n >= 8 ? n - n % 8 : 0;
    double2 rd = make_double2(0.0, 0.0), rs = rd;
    for (int i = 0; i < nfull; i += 8) {
        double2 d, sm;
        zz(e0 + i / 2 + sub, d, sm);
        if (i == 0) { rd = d; rs = sm; }
        else {
            rd.x = __dadd_rn(rd.x, d.x); rd.y = __dadd_rn(rd.y, d.y);
            rs.x = __dadd_rn(rs.x, sm.x); rs.y = __dadd_rn(rs.y, sm.y);
        }
    }
    auto quad2 = [](double v) {
        const double a = v + dpp_full_f64<PAC_DPP_QXOR1>(v);      // r[2s] + r[2s+2] pairs
        return a + dpp_full_f64<PAC_DPP_QXOR2>(a);
    };
    rd.x = quad2(rd.x); rd.y = quad2(rd.y);
    rs.x = quad2(rs.x); rs.y = quad2(rs.y);
    double2 lv0 = make_double2(0.0, 0.0), lv1 = lv0;
    if (has && sub == 0) {
        if (n >= 8) { lv0 = rd; lv1 = rs; }
        for (int i = nfull; i < n; i += 2) {      // the tail (n < 8: the whole plain loop from 0)
            double2 d, sm;
            zz(e0 + i / 2, d, sm);
            lv0.x = __dadd_rn(lv0.x, d.x); lv0.y = __dadd_rn(lv0.y, d.y);
            lv1.x = __dadd_rn(lv1.x, sm.x); lv1.y = __dadd_rn(lv1.y, sm.y);
        }
    }
    if (CODED) mdct_lines();
    lds_sync();                                    // every spectrum read: bufA's start holds the leaves
    double2* leafv0 = bufA;
    double2* leafv1 = bufA + 64;
    if (has && sub == 0) { leafv0[lf] = lv0; leafv1[lf] = lv1; }
    // CODED: the waves' maxima of |line| (max is order-free: the front's block
    // maxima exactly) and then the decision's band mask in bufB's start
    double* wmax = reinterpret_cast<double*>(bufB);
    if constexpr (CODED) {
        mL = wave_max(mL);
        mR = wave_max(mR);
        if ((tid & (WAVE - 1)) == 0) {
            wmax[tid / WAVE] = mL;
            wmax[4 + tid / WAVE] = mR;
        }
    }
    lds_sync();
    if (tid < WAVE) {                              // wave 0: the decisions and the rows they select
        int rows = 0, ms = 0;
        if (tid < PAC_NB) {
            int i0 = fl0, i1 = i0;
            const int nl = nlb;
            const double2 sd = np_csum_combine<5>(leafv0, i0, 2 * nl);
            const double2 ss = np_csum_combine<5>(leafv1, i1, 2 * nl);
            ms = hypot(sd.x, sd.y) < 0.8 * hypot(ss.x, ss.y) ? 1 : 0;
            F.lrms[gb * PAC_NB + tid] = (uint8_t)ms;
            if (nl) {                              // the 64-line rows of the band's lines
                const int r0 = lob / WAVE, r1 = (lob + nl - 1) / WAVE;
                rows = ((2 << r1) - (1 << r0)) << (ms ? 16 : 0);
            }
        }
        rows = wave_or_i(rows);
        const uint32_t msm = (uint32_t)__ballot(ms);
        if (tid == 0) {
            F.rowm[gb] = (uint32_t)rows;
            F.msm[gb] = msm;
            F.mldm[gb] = 0xffffffffu;              // every MLD row, unless the MLD skip narrows it
            if (CODED) reinterpret_cast<uint32_t*>(wmax + 8)[0] = msm;
        }
    }
    if constexpr (CODED) {
        // the lines' bands loaded before the barrier (unconditionally: under
        // the k < lend test the load was issued after it and waited on at once)
        const int lend = T->lower[PAC_NB - 1] + T->nlines[PAC_NB - 1];
        int bl[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) bl[i] = T->band_of_line[1023 - 256 * i - tid];
        lds_sync();
        const int oL = pac_scale_factor(fmax(fmax(wmax[0], wmax[1]), fmax(wmax[2], wmax[3])), 5);
        const int oR = pac_scale_factor(fmax(fmax(wmax[4], wmax[5]), fmax(wmax[6], wmax[7])), 5);
        const uint32_t msm = reinterpret_cast<const uint32_t*>(wmax + 8)[0];
        const double gL = (double)(1 << oL), gR = (double)(1 << oR);
        if (tid == 0) {
            F.overall[gb * 2] = (uint8_t)oL;
            F.overall[gb * 2 + 1] = (uint8_t)oR;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = 1023 - 256 * i - tid;
            const bool ms = k < lend && ((msm >> bl[i]) & 1u);
            const double xl = __dmul_rn(cl[i], gL), xr = __dmul_rn(cr[i], gR);
            const double M = __dadd_rn(xl, xr) / 2.0, S = __dsub_rn(xl, xr) / 2.0;
            __builtin_nontemporal_store(ms ? M : xl, mdct + k);
            __builtin_nontemporal_store(ms ? S : xr, mdct + PAC_HALFN + k);
        }
    }
    MPROF(2);
}


__global__ __launch_bounds__(256) void k_master_lrms(PacSource src, const PacTables* __restrict__ T,
                                                     PacMasterFields F, PacMasterChunk ck) {
    __shared__ double2 bufA[1024], bufB[1024];    // 32 KB: the L and R spectra, then the leaf sums
    ChunkPos cp;
    if (!chunk_block(src.blk_off, ck, blockIdx.x, &cp)) return;
    lrms_block<false>(src, T, F, cp, bufA, bufB, nullptr);
}

// One 256-thread workgroup per stereo block: the complex spectra A = FFT(a),
// B = FFT(b), bins 0..1024, of the two channels' windowed blocks
// a = (x_L w) hann, b = (x_R w) hann (the first in-place chains of
// EncodeDualChannel / calcBTHR, psychoac.py:540-545) -> K.spec, from which
// k_master_thr derives all six threshold variants' spectra (grp_variant_pow).
__device__ __forceinline__ void spec_block(const PacSource& src, const PacTables* __restrict__ T,
                                           const PacMasterChunkBuf& K, const PacMasterFields& F,
                                           const PacMasterChunk& ck, const ChunkPos& cp, int64_t j, double2* bufA,
                                           double2* bufB, const BlockRef* pre = nullptr) {
    const int tid = threadIdx.x;
    const int64_t gb = cp.gb;
    const int fl = F.bsf ? F.bsf[gb] : 0;
    if (fl & PAC_BS_SHORT) return;                 // k_master_thr_short's
    const BlockRef bL = pre ? pre[0] : locate_sb(src, cp.s, cp.t, gb, 0);
    const BlockPcm rL(bL);
    const BlockPcm rR(pre ? pre[1] : locate_sb(src, cp.s, cp.t, gb, ck.nch == 2 ? 1 : 0));   // mono: B = A, unused
    // bins -2..1026 at o[bin + 2], written by the real split straight from its
    // registers (no LDS round trip): the mirrored edge bins X[-k] = X[2048-k] =
    // conj X[k] stored too, so the taps of k_master_thr need no index arithmetic
    double2* o = K.spec + j * 2 * PAC_SPEC_LD + 2;
    auto put = [&](int u, int k, double2 X) {
        double2* q = o + u * PAC_SPEC_LD;
        nt_store(q + k, X);
        if (k == 1 || k == 2) q[-k] = make_double2(X.x, -X.y);
        if (k == 1022 || k == 1023) q[2048 - k] = make_double2(X.x, -X.y);
    };
    if (ck.nch == 2 && !rL.f) {
        const StereoFrames sf(bL);
        grp_spectrum_cplx2p_put<256>([&](int n) {   // frames 2n, 2n+1 of both channels, one load each
            const int i0 = 2 * n;
            const double2 f0 = sf(i0), f1 = sf(i0 + 1);
            const double2 h = *reinterpret_cast<const double2*>(T->hann + i0);
            const double2 w = fl ? make_double2(bs_long_win(T, fl, i0), bs_long_win(T, fl, i0 + 1))
                                 : *reinterpret_cast<const double2*>(T->sine + i0);
            return make_double4(__dmul_rn(__dmul_rn(f0.x, w.x), h.x), __dmul_rn(__dmul_rn(f1.x, w.y), h.y),
                                __dmul_rn(__dmul_rn(f0.y, w.x), h.x), __dmul_rn(__dmul_rn(f1.y, w.y), h.y));
        }, T, bufA, bufB, tid, put);
    } else {
        grp_spectrum_cplx2p_put<256>([&](int n) {
            return make_double4(variant_sample(rL, rR, T, 0, 2 * n, fl), variant_sample(rL, rR, T, 0, 2 * n + 1, fl),
                                variant_sample(rL, rR, T, 1, 2 * n, fl), variant_sample(rL, rR, T, 1, 2 * n + 1, fl));
        }, T, bufA, bufB, tid, put);
    }
    MPROF(3);
    MPROF(4);
}


__global__ __launch_bounds__(256) void k_master_spec(PacSource src, const PacTables* __restrict__ T,
                                                     PacMasterChunkBuf K, PacMasterFields F, PacMasterChunk ck) {
    __shared__ double2 bufA[1024], bufB[1024];    // 32 KB
    ChunkPos cp;
    if (!chunk_block(src.blk_off, ck, blockIdx.x, &cp)) return;
    spec_block(src, T, K, F, ck, cp, blockIdx.x, bufA, bufB);
}

// Both, one workgroup per block: the LRMS decisions, then the windowed
// spectra in the same 32 KB (one launch and one workgroup prologue per block
// on the side stream instead of two).
// CODED: the call's front is k_master_front<true>, whose coded lines and
// overall scale factors this kernel writes (lrms_block<true>: K.lines, F.overall).
// (5 waves per SIMD, as its LDS allows)
template <bool CODED>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_master_lrms_spec(PacSource src, const PacTables* __restrict__ T,
                                                          PacMasterChunkBuf K, PacMasterFields F, PacMasterChunk ck) {
    __shared__ double2 bufA[1024], bufB[1024];    // 32 KB
    ChunkPos cp;
    if (!chunk_block(src.blk_off, ck, blockIdx.x, &cp)) return;
    // K.mdct (the <false> instantiation): set by the host for sine-window
    // stereo calls whose front is k_master_front<false> -- block switching, or
    // PAC_SIDE_CODED=0 -- the plain long frames' lines (the other frames
    // transform in the front).  waves_per_eu(5) holds both instantiations at
    // 95 VGPRs with no spills (libpacgpu.resources.json, tests/test_host.py).
    // (CODED calls are stereo; the nch test is kept in both instantiations: without
    // it the compiler schedules the CODED kernel into 111 VGPRs, or 17 spills at 96)
    // the block's PCM located once for both stages: after the LRMS stage's
    // stores the spectra stage would reload the stream offsets from global
    // memory (not provably unchanged) and wait on them
    const BlockRef pre[2] = {locate_sb(src, cp.s, cp.t, cp.gb, 0),
                             locate_sb(src, cp.s, cp.t, cp.gb, ck.nch == 2 ? 1 : 0)};
    if (CODED && ck.nch == 2) {
        lrms_block<true>(src, T, F, cp, bufA, bufB, K.lines + blockIdx.x * 2 * PAC_HALFN, pre);
    } else if (!CODED && ck.nch == 2) {
        const bool md = K.mdct && !(F.bsf && F.bsf[cp.gb]);
        lrms_block<false>(src, T, F, cp, bufA, bufB, md ? K.mdct + blockIdx.x * 2 * PAC_HALFN : nullptr, pre);
    }
    lds_sync();                                   // the leaf sums are read before the spectra overwrite them
    spec_block(src, T, K, F, ck, cp, blockIdx.x, bufA, bufB, pre);
}

// lane i <- lane i + OFF of its DPP row (row_shl:OFF; bound_ctrl: 0 past the
// row, never taken: the callers' segments end inside the row)
template <int OFF>
__device__ __forceinline__ unsigned long long row_shl_u64(unsigned long long v) {
    const int lo = __builtin_amdgcn_mov_dpp((int)v, 0x100 + OFF, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(v >> 32), 0x100 + OFF, 0xf, 0xf, true);
    return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}
template <int OFF>
__device__ __forceinline__ void seg_max_step(unsigned long long& k0, unsigned long long& k1,
                                             unsigned long long& k2, unsigned long long& k3, bool take) {
    const unsigned long long o0 = row_shl_u64<OFF>(k0), o1 = row_shl_u64<OFF>(k1);
    const unsigned long long o2 = row_shl_u64<OFF>(k2), o3 = row_shl_u64<OFF>(k3);
    if (take) {
        k0 = o0 > k0 ? o0 : k0;
        k1 = o1 > k1 ? o1 : k1;
        k2 = o2 > k2 ? o2 : k2;
        k3 = o3 > k3 ? o3 : k3;
    }
}

// One 256-thread workgroup per stereo block: MDCT L/R and overall scales, M/S
// lines, MLD threshold combination, SMR selection and the band maxima (LDS
// atomic max on order-preserving keys).  Only the thresholds of each band's
// coding mode are read (k_master_thr computes no others).  FAST: a stereo
// sine-window call without block switching, whose coded lines and overall
// scale factors the side kernel formed from the LRMS spectra
// (k_master_lrms_spec<true>: K.lines, F.overall): no transform, no scaling and
// no line stores here, 1.5 KB of LDS.  (The general kernel reads the side
// kernel's MDCT lines, K.mdct, where it has them.)
template <bool FAST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_master_front(PacSource src, const PacTables* __restrict__ T,
                                                      PacMasterChunkBuf K, PacMasterFields F,
                                                      PacMasterChunk ck) {
    __shared__ double2 bufA[FAST ? 1 : 1024], bufB[FAST ? 96 : 1024];    // 32 KB (5 workgroups per CU) / 1.5 KB
    // after the MDCTs: SMR 0/1, |line| 0/1, max|X| L/R keys and the LRMS flags
    // in the free upper half of bufB
    unsigned long long (*key)[32] = reinterpret_cast<unsigned long long (*)[32]>(FAST ? bufB : bufB + 512);
    const int tid = threadIdx.x;
    const int64_t j = blockIdx.x;
    ChunkPos cp;
    if (!chunk_block(src.blk_off, ck, j, &cp)) return;
    const int64_t gb = cp.gb;
    const bool st = FAST || ck.nch == 2;         // mono master: channel 0 alone, LRMS all 0
    const int fl = (!FAST && F.bsf) ? F.bsf[gb] : 0;   // block-switching flags (pac_bs.h), 0: off
    const bool sh = fl & PAC_BS_SHORT;
    // each thread's four lines l = 256 i + tid: bands, and the block's LRMS
    // band mask, loaded before the MDCT (no wait: the LDS barriers leave them
    // in flight) so that the threshold loads can all issue right after it
    const int lend = T->lower[PAC_NB - 1] + T->nlines[PAC_NB - 1];
    int sp4[4];                                   // band | its first and last line (band_span)
#pragma unroll
    for (int i = 0; i < 4; ++i) sp4[i] = T->band_span[i * 256 + tid];
    const uint32_t msm = st ? F.msm[gb] : 0u;     // mono: all L/R
    const uint32_t mldm = st ? F.mldm[gb] : 0u;   // the MLD rows that exist (k_master_thr)
    MPROF(0);

    // --- MDCT L and R, overall scale factors (codec.py:237-246) -------------
    double xl4[4], xr4[4];   // FAST: the coded lines
    // the lines come from the side kernel: every block of a FAST call (coded,
    // K.lines); with block switching, the plain long frames (MDCT, K.mdct)
    const bool from_md = FAST || (K.mdct && st && !fl);
    if (from_md) {
        const double* md = (FAST ? K.lines : K.mdct) + j * 2 * PAC_HALFN;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            xl4[i] = md[i * 256 + tid];
            xr4[i] = md[PAC_HALFN + i * 256 + tid];
        }
    }
    const double* XL = nullptr;
    const double* XR = nullptr;
    if (from_md) {
    } else if (sh) {   // four short MDCTs per channel, interleaved (scratch: the buffers' upper halves)
        const BlockPcm rL(locate_sb(src, cp.s, cp.t, gb, 0));
        const BlockPcm rR(locate_sb(src, cp.s, cp.t, gb, st ? 1 : 0));
        double* xl = reinterpret_cast<double*>(bufA);
        double* xr = reinterpret_cast<double*>(bufB);
        grp_short_mdct(rL, T, bufA + 512, bufB + 512, xl, tid);
        if (st) grp_short_mdct(rR, T, bufA + 512, bufB + 512, xr, tid);
        XL = xl;
        XR = xr;
    } else if (fl) {   // long frame next to a short one: start / stop window
        const BlockPcm rL(locate_sb(src, cp.s, cp.t, gb, 0));
        const BlockPcm rR(locate_sb(src, cp.s, cp.t, gb, st ? 1 : 0));
        XL = grp_mdct<256>([&](int i) { return __dmul_rn(rL(i), bs_long_win(T, fl, i)); }, T, bufA, tid);
        if (st) XR = grp_mdct<256>([&](int i) { return __dmul_rn(rR(i), bs_long_win(T, fl, i)); }, T, bufB, tid);
    } else if (st) {   // both channels' MDCTs stage by stage together
        const BlockPcm rL(locate_sb(src, cp.s, cp.t, gb, 0));
        const BlockPcm rR(locate_sb(src, cp.s, cp.t, gb, 1));
        if (!rL.f) {
            grp_mdct2<256>([&](int i, int u) { return __dmul_rn(stereo_sample(rL, i, u), T->sine[i]); },
                           T, bufA, bufB, tid);
        } else {
            grp_mdct2<256>([&](int i, int u) { return __dmul_rn(u ? rR(i) : rL(i), T->sine[i]); },
                           T, bufA, bufB, tid);
        }
        XL = reinterpret_cast<const double*>(bufA);
        XR = reinterpret_cast<const double*>(bufB);
    } else {
        const BlockPcm rL(locate_sb(src, cp.s, cp.t, gb, 0));
        XL = grp_mdct<256>([&](int i) { return __dmul_rn(rL(i), T->sine[i]); }, T, bufA, tid);
    }
    // (every MDCT ended with a barrier: the upper halves are free)
    MPROF(1);
    // the thresholds of the four lines' coding modes, all loads in flight
    // together (the selection loop below stores to HBM, which the compiler
    // cannot move these loads across): L, R or M, S and the MLD-scaled M, S
    const double* thr = K.thr + j * 6 * PAC_HALFN;
    // (the MLD pair under the line's mode mask: an L/R line fetches 16 B, an
    // M/S line 32 B -- the front is HBM-heavy, 50 KB per block); the MLD pair arrives as MLD_M, MLD_S
    double t4[4][4];
    int ms4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int l = i * 256 + tid;
        ms4[i] = l < lend ? (int)((msm >> (sp4[i] >> 20)) & 1u) : 0;
        const double* tp = thr + (ms4[i] ? 2 * PAC_HALFN : 0) + l;
        t4[i][0] = tp[0];
        t4[i][1] = tp[PAC_HALFN];
        // the MLD pair: M/S lines of rows whose MLD rows exist only (masked
        // lanes fetch nothing); +inf elsewhere, as the reference's min() takes it
        const int rw = l / WAVE;
        t4[i][2] = t4[i][3] = INFINITY;
        if (ms4[i] && ((mldm >> rw) & 1u)) t4[i][2] = tp[2 * PAC_HALFN];
        if (ms4[i] && ((mldm >> (16 + rw)) & 1u)) t4[i][3] = tp[3 * PAC_HALFN];
    }
    if (tid < 6 * 32) key[tid / 32][tid % 32] = 0ull;
    lds_sync();
    int oL, oR;
    if constexpr (FAST) {
        oL = F.overall[gb * 2];
        oR = F.overall[gb * 2 + 1];
    } else {
        double mL = 0.0, mR = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (!from_md) {
                xl4[i] = XL[i * 256 + tid];
                xr4[i] = st ? XR[i * 256 + tid] : 0.0;
            }
            mL = fmax(mL, fabs(xl4[i]));
            mR = fmax(mR, fabs(xr4[i]));
        }
        mL = wave_max(mL);                           // one LDS atomic per wave, not per thread
        mR = wave_max(mR);
        if ((tid & (WAVE - 1)) == 0) {
            atomicMax(&key[4][0], (unsigned long long)__double_as_longlong(mL));
            atomicMax(&key[5][0], (unsigned long long)__double_as_longlong(mR));
        }
        lds_sync();
        oL = pac_scale_factor(__longlong_as_double((long long)key[4][0]), 5);
        oR = pac_scale_factor(__longlong_as_double((long long)key[5][0]), 5);
        if (tid == 0) {
            F.overall[gb * ck.nch] = (uint8_t)oL;
            if (st) F.overall[gb * 2 + 1] = (uint8_t)oR;
        }
    }
    const double gL = (double)(1 << oL), gR = (double)(1 << oR);
    const double offL = 6.02 * oL, offR = 6.02 * oR;
    MPROF(2);

    // --- per-line SMR terms (psychoac.py:533-597), selection (:662-682) ----
    double* lines = K.lines + j * 2 * PAC_HALFN;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int l = i * 256 + tid;
        const int b = sp4[i] >> 20;
        const int ms = ms4[i];
        // the coded lines: M/S of the scaled channels, or the scaled L, R
        double v0, v1;
        if constexpr (FAST) {                     // formed by the side kernel (lrms_block<true>)
            v0 = xl4[i];
            v1 = xr4[i];
        } else {
            const double xl = __dmul_rn(xl4[i], gL), xr = __dmul_rn(xr4[i], gR);
            const double M = __dadd_rn(xl, xr) / 2.0, S = __dsub_rn(xl, xr) / 2.0;
            v0 = ms ? M : xl;
            v1 = ms ? S : xr;
        }
        // the SMR terms SPL(4 x^2) - THR as intensity ratios (pac_spl_ratio: the
        // thresholds are intensities, SPL is monotone, so the band maximum of
        // the ratios gives the band's SMR with one log10; the scale offsets
        // come off per band)
        double d0, d1;
        if (ms) {
            const double bM = t4[i][0], bS = t4[i][1];
            const double mldM = t4[i][2], mldS = t4[i][3];   // MLD_M, MLD_S
            const double a = bS < mldS ? bS : mldS;        // np.minimum(BTHR_S, MLD_S)
            const double thrM = bM > a ? bM : a;           // np.maximum(BTHR_M, .)
            const double c = bM < mldM ? bM : mldM;
            const double thrS = bS > c ? bS : c;
            d0 = pac_spl_ratio(4. * (v0 * v0), thrM);
            d1 = pac_spl_ratio(4. * (v1 * v1), thrS);
        } else {
            d0 = pac_spl_ratio(4. * (v0 * v0), t4[i][0]);
            d1 = st ? pac_spl_ratio(4. * (v1 * v1), t4[i][1]) : 0.0;
        }
        if constexpr (!FAST) {
            lines[l] = v0;
            lines[PAC_HALFN + l] = v1;
        }
        // band maxima: each DPP row of 16 lines holds whole band pieces; a
        // segmented max (row_shl DPP, no LDS crossbar) down to each piece's
        // first lane, then one LDS atomic per piece (same-address atomics
        // serialise: at most 4 per band and wave)
        const bool in = l < lend;
        const int lane = tid & (WAVE - 1);
        const int e = in ? min(lane | 15, lane + (((sp4[i] >> 10) & 1023) - l)) : lane;
        unsigned long long k0 = in ? (unsigned long long)__double_as_longlong(d0) : 0ull;   // positive: bits order
        unsigned long long k1 = in ? (unsigned long long)__double_as_longlong(d1) : 0ull;
        unsigned long long k2 = in ? (unsigned long long)__double_as_longlong(fabs(v0)) : 0ull;
        unsigned long long k3 = in ? (unsigned long long)__double_as_longlong(fabs(v1)) : 0ull;
        seg_max_step<1>(k0, k1, k2, k3, lane + 1 <= e);
        seg_max_step<2>(k0, k1, k2, k3, lane + 2 <= e);
        seg_max_step<4>(k0, k1, k2, k3, lane + 4 <= e);
        seg_max_step<8>(k0, k1, k2, k3, lane + 8 <= e);
        if (in && ((lane & 15) == 0 || l == (sp4[i] & 1023))) {
            atomicMax(&key[0][b], k0);
            atomicMax(&key[1][b], k1);
            atomicMax(&key[2][b], k2);
            atomicMax(&key[3][b], k3);
        }
    }
    lds_sync();
    MPROF(3);
    if (tid < PAC_NB) {
        const bool has = T->nlines[tid] != 0;
        // SMR = (SPL(4 x^2) - 6.02 scale) - THR = 10 log10(max ratio) - 6.02 scale
        // (mono: channel 1 unused, 0 as before)
        K.smr[(j * 2 + 0) * PAC_NB + tid] =
            has ? pac_ratio_db(__longlong_as_double((long long)key[0][tid])) - offL : -96.0;
        K.smr[(j * 2 + 1) * PAC_NB + tid] =
            has ? (st ? pac_ratio_db(__longlong_as_double((long long)key[1][tid])) - offR : 0.0) : -96.0;
        K.bandpeak[(j * 2 + 0) * PAC_NB + tid] = has ? __longlong_as_double((long long)key[2][tid]) : 0.0;
        K.bandpeak[(j * 2 + 1) * PAC_NB + tid] = has ? __longlong_as_double((long long)key[3][tid]) : 0.0;
    }
}

// --- the reservoir tail: one lane per stream ------------------------------
// The tail's work is a serial chain per stream (withdrawBits -> BitAlloc ->
// quantizer -> Huffman length scoring -> depositBits -> the next block), and
// it runs beside the next chunk's threshold kernel, whose VALU issue it
// shares: what it costs the pipeline is its VALU instruction count, not its
// latency.  So every lane runs one stream's chain in program order, as the
// reference's per-block calls do (no cross-lane reductions: 64 streams per
// wave instruction), with the per-band state in LDS columns (band-major,
// lane-minor: every lane's dynamically indexed access is conflict-free).

// Huffman length scoring table (built by pac_huffman_load): for a band of ba
// bits, symbol sym < 2^(ba-1), entry ((1 << (ba - 1)) - 2) + sym holds the
// ten tables' costs of coding it -- the code length, or the escape code's
// length + ba when the table lacks the symbol (Huffman.py:284-300) -- as
// 16-bit fields, table t at bits 16 (t & 1) of dword t / 2 (dword 5 unused).
// A channel-block's sums stay below 1024 * 46 < 2^16, so five 32-bit adds
// per line score all ten tables.
#define PAC_HSC_W 6
#define PAC_HSC_N 65534     // sum over ba = 2..16 of 2^(ba-1)

// BitAlloc (bitalloc.py:129-184) of one channel-block in one lane: each round
// gives one bit to the first band with the largest SMR - 6 bits among the
// valid ones (np.argmax); the stop test takes max(SMR - (bits - 1) 6) over ALL
// bands -- the valid ones' maximum is the chosen band's (the map is monotone),
// the invalid ones' is the running max of their frozen values.  A band's
// value is SMR - 6 bits (one rounding, as the reference's expression), -inf
// once the band is invalid (bit 7 of its bits byte).  Returns the bits left
// minus extra; bits[b][lane] = the allocation.
//
// The argmax is a two-level tournament: the 25 bands in five groups of five
// consecutive bands, gmax[g] / gidx[g] = the group's first maximum.  A round
// takes the first maximum of the five group maxima (groups in band order, so
// the first group holding the maximum, whose first maximum is the global first
// maximum: np.argmax's tie rule) and, after updating the chosen band,
// re-evaluates only that band's group: 10 + 10 LDS reads and 8 compare-selects
// per round instead of 50 reads and a 25-deep compare chain.  The band values
// are recomputed from (bits, SMR) rather than kept: the tail's LDS must stay
// within what a CU has left beside four threshold workgroups.
#define PAC_TT_G 5
#define PAC_BA_OFF 0x80       // bits byte: the band is no longer valid
__device__ __forceinline__ double tt_value(double sv, int nb) {
    return (nb & PAC_BA_OFF) ? -INFINITY : __builtin_fma(-6.0, (double)nb, sv);
}
__device__ __forceinline__ void tt_group(const double (*smr)[WAVE], const uint8_t (*bits)[WAVE], double (*gmax)[WAVE],
                                         uint8_t (*gidx)[WAVE], int g, int lane) {
    const int b0 = PAC_TT_G * g;
    double v[PAC_TT_G];
#pragma unroll
    for (int k = 0; k < PAC_TT_G; ++k) v[k] = tt_value(smr[b0 + k][lane], bits[b0 + k][lane]);
    double best = v[0];
    int bi = b0;
#pragma unroll
    for (int k = 1; k < PAC_TT_G; ++k) {
        const bool take = v[k] > best;               // strict: the first maximum
        best = take ? v[k] : best;
        bi = take ? b0 + k : bi;
    }
    gmax[g][lane] = best;
    gidx[g][lane] = (uint8_t)bi;
}

__device__ __forceinline__ long bitalloc_lane(double (*smr)[WAVE], uint8_t (*bits)[WAVE], double (*gmax)[WAVE],
                                              uint8_t (*gidx)[WAVE], const int* __restrict__ nl_s,
                                              const double* __restrict__ smr_g, uint32_t lrms_bits, double bitBudget,
                                              long extra, int maxMantBits, int lane) {
    static_assert(PAC_NB == PAC_TT_G * PAC_TT_G, "five groups of five bands");
#pragma unroll
    for (int g = 0; g < PAC_TT_G; ++g) {           // values SMR - 6 * 0 = SMR: the groups from the loads
        double v[PAC_TT_G];
#pragma unroll
        for (int k = 0; k < PAC_TT_G; ++k) {
            const int b = PAC_TT_G * g + k;
            v[k] = smr_g[b];
            smr[b][lane] = v[k];
            bits[b][lane] = 0;
        }
        double best = v[0];
        int bi = PAC_TT_G * g;
#pragma unroll
        for (int k = 1; k < PAC_TT_G; ++k) {
            const bool take = v[k] > best;
            best = take ? v[k] : best;
            bi = take ? PAC_TT_G * g + k : bi;
        }
        gmax[g][lane] = best;
        gidx[g][lane] = (uint8_t)bi;
    }
    long total = (long)(bitBudget + (double)extra);
    double frozen = -INFINITY;
    while (true) {
        double best = gmax[0][lane];
        int ib = gidx[0][lane];
#pragma unroll
        for (int g = 1; g < PAC_TT_G; ++g) {
            const double v = gmax[g][lane];
            const bool take = v > best;
            best = take ? v : best;
            ib = take ? (int)gidx[g][lane] : ib;
        }
        if (best == -INFINITY) break;                  // no valid band left
        const int n = bits[ib][lane], nl = nl_s[ib];   // valid: no PAC_BA_OFF flag
        const double sv = smr[ib][lane];
        const double gall = fmax(__builtin_fma(-6.0, (double)(n - 1), sv), frozen);
        bool drop = gall < (((lrms_bits >> ib) & 1u) ? -5.0 : -15.0);
        int nn = n;
        if (total - nl >= 0) {
            nn = n + 1;
            total -= nl;
            drop |= nn >= maxMantBits;
        } else {
            drop = true;
        }
        bits[ib][lane] = (uint8_t)(nn | (drop ? PAC_BA_OFF : 0));
        if (drop) frozen = fmax(frozen, __builtin_fma(-6.0, (double)(nn - 1), sv));
        tt_group(smr, bits, gmax, gidx, (ib * 13) >> 6, lane);    // ib / 5 for ib < 25
    }
    int back = 0;                                      // bits[bits == 1] = 0, their lines back
#pragma unroll
    for (int b = 0; b < PAC_NB; ++b) {
        int n = bits[b][lane] & ~PAC_BA_OFF;
        if (n == 1) {
            back += nl_s[b];
            n = 0;
        }
        bits[b][lane] = (uint8_t)n;
    }
    return total + back - extra;
}

#ifndef PAC_TAIL_U
#define PAC_TAIL_U 8      // lines per lane whose loads are in flight together
#endif
#define PAC_BUF_OOB ((int)0xF0000000)    // a raw-buffer offset past any 2 GB range: the load returns 0
// the tail addresses a chunk's coded lines through one raw buffer with 32-bit
// byte offsets up to 2 * chunk_blocks * PAC_HALFN * 8: run_master refuses
// chunks of more than PAC_CHUNK_MAX blocks, so no offset wraps
// into the out-of-range value that would silently read zeros
static_assert(2LL * PAC_CHUNK_MAX * PAC_HALFN * 8 < 0x7fffffffLL, "tail line offsets exceed the buffer range");
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// exclusive prefix of an int across the wave by DPP; *total = the wave's sum
__device__ __forceinline__ int wave_excl_scan_i(int v, int* total) {
    int x = v;
    x += __builtin_amdgcn_update_dpp(0, x, PAC_DPP_SHR(1), 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, PAC_DPP_SHR(2), 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, PAC_DPP_SHR(4), 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, PAC_DPP_SHR(8), 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, PAC_DPP_BCAST15, 0xa, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, PAC_DPP_BCAST31, 0xc, 0xf, false);
    *total = __builtin_amdgcn_readlane(x, 63);
    return x - v;
}

// MSB-first bit writer of one lane (big-endian words: the bytes in file
// order) whose words leave in bursts of PAC_EMIT_WORDS: the finished words of
// a burst wait in registers (b[], oldest first) and go out with its last one
// as 16-byte stores.  One lane per channel-block writes 64 different lines per
// store instruction, and a line the L2 evicts half-written costs a partial
// write: a 4-byte store per word wrote 4.56 KB per block (592 B of
// bitstream), bursts of 4 words 1.89 KB, of 8 words 0.97 KB (PMC WRITE_SIZE,
// configs[2]); emission VALU 530 -> 745 -> 863 per block, and the threshold
// kernel beside it 799 -> 787 ms per 10^7 blocks (fewer store instructions).
// The region starts 16-byte aligned and is padded to a whole burst
// (k_master_emit, k_master_place).
#ifndef PAC_EMIT_WORDS
#define PAC_EMIT_WORDS 8  // words per lane store burst (a multiple of 4)
#endif
struct LaneBits16 {
    static constexpr int NW = PAC_EMIT_WORDS;
    static_assert(NW % 4 == 0, "bursts of whole 16-byte stores");
    uint4* w;
    uint64_t acc;
    int n, nw;
    uint32_t b[NW - 1];
    __device__ __forceinline__ void word(uint32_t x) {
        if (nw == NW - 1) {
#pragma unroll
            for (int k = 0; k + 4 <= NW - 1; k += 4) w[k / 4] = make_uint4(b[k], b[k + 1], b[k + 2], b[k + 3]);
            w[NW / 4 - 1] = make_uint4(b[NW - 4], b[NW - 3], b[NW - 2], x);
            w += NW / 4;
            nw = 0;
        } else {
#pragma unroll
            for (int k = 0; k < NW - 2; ++k) b[k] = b[k + 1];
            b[NW - 2] = x;
            ++nw;
        }
    }
    __device__ __forceinline__ void put(uint32_t v, int bits) {    // bits <= 32, v < 2^bits
        acc = (acc << bits) | v;
        n += bits;
        if (n >= 32) {
            n -= 32;
            word(__builtin_bswap32((uint32_t)(acc >> n)));
        }
    }
    __device__ __forceinline__ void flush() {
        if (n > 0) word(__builtin_bswap32((uint32_t)(acc << (32 - n))));
        // the last nw words (b[NW-1-nw] ..), then padding: zeros shifted in
        // until the burst completes
        while (nw > 0) word(0u);
    }
};

// LDS: launched with PAC_TAIL_LDS bytes of dynamic shared memory -- declared
// statically, the compiler's occupancy estimate would become LDS-bound and it
// would then ignore the 5-waves-per-SIMD register budget (96 VGPRs) that lets
// a tail wave sit beside 4 threshold waves (104 VGPRs each) on a SIMD.
// layout: smr[25][64] double | gmax[5][64] double (after BitAlloc: sf[25][64]
// u8) | bits[25][64] u8 | gidx[5][64] u8 | nl[25] int | the line quarters'
// Huffman sums acc[4][5][64] u32 -- 22.5 KB.  Measured: 28.9 KB still let a
// tail workgroup sit beside four threshold workgroups on a CU, 31.8 KB did not
// (the thresholds +72 ms per 10^7 blocks).
#define PAC_TAIL_LDS_GMAX (PAC_NB * WAVE * 8)
#define PAC_TAIL_LDS_BITS (PAC_TAIL_LDS_GMAX + PAC_TT_G * WAVE * 8)
#define PAC_TAIL_LDS_GIDX (PAC_TAIL_LDS_BITS + PAC_NB * WAVE)
#define PAC_TAIL_LDS_NL (PAC_TAIL_LDS_GIDX + PAC_TT_G * WAVE)
#define PAC_TAIL_LDS_ACC (PAC_TAIL_LDS_NL + PAC_NB * 4)
#define PAC_TAIL_Q 4           // waves per tail workgroup: line quarters of a channel-block
#define PAC_TAIL_LDS (PAC_TAIL_LDS_ACC + PAC_TAIL_Q * 5 * WAVE * 4)
static_assert(PAC_TT_G * WAVE * 8 >= PAC_NB * WAVE, "sf aliases gmax");
static_assert(PAC_TAIL_LDS <= 28900, "tail LDS beside k_master_thr");
static_assert(PAC_TAIL_LDS_ACC % 4 == 0, "acc alignment");

// 64 streams of the chunk per workgroup of four waves, lane l of every wave
// serving stream blockIdx * 64 + l: for the stream's blocks t0 .. t0+S-1 in
// order -- withdrawBits (Huffman.py:363-371, codec.py:229), per channel
// BitAlloc with the extraBits carry (codec.py:249-260) and the scale factors
// (quantize.py:148-177) in wave 0, one lane per stream (the reservoir chain,
// no cross-lane work: the fewest VALU instructions); then vMantissa
// (quantize.py:315-342), StripSignBits + Huffman.encodeData's ten table
// lengths (Huffman.py:274-309) over the channel-block's lines, a quarter of
// them per wave; then in wave 0 the table choice, depositBits
// (codec.py:111-124) and each channel-block's byte count.  The line quarters
// cut the chain's longest part -- dependent memory round trips, two per eight
// lines -- by four with the same instructions (measured alone: 555 ms per
// 10^7 blocks, 366 of them in the lines).  The signed mantissa codes go to the
// chunk's K.codes for k_master_emit, or to F.codes for k_master_pack.
__global__ __launch_bounds__(PAC_TAIL_Q * WAVE) __attribute__((amdgpu_waves_per_eu(5))) void k_master_tail(
    const PacTables* __restrict__ T, const uint32_t* __restrict__ hsc, PacMasterChunkBuf K, PacMasterFields F,
    const int64_t* __restrict__ blk_off, PacMasterChunk ck, int64_t* __restrict__ st_extra,
    int64_t* __restrict__ st_deposit, double bitBudget) {
    extern __shared__ __attribute__((aligned(16))) char tail_lds[];
    double (*smr_s)[WAVE] = reinterpret_cast<double (*)[WAVE]>(tail_lds);
    double (*gmax_s)[WAVE] = reinterpret_cast<double (*)[WAVE]>(tail_lds + PAC_TAIL_LDS_GMAX);
    uint8_t (*sf_s)[WAVE] = reinterpret_cast<uint8_t (*)[WAVE]>(tail_lds + PAC_TAIL_LDS_GMAX);   // after BitAlloc
    uint8_t (*bits_s)[WAVE] = reinterpret_cast<uint8_t (*)[WAVE]>(tail_lds + PAC_TAIL_LDS_BITS);
    uint8_t (*gidx_s)[WAVE] = reinterpret_cast<uint8_t (*)[WAVE]>(tail_lds + PAC_TAIL_LDS_GIDX);
    int* nl_s = reinterpret_cast<int*>(tail_lds + PAC_TAIL_LDS_NL);
    uint32_t (*acc_s)[5][WAVE] = reinterpret_cast<uint32_t (*)[5][WAVE]>(tail_lds + PAC_TAIL_LDS_ACC);
    const int lane = threadIdx.x & (WAVE - 1);
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
    __builtin_amdgcn_s_setprio(3);    // beside k_master_thr's waves (see thr_variant)
    if (threadIdx.x < PAC_NB) nl_s[threadIdx.x] = T->nlines[threadIdx.x];
    lds_sync();
    const int sl = blockIdx.x * WAVE + lane;
    const bool live = sl < ck.n_s;                     // every lane stays for the wave-wide steps
    const int nch = ck.nch;
    const int s = ck.perm[ck.s_first + (live ? sl : 0)];
    const int64_t bb0 = blk_off[s];
    const int64_t len = blk_off[s + 1] - bb0;
    const int64_t t_end = !live ? ck.t0 : (ck.t0 + ck.S < len ? ck.t0 + ck.S : len);
    long extra = 0, deposit = 0;                        // the reservoir state: wave 0's lanes
    if (w == 0 && live) {
        extra = st_extra[s];
        deposit = st_deposit[s];
    }
    const int lend = T->lower[PAC_NB - 1] + T->nlines[PAC_NB - 1];
    const int q0 = w * (PAC_HALFN / PAC_TAIL_Q);       // this wave's quarter of the lines
    const int q1 = min(q0 + PAC_HALFN / PAC_TAIL_Q, lend);
    // the chunk's coded lines and the Huffman scoring table as raw buffers (2 GB
    // ranges: PAC_BUF_OOB offsets read 0 without a memory access)
    const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc((void*)K.lines, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc((void*)hsc, 0, 0x7fffffff, 0x00020000);
    for (int64_t t = ck.t0; t < ck.t0 + ck.S; ++t) {   // uniform trip count: every barrier is reached
        const bool act = t < t_end;
        const int64_t j = (int64_t)sl * ck.S + (t - ck.t0);
        const int64_t gb = bb0 + t;
        uint32_t lrms_bits = 0;
        long dep_add = 0;
        if (w == 0 && act) {
            // Huffman.withdrawBits (Huffman.py:363-371), codec.py:229
            long e = 0;
            if (deposit > 10) { e = deposit / 100; deposit -= e; }
            else if (deposit < 0) { e = deposit; deposit = 0; }
            extra += e;
            lrms_bits = nch == 2 ? F.msm[gb] : 0u;      // the LRMS flags as one band mask (k_master_lrms)
        }
        for (int ch = 0; ch < nch; ++ch) {
            const int64_t gl = j * 2 + ch, g = gb * nch + ch;
            uint16_t* cs = F.codes ? F.codes + g * PAC_HALFN : K.codes + gl * PAC_HALFN;
            int orig = 0, nsign = 0;
            if (w == 0 && act) {
                extra += bitalloc_lane(smr_s, bits_s, gmax_s, gidx_s, nl_s, K.smr + gl * PAC_NB, lrms_bits,
                                       bitBudget, extra, 16, lane);
                // scale factors; the allocation's mantissa and sign bits.  Five
                // band peaks in flight at a time (25 would not fit the 96
                // VGPRs; one at a time was 25 dependent memory round trips)
#pragma unroll 1
                for (int b0 = 0; b0 < PAC_NB; b0 += 5) {
                    double pk[5];
#pragma unroll
                    for (int k = 0; k < 5; ++k) pk[k] = K.bandpeak[gl * PAC_NB + b0 + k];
#pragma unroll
                    for (int k = 0; k < 5; ++k) {
                        const int b = b0 + k;
                        const int ba = bits_s[b][lane];
                        const int f = pac_scale_factor(pk[k], ba);
                        sf_s[b][lane] = (uint8_t)f;
                        F.ba[g * PAC_NB + b] = (uint8_t)ba;
                        F.sf[g * PAC_NB + b] = (uint8_t)f;
                        orig += ba * nl_s[b];
                        nsign += ba ? nl_s[b] : 0;
                    }
                }
            }
            lds_sync();                                // bits and scale factors for every wave
            uint32_t acc[5] = {0u, 0u, 0u, 0u, 0u};
            if (act) {
                // mantissas (stored for the emission / the pack) and the ten
                // tables' total lengths of this wave's quarter, PAC_TAIL_U lines
                // at a time, branch-free: the group's bands from one scalar
                // load, its lanes' bits and scale factors from LDS, then the
                // lines and the scoring-table entries by raw buffer loads whose
                // offset is out of range for a line without bits -- the load
                // returns 0 and touches no memory -- instead of a predicated
                // branch per line
                const int64_t lane_off = (int64_t)gl * PAC_HALFN * 8;   // < 2^31: the chunk's line set
                for (int l0 = q0; l0 < q1; l0 += PAC_TAIL_U) {
                    int bo[PAC_TAIL_U];
#pragma unroll
                    for (int u = 0; u < PAC_TAIL_U; ++u) bo[u] = T->band_of_line[l0 + u];   // uniform, one s_load
                    int bal[PAC_TAIL_U], sfl[PAC_TAIL_U];
#pragma unroll
                    for (int u = 0; u < PAC_TAIL_U; ++u) {
                        bal[u] = l0 + u < lend ? bits_s[bo[u]][lane] : 0;
                        sfl[u] = sf_s[bo[u]][lane];
                    }
                    double x[PAC_TAIL_U];
#pragma unroll
                    for (int u = 0; u < PAC_TAIL_U; ++u)
                        x[u] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                            lrs, bal[u] ? (int)(lane_off + (l0 + u) * 8) : PAC_BUF_OOB, 0, 0));
                    uint32_t m[PAC_TAIL_U];
                    int eo[PAC_TAIL_U];
#pragma unroll
                    for (int u = 0; u < PAC_TAIL_U; ++u) {
                        const int ba = bal[u];
                        m[u] = ba ? pac_mantissa(x[u], sfl[u], ba) : 0u;
                        // < 2^19 entries of 24 B: a 32-bit offset
                        eo[u] = ba ? ((((1 << (ba - 1)) - 2) + (int)(m[u] & ((1u << (ba - 1)) - 1u))) * PAC_HSC_W) * 4
                                   : PAC_BUF_OOB;
                    }
#pragma unroll
                    for (int u = 0; u < PAC_TAIL_U; ++u) {
                        const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(hrs, eo[u], 0, 0);
                        const uint32_t c4 = __builtin_amdgcn_raw_buffer_load_b32(hrs, eo[u] + 16, 0, 0);
                        acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w; acc[4] += c4;
                    }
#pragma unroll
                    for (int u = 0; u < PAC_TAIL_U; u += 4) {      // four codes per 8-byte store
                        const uint64_t wd = (uint64_t)m[u] | ((uint64_t)m[u + 1] << 16) | ((uint64_t)m[u + 2] << 32) |
                                            ((uint64_t)m[u + 3] << 48);
                        *reinterpret_cast<uint64_t*>(cs + l0 + u) = wd;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < 5; ++k) acc_s[w][k][lane] = acc[k];
            lds_sync();                                // the quarters' sums; bits / sf read by every wave
            if (w == 0 && act) {
                int best = 0, bestid = 1;
                uint32_t tot[5];
#pragma unroll
                for (int k = 0; k < 5; ++k)            // 16-bit fields, no carry across: sums < 2^16
                    tot[k] = (acc_s[0][k][lane] + acc_s[1][k][lane]) + (acc_s[2][k][lane] + acc_s[3][k][lane]);
#pragma unroll
                for (int tb = 0; tb < PAC_NTAB; ++tb) {
                    const int v = (int)((tot[tb >> 1] >> (16 * (tb & 1))) & 0xffffu);
                    if (tb == 0 || v < best) { best = v; bestid = tb + 1; }
                }
                dep_add += (long)orig - ((long)best + nsign + 4);
                F.tid[g] = (uint8_t)bestid;
                F.nbytes[g] = 4 + (8 + 8 * PAC_NB + nsign + best + PAC_NB + (F.bsf ? 1 : 0) + 7) / 8;
            }
        }
        if (w == 0 && act) deposit += dep_add;   // depositBits per channel (codec.py:120)
    }
    if (w == 0 && live) {
        st_extra[s] = extra;
        st_deposit[s] = deposit;
    }
}

// --- the reservoir tail for few streams: one wave per stream --------------
// The one-lane tail spends ~0.7 ms per block of a stream (its chain is a
// string of dependent memory round trips), so a call with few streams --
// S = 32768 / streams blocks per stream and chunk -- is bound by it.  For a
// chunk of at most PAC_WIDE_MAX streams this kernel runs the same chain with
// a whole wave per stream: the 25 bands in lanes 0-24 (BitAlloc's argmax as a
// DPP + permlane reduction), 16 lines per lane for the mantissas and the
// Huffman scoring (coalesced).  ~10x the VALU instructions per block, ~1/10
// of the latency; the same arithmetic, so the same bytes.
#ifndef PAC_WIDE_MAX
#define PAC_WIDE_MAX 4096
#endif

// the first maximum of (v, b) over lanes 0-31 (larger v, then lower b),
// wave-uniform (read from lane 0)
template <int CTRL>
__device__ __forceinline__ void argmax_dpp(double& v, int& b) {
    const double ov = dpp_full_f64<CTRL>(v);
    const int ob = __builtin_amdgcn_mov_dpp(b, CTRL, 0xf, 0xf, true);
    const bool take = ov > v || (ov == v && ob < b);
    v = take ? ov : v;
    b = take ? ob : b;
}
__device__ __forceinline__ void argmax32(double& v, int& b) {
    argmax_dpp<PAC_DPP_QXOR1>(v, b);
    argmax_dpp<PAC_DPP_QXOR2>(v, b);
    argmax_dpp<PAC_DPP_HMIRROR>(v, b);
    argmax_dpp<PAC_DPP_MIRROR>(v, b);                  // row maxima
    const long long iv = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)iv, (unsigned)iv, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(iv >> 32), (unsigned)(iv >> 32), false, false);
    const auto bb = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
    // lanes of row 0 get row 1's maximum in [1] (and row 1 row 0's in [0])
    const double v0 = __longlong_as_double(((long long)hi[0] << 32) | (long long)lo[0]);
    const double v1 = __longlong_as_double(((long long)hi[1] << 32) | (long long)lo[1]);
    const int b0 = (int)bb[0], b1 = (int)bb[1];
    const bool take = v1 > v0 || (v1 == v0 && b1 < b0);
    v = take ? v1 : v0;
    b = take ? b1 : b0;
    v = readlane_f64(v, 0);
    b = __builtin_amdgcn_readlane(b, 0);
}

// BitAlloc of one channel-block by a wave (lane b < 25 = band b), the
// reference's rounds as bitalloc_lane.  *ba = the lane's band allocation.
__device__ __forceinline__ long bitalloc_wave(const int nl, const double sm, uint32_t lrms_bits, double bitBudget,
                                              long extra, int maxMantBits, int lane, int* ba) {
    const bool has = lane < PAC_NB;
    int n = 0;
    bool valid = has;
    long total = (long)(bitBudget + (double)extra);
    double frozen = -INFINITY;
    while (true) {
        double v = valid ? __builtin_fma(-6.0, (double)n, sm) : -INFINITY;
        int b = lane;
        argmax32(v, b);
        if (v == -INFINITY) break;                     // no valid band left (uniform)
        const int ib = b;
        const int nb_ = __builtin_amdgcn_readlane(n, ib), nli = __builtin_amdgcn_readlane(nl, ib);
        const double sv = readlane_f64(sm, ib);
        const double gall = fmax(__builtin_fma(-6.0, (double)(nb_ - 1), sv), frozen);
        bool drop = gall < (((lrms_bits >> ib) & 1u) ? -5.0 : -15.0);
        int nn = nb_;
        if (total - nli >= 0) {
            nn = nb_ + 1;
            total -= nli;
            drop |= nn >= maxMantBits;
        } else {
            drop = true;
        }
        if (lane == ib) {
            n = nn;
            valid = !drop;
        }
        if (drop) frozen = fmax(frozen, __builtin_fma(-6.0, (double)(nn - 1), sv));
    }
    int back = 0;                                      // bits[bits == 1] = 0, their lines back
    if (has && n == 1) { back = nl; n = 0; }
    *ba = n;
    return total + wave_sum_i(back) - extra;
}

__global__ __launch_bounds__(64) void k_master_tail_wide(
    const PacTables* __restrict__ T, const uint32_t* __restrict__ hsc, PacMasterChunkBuf K, PacMasterFields F,
    const int64_t* __restrict__ blk_off, PacMasterChunk ck, int64_t* __restrict__ st_extra,
    int64_t* __restrict__ st_deposit, double bitBudget) {
    __shared__ uint8_t ba_s[32], sf_s[32];
    const int lane = threadIdx.x;
    const int sl = blockIdx.x;
    const int nch = ck.nch;
    const int s = ck.perm[ck.s_first + sl];
    const int64_t bb0 = blk_off[s];
    const int64_t len = blk_off[s + 1] - bb0;
    const int64_t t_end = ck.t0 + ck.S < len ? ck.t0 + ck.S : len;
    long extra = st_extra[s], deposit = st_deposit[s];
    const int lend = T->lower[PAC_NB - 1] + T->nlines[PAC_NB - 1];
    const bool has = lane < PAC_NB;
    const int nl = has ? T->nlines[lane] : 0;
    for (int64_t t = ck.t0; t < t_end; ++t) {
        const int64_t j = (int64_t)sl * ck.S + (t - ck.t0);
        const int64_t gb = bb0 + t;
        // Huffman.withdrawBits (Huffman.py:363-371), codec.py:229
        long e = 0;
        if (deposit > 10) { e = deposit / 100; deposit -= e; }
        else if (deposit < 0) { e = deposit; deposit = 0; }
        extra += e;
        const uint32_t lrms_bits =
            (uint32_t)__ballot(has && F.lrms[gb * PAC_NB + (has ? lane : 0)] != 0) & ((1u << PAC_NB) - 1u);
        long dep_add = 0;
        for (int ch = 0; ch < nch; ++ch) {
            const int64_t gl = j * 2 + ch, g = gb * nch + ch;
            uint16_t* cs = F.codes ? F.codes + g * PAC_HALFN : K.codes + gl * PAC_HALFN;
            const double sm = has ? K.smr[gl * PAC_NB + lane] : 0.0;
            int ba;
            extra += bitalloc_wave(nl, sm, lrms_bits, bitBudget, extra, 16, lane, &ba);
            int f = 0;
            if (has) {
                f = pac_scale_factor(K.bandpeak[gl * PAC_NB + lane], ba);
                ba_s[lane] = (uint8_t)ba;
                sf_s[lane] = (uint8_t)f;
                F.ba[g * PAC_NB + lane] = (uint8_t)ba;
                F.sf[g * PAC_NB + lane] = (uint8_t)f;
            }
            const int orig = wave_sum_i(has ? ba * nl : 0);
            const int nsign = wave_sum_i(has && ba ? nl : 0);
            wave_sync();                               // ba_s / sf_s visible
            const double* ln = K.lines + gl * PAC_HALFN;
            uint32_t acc[5] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll 4
            for (int q = 0; q < PAC_HALFN / WAVE; ++q) {
                const int l = q * WAVE + lane;
                uint32_t m = 0u;
                if (l < lend) {
                    const int b = T->band_of_line[l];
                    const int bl = ba_s[b];
                    if (bl) {
                        m = pac_mantissa(ln[l], sf_s[b], bl);
                        const uint32_t* en = hsc + (int64_t)(((1 << (bl - 1)) - 2) + (m & ((1u << (bl - 1)) - 1u))) *
                                                       PAC_HSC_W;
                        const uint2 a = *reinterpret_cast<const uint2*>(en);
                        const uint2 b2 = *reinterpret_cast<const uint2*>(en + 2);
                        acc[0] += a.x; acc[1] += a.y; acc[2] += b2.x; acc[3] += b2.y; acc[4] += en[4];
                    }
                }
                cs[l] = (uint16_t)m;
            }
            int best = 0, bestid = 1;
#pragma unroll
            for (int w = 0; w < 5; ++w) {
                const uint32_t tot = (uint32_t)wave_sum_i((int)acc[w]);   // two 16-bit fields, no carry across
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int tb = 2 * w + h;
                    const int v = (int)((tot >> (16 * h)) & 0xffffu);
                    if (tb == 0 || v < best) { best = v; bestid = tb + 1; }
                }
            }
            dep_add += (long)orig - ((long)best + nsign + 4);
            if (lane == 0) {
                F.tid[g] = (uint8_t)bestid;
                F.nbytes[g] = 4 + (8 + 8 * PAC_NB + nsign + best + PAC_NB + (F.bsf ? 1 : 0) + 7) / 8;
            }
            wave_sync();                               // ba_s / sf_s rewritten by the next channel
        }
        deposit += dep_add;   // depositBits per channel (codec.py:120)
    }
    if (lane == 0) {
        st_extra[s] = extra;
        st_deposit[s] = deposit;
    }
}

#ifndef PAC_EMIT_U
#define PAC_EMIT_U 8      // lines per lane whose code + table loads are in flight together
#endif

// PACFile.WriteDataBlock's packing (pacfile.py:288-351) of the chunk's
// channel-blocks, one lane per channel-block, right after the chunk's tail
// (on its own stream, beside the next chunk's tail): '<L' nBytes, then
// overall(4) tableID(4), per band (ba?ba-1:0)(4) sf(4) [+ the band's sign
// bits + its Huffman codes (escape: escape code + ba raw bits)], LRMS(25)
// [+ the short-frame bit], MSB-first, into the staging buffer -- the wave's
// channel-blocks take consecutive pieces of one bump allocation; the offset
// goes to F.stoff for k_master_place.  No cross-channel-block dependency, so
// 64 per wave and many waves: the packing's latency stays off the reservoir
// chain.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) void k_master_emit(
    const PacTables* __restrict__ T, const PacHuffTables* __restrict__ H, const uint64_t* __restrict__ hcode,
    PacMasterChunkBuf K, PacMasterFields F, const int64_t* __restrict__ blk_off, PacMasterChunk ck) {
    const int lane = threadIdx.x;
    __builtin_amdgcn_s_setprio(3);    // beside k_master_thr's waves (see thr_variant)
    const int nch = ck.nch;
    const int64_t q = (int64_t)blockIdx.x * WAVE + lane;      // chunk-local channel-block: j nch + ch
    const int64_t j = q / nch;
    const int ch = (int)(q % nch);
    ChunkPos cp;
    const bool act = j < (int64_t)ck.n_s * ck.S && chunk_block(blk_off, ck, j, &cp);
    const int64_t gb = act ? cp.gb : 0;
    const int64_t g = gb * nch + ch, gl = j * 2 + ch;
    const int nb = act ? F.nbytes[g] : 0;
    const int sz = act ? (nb + 4 * PAC_EMIT_WORDS - 1) & -(4 * PAC_EMIT_WORDS) : 0;   // LaneBits16 bursts
    int tot;
    const int pre = wave_excl_scan_i(sz, &tot);
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(F.stg_next, (unsigned long long)tot);
    base = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(base >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)base);    // 64-bit broadcast
    const int64_t so = (int64_t)base + pre;
    if (!act) return;
    F.stoff[g] = so;
    if (so + sz > F.stg_cap) return;                         // over the staging capacity: the host re-runs
    const uint16_t* cs = K.codes + gl * PAC_HALFN;
    const uint8_t* bag = F.ba + g * PAC_NB;
    const uint8_t* sfg = F.sf + g * PAC_NB;
    const int tb = F.tid[g] - 1;
    uint32_t lrms_rev = 0;                                   // band 0 first
    for (int b = 0; b < PAC_NB; ++b) lrms_rev = (lrms_rev << 1) | (uint32_t)(F.lrms[gb * PAC_NB + b] & 1);
    LaneBits16 out{reinterpret_cast<uint4*>(F.stg + so), 0ull, 0, 0, {}};
    out.word((uint32_t)(nb - 4));                            // '<L' nBytes
    out.put(((uint32_t)F.overall[g] << 4) | (uint32_t)(tb + 1), 8);
    const uint32_t eb = H->esc_bits[tb];
    const int el = H->esc_len[tb];
    const uint64_t* hc = hcode + (int64_t)tb * PAC_NSYM;
    for (int b = 0; b < PAC_NB; ++b) {
        const int ba = bag[b];
        const int nl = T->nlines[b], lo = T->lower[b];     // uniform
        out.put(((uint32_t)(ba ? ba - 1 : 0) << 4) | sfg[b], 8);
        if (!ba) continue;
        uint32_t sb = 0;                                     // sign bits, 32 at a time
        int k = 0;
        for (int i0 = 0; i0 < nl; i0 += PAC_EMIT_U) {
            uint32_t m[PAC_EMIT_U];
#pragma unroll
            for (int u = 0; u < PAC_EMIT_U; ++u) m[u] = i0 + u < nl ? cs[lo + i0 + u] : 0u;
#pragma unroll
            for (int u = 0; u < PAC_EMIT_U; ++u) {
                if (i0 + u < nl) {
                    sb = (sb << 1) | ((m[u] >> (ba - 1)) & 1u);
                    if (++k == 32) { out.put(sb, 32); sb = 0; k = 0; }
                }
            }
        }
        if (k) out.put(sb, k);
        const uint32_t mask = (1u << (ba - 1)) - 1u;
        for (int i0 = 0; i0 < nl; i0 += PAC_EMIT_U) {
            uint32_t sym[PAC_EMIT_U];
            uint64_t e[PAC_EMIT_U];
#pragma unroll
            for (int u = 0; u < PAC_EMIT_U; ++u) sym[u] = i0 + u < nl ? (cs[lo + i0 + u] & mask) : 0u;
#pragma unroll
            for (int u = 0; u < PAC_EMIT_U; ++u) e[u] = hc[sym[u]];
#pragma unroll
            for (int u = 0; u < PAC_EMIT_U; ++u) {
                if (i0 + u < nl) {
                    const int L = (int)(e[u] >> 32);
                    if (L) {
                        out.put((uint32_t)e[u], L);
                    } else {
                        out.put(eb, el);
                        out.put(sym[u], ba);
                    }
                }
            }
        }
    }
    out.put(lrms_rev, PAC_NB);
    if (F.bsf) out.put((uint32_t)(F.bsf[gb] & PAC_BS_SHORT ? 1 : 0), 1);
    out.flush();
}

// Pass 2 with the tail's emission: every channel-block's bytes from the
// staging buffer to its file offset (one wave per channel-block, 64 bytes per
// step).  A channel-block that would end past cap is skipped; the host reports
// PAC_E_CAPACITY from the total.
__global__ __launch_bounds__(256) void k_master_place(PacMasterFields F, int64_t G, const int64_t* __restrict__ off,
                                                      uint8_t* __restrict__ out, int64_t cap) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t g = (int64_t)blockIdx.x * 4 + threadIdx.x / WAVE;
    if (g >= G) return;
    const int nb = F.nbytes[g];
    const int64_t og = off[g], so = F.stoff[g];
    // k_master_emit's padded size: a channel-block it skipped is skipped here too
    if (og + nb > cap || so + ((nb + 4 * PAC_EMIT_WORDS - 1) & -(4 * PAC_EMIT_WORDS)) > F.stg_cap) return;
    const uint8_t* src = F.stg + so;
    uint8_t* dst = out + og;
    for (int i = lane; i < nb; i += WAVE) dst[i] = src[i];
}

// worst-case master channel-block: 8 + 25 * 8 + 25 (+ 1 block-switching) bits
// + per line one sign bit and a code of at most max(code length, escape
// length + ba) <= 30 + 16 bits (pac_huffman_load rejects longer codes)
#define PAC_MASTER_MAX_BITS (8 + PAC_NB * 8 + PAC_NB + 1 + PAC_HALFN * (1 + 30 + 16))
#define PACK_WORDS_MASTER ((PAC_MASTER_MAX_BITS + 31) / 32)
static_assert(PACK_WORDS_MASTER * 4 <= 16384, "packed words must fit a 16 KB line buffer");


// Pass 2: one 256-thread workgroup per block gb (XCD-aware order):
// PACFile.WriteDataBlock's packing of its channel-blocks (pacfile.py:288-351)
// from the signed mantissa codes the tail stored (F.codes): overall(4)
// tableID(4), per band (ba?ba-1:0)(4) sf(4) [+ nLines sign bits + the Huffman
// codes], LRMS(25) [+ the block-switching bit], MSB-first.  Waves 2c and 2c+1
// pack channel c, rows 0-7 and 8-15 of its lines; the code-bit prefix crosses
// the halves through LDS.  A channel-block that would end past cap is
// skipped; the host reports PAC_E_CAPACITY from the total.  Latency bound:
// a chain of dependent memory round trips, so every load that depends only on
// the channel-block is issued before the first barrier (182 -> 108 ms per
// 10^7 blocks with 5 waves per SIMD; 6 waves alone gave 157, 6 with the early
// loads spills and is no faster).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 8))) void k_master_pack(const PacTables* __restrict__ T,
                                                     const PacHuffTables* __restrict__ H, PacMasterFields F,
                                                     int nch, int64_t nblocks, const int64_t* __restrict__ off,
                                                     uint8_t* __restrict__ out, int64_t cap) {
    __shared__ uint32_t words[2][PACK_WORDS_MASTER];   // the two channel-blocks' packed bits
    __shared__ int bas[2][PAC_NB], sfs[2][PAC_NB], bstart[2][PAC_NB + 1], pal[2][PAC_NB];
    __shared__ int half_bits[2], tot_bits[2];
    __shared__ uint8_t lr[PAC_NB];
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    const int w = tid / WAVE;
    const int c = w >> 1, h = w & 1;
    const int64_t gb = xcd_item(blockIdx.x, nblocks);
    const int fl = F.bsf ? F.bsf[gb] : 0;
    const bool act = c < nch;                  // mono: waves 2, 3 only zero the words and meet the barriers
    const int64_t g = gb * nch + (act ? c : 0);
    // every load that depends on nothing but g first (the kernel is a chain of
    // dependent memory round trips): table id, this wave's codes and band
    // indices, the byte count and offset of the store at the end
    const int tb = F.tid[g] - 1;
    const int nb = F.nbytes[g];
    const int64_t og = off[g];
    const uint16_t* cm = F.codes + g * PAC_HALFN;
    uint32_t mc[8];
    int bl[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int l = (8 * h + q) * WAVE + lane;
        bl[q] = T->band_of_line[l];
        mc[q] = cm[l];                         // 0 where ba == 0 (k_master_tail)
    }
    if (tid < PAC_NB) lr[tid] = F.lrms[gb * PAC_NB + tid];
    if (tid < nch * PAC_NB) {
        const int cc = tid / PAC_NB, b = tid % PAC_NB;
        bas[cc][b] = F.ba[(gb * nch + cc) * PAC_NB + b];
        sfs[cc][b] = F.sf[(gb * nch + cc) * PAC_NB + b];
    }
    for (int i = tid; i < PACK_WORDS_MASTER; i += 256) {
        words[0][i] = 0u;
        words[1][i] = 0u;
    }
    __syncthreads();
    // this wave's 8 rows: sign + code of length clen per line (0 for ba == 0 bands)
    uint32_t code[8], sgn[8];
    int clen[8], esc[8], pre[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int l = (8 * h + q) * WAVE + lane;
        const int b = bl[q];
        const int ba = bas[c][b];
        clen[q] = 0; esc[q] = 0; code[q] = 0; sgn[q] = 0;
        uint32_t m = 0;
        if (ba && act) {
            m = mc[q];
            const uint32_t sym = m & ((1u << (ba - 1)) - 1u);
            sgn[q] = (m >> (ba - 1)) & 1u;
            const int L = H->len[tb][sym];
            if (L) { clen[q] = L; code[q] = H->bits[tb][sym]; }
            else { clen[q] = H->esc_len[tb] + ba; esc[q] = 1; code[q] = sym; }
        }
        if (F.dbg_code && act) {
            const int64_t i = g * PAC_HALFN + l;
            F.dbg_mant[i] = m;
            F.dbg_code[i] = esc[q] ? (((uint64_t)H->esc_bits[tb] << ba) | code[q]) : (uint64_t)code[q];
            F.dbg_len[i] = (uint8_t)clen[q];
        }
    }
    // exclusive prefix of the code lengths in line order
    int run = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        int t;
        pre[q] = run + wave_excl_scan_i(clen[q], &t);
        run += t;
    }
    if (act && h == 0 && lane == 0) half_bits[c] = run;
    __syncthreads();
    uint32_t* wd = words[c];
    if (!act) {
    } else if (h) {
        const int hoff = half_bits[c];
#pragma unroll
        for (int q = 0; q < 8; ++q) pre[q] += hoff;
        if (lane == 0) tot_bits[c] = hoff + run;
    } else if (lane == 0) {           // band starts without code bits: 8 + sum_{b'<b} (8 + [ba>0] nl)
        int p = 8;
        for (int b = 0; b < PAC_NB; ++b) { bstart[c][b] = p; p += 8; if (bas[c][b]) p += T->nlines[b]; }
        bstart[c][PAC_NB] = p;
    }
    // code bits of all earlier bands = the prefix at the band's first line
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int l = (8 * h + q) * WAVE + lane;
        const int b = bl[q];
        if (act && l == T->lower[b] && T->nlines[b]) pal[c][b] = pre[q];
    }
    __syncthreads();
    if (!act) {
    } else if (h == 0) {
        if (lane == 0) {
            put_bits(wd, 0, (uint32_t)F.overall[g], 4);
            put_bits(wd, 4, (uint32_t)(tb + 1), 4);
        }
        if (lane < PAC_NB) {
            const int b = lane, ba = bas[c][b];
            int pa;
            if (T->nlines[b]) {
                pa = pal[c][b];
            } else {                  // empty band: the prefix of the next non-empty one
                int bb = b + 1;
                while (bb < PAC_NB && !T->nlines[bb]) bb++;
                pa = bb < PAC_NB ? pal[c][bb] : tot_bits[c];
            }
            const int p = bstart[c][b] + pa;
            put_bits(wd, p, (uint32_t)(ba ? ba - 1 : 0), 4);
            put_bits(wd, p + 4, (uint32_t)sfs[c][b], 4);
        }
    } else if (lane < PAC_NB) {
        put_bits(wd, bstart[c][PAC_NB] + tot_bits[c] + lane, (uint32_t)lr[lane], 1);
    } else if (lane == PAC_NB && F.bsf) {     // block switching: the short-frame bit
        put_bits(wd, bstart[c][PAC_NB] + tot_bits[c] + PAC_NB, (uint32_t)(fl & PAC_BS_SHORT), 1);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int l = (8 * h + q) * WAVE + lane;
        const int b = bl[q];
        const int ba = act ? bas[c][b] : 0;
        if (!ba) continue;
        const int p0 = bstart[c][b] + pal[c][b] + 8;
        put_bits(wd, p0 + (l - T->lower[b]), sgn[q], 1);
        const int pc = p0 + T->nlines[b] + (pre[q] - pal[c][b]);
        if (esc[q]) {
            const int el = H->esc_len[tb];
            put_bits(wd, pc, H->esc_bits[tb], el);
            put_bits(wd, pc + el, code[q], ba);
        } else {
            put_bits(wd, pc, code[q], clen[q]);
        }
    }
    __syncthreads();
    if (!act || og + nb > cap) return;
    uint8_t* o = out + og;
    if (h == 0 && lane < 4) o[lane] = (uint8_t)((uint32_t)(nb - 4) >> (8 * lane));   // '<L' nBytes
    for (int i = h * WAVE + lane; i < nb - 4; i += 2 * WAVE) o[4 + i] = be_byte(wd, i);
}
