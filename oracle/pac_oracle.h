/* pac_oracle.h -- CPU restatement of the reference encoder (TEST INFRASTRUCTURE
 * ONLY; see pac_oracle.c).  Loaded by tests/ and bench.py's cpu_baseline leg. */
#ifndef PAC_ORACLE_H
#define PAC_ORACLE_H
#include <stdint.h>

#define PAC_ORACLE_ORIGIN 0
#define PAC_ORACLE_MASTER 1
#define PAC_NTABLES 10
#define PAC_NSYM 32768
/* block-switching extension (not in the reference; parity unpinned) */
#define PAC_BS_SHORT 1      /* four N = 512 blocks, interleaved        */
#define PAC_BS_PREV 2       /* long frame after a short one (stop)     */
#define PAC_BS_NEXT 4       /* long frame before a short one (start)   */
#define PAC_BS_RATIO 10.0
#define PAC_BS_EMIN 1e-3

typedef struct pac_oracle pac_oracle;

typedef struct {            /* one channel-block, origin profile */
    double mdct[1024];      /* MDCT output before the overall scale */
    int overall;
    int npeaks;
    double thr[1024];       /* getMaskedThreshold() */
    double smr[25];
    int ba[25];
    int sf[25];
    int32_t mant[1024];     /* by MDCT line; 0 where ba == 0 */
    int nbits;
} pac_oracle_chblock;

typedef struct {            /* master reservoir state (codec.py:229,260; Huffman.py:262) */
    long extraBits;
    long deposit;
} pac_oracle_state;

typedef struct {            /* one stereo block, master profile */
    int lrms[25];
    double mdct[2][1024];   /* before overall scale */
    int overall[2];
    int npeaks[6];
    double bthr[6][1024];   /* calcBTHR: L, R, M, S, M_MLD, S_MLD */
    double smr[2][25];
    double lines[2][1024];  /* LRMSmdctLines */
    long extra_in, extra_out, deposit_out;
    int ba[2][25];
    int sf[2][25];
    int32_t mant[2][1024];
    int table_id[2];
    long huff_bits[2];
    int nbits[2];
} pac_oracle_stblock;

#ifdef __cplusplus
extern "C" {
#endif
pac_oracle *pac_oracle_create(int sample_rate);
/* MDCT window: 0 SineWindow (the reference coders), 1 KBDWindow alpha 4 (extension) */
void pac_oracle_set_window(pac_oracle *o, int kind);
/* block switching on/off (master profile only; extension, parity unpinned) */
void pac_oracle_set_block_switch(pac_oracle *o, int on);
/* per-block flags PAC_BS_* the block-switching encoder uses for a stream
 * (nblocks = hops + 1 flush entries); returns nblocks */
void pac_oracle_bs_roundtrip(const pac_oracle *o, const double *x, int64_t n_frames, const uint8_t *fl,
                             double *out);
int64_t pac_oracle_bs_plan(const pac_oracle *o, const int16_t *pcm, int64_t n_frames, int n_ch,
                           uint8_t *flags, int64_t cap);
double pac_oracle_window(const pac_oracle *o, int n);
void pac_oracle_destroy(pac_oracle *t);
int pac_oracle_nlines(const pac_oracle *t, int *out25);
int pac_oracle_load_huffman(pac_oracle *t, const uint8_t *buf, int64_t len);
double pac_oracle_pcm_to_float(int16_t c);
void pac_oracle_mdct(const pac_oracle *t, const double *x, double *X);
int pac_oracle_threshold(const pac_oracle *t, double *data, int noDrop, double *thr,
                         int *peaks_out);
void pac_oracle_block_origin(const pac_oracle *t, double *x, pac_oracle_chblock *o);
void pac_oracle_block_master(const pac_oracle *t, double *xL, double *xR,
                             pac_oracle_state *st, pac_oracle_stblock *o);
int64_t pac_oracle_encode(const pac_oracle *t, int profile, const int16_t *pcm,
                          int64_t n_frames, int n_ch, int64_t max_blocks,
                          uint8_t *out, int64_t cap, pac_oracle_state *state);
void pac_oracle_imdct_window(const pac_oracle *t, const double *X, double *y);
int16_t pac_oracle_float_to_pcm(double x);
int64_t pac_oracle_decode(const pac_oracle *t, int profile, const uint8_t *data, int64_t nbytes, int n_ch,
                          int16_t *pcm, double *fout, int64_t max_frames);
#ifdef __cplusplus
}
#endif
#endif
