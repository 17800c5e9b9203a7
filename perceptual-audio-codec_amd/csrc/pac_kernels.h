// pac_kernels.h -- internal kernel interface (device structs + kernel decls).
#pragma once
#include "pac_common.h"

// Where the channel-blocks' samples come from.
struct PacSource {
    const int16_t* pcm;        // interleaved int16 frames of all streams (device)
    const int64_t* frame_off;  // [n_streams+1] frame prefix (device)
    const int64_t* blk_off;    // [n_streams+1] block prefix incl. flush block (device)
    const double* fsrc;        // OR float64 blocks [n_blocks][n_ch][2048] (device), per-block API
    int n_streams;
    int n_ch;
    int dbg;                   // diagnostic phase switches (PAC_DEBUG_FLAGS), 0 in production
    long long* prof;           // diagnostic per-wave phase clocks (PAC_DEBUG_FLAGS & 16), else null
    const int32_t* lead;       // [n_streams] frames before the first hop (1024: the stream carries its
                               // priorBlock, PAC_STREAM_HAS_PRIOR), or null (all 0)
};

#define PAC_PROF_WG 4096       // workgroups sampled by the phase clocks
#define PAC_PROF_MARKS 16   // 0..8 phase marks, 10..13 end of each masking row

// Per-channel-block work arrays, index [g * 25 + band]: a workgroup writes
// its channel-block's bands as one contiguous run.
struct PacOriginWork {
    double* smr;        // [G][25]
    double* bandpeak;   // [G][25] max |scaled line| per band
    uint8_t* overall;   // [G]
    uint8_t* ba;        // [G][25]
    uint8_t* sf;        // [G][25]
    int32_t* nbytes;    // [G] 4 + payload bytes
};

#define SCAN_TILE 2048
