// pac_wav.hip -- WAV ingest and egress on the device:
// PCMFile.ReadFileHeader's chunk scan (codec/pcmfile.py:32-65), the
// ReadDataBlock hop reads with their zero padding (pcmfile.py:66-100) incl.
// the extra hop the driver reads when numSamples is an exact multiple of
// nMDCTLines (PACFile.WriteFileHeader bumps the shared numSamples,
// pacfile.py:240-242), and PCMFile.WriteFileHeader + the decode driver's
// frames (pcmfile.py:103-147, pacfile.py:478-499).
//
//   k_wav_scan    one thread per file: the 4-byte-step tag scan for 'fmt ' and
//                 'data' exactly as the reference (not a RIFF chunk walk)
//   k_wav_gather  one workgroup per (file, 64 KiB of output): the file's frames
//                 (+ the quirk hop) into the contiguous int16 PCM the encoder
//                 reads, bytes past the file end as zeros (byte granular, as
//                 the reference pads a short read)
//   k_wav_write   one workgroup per (stream, 64 KiB of output): the 44-byte
//                 header from the coded file's numSamples, then the frames

struct PacWavInfo {        // = pac_wav_info (include/pac_gpu.h)
    int32_t sample_rate, n_channels, bits_per_sample, status;
    int64_t num_samples, data_offset, frames, extra_bytes;
};

__device__ __forceinline__ uint32_t rd_u32(const uint8_t* p) {
    return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint32_t rd_u16(const uint8_t* p) { return p[0] | (p[1] << 8); }
__device__ __forceinline__ bool tag_is(const uint8_t* p, char a, char b, char c, char d) {
    return p[0] == (uint8_t)a && p[1] == (uint8_t)b && p[2] == (uint8_t)c && p[3] == (uint8_t)d;
}

#define PAC_WAV_NOT_RIFF (-1)
#define PAC_WAV_NO_FMT (-2)
#define PAC_WAV_NOT_PCM (-3)
#define PAC_WAV_NOT_16BIT (-4)
#define PAC_WAV_NO_DATA (-5)

__global__ void k_wav_scan(const uint8_t* __restrict__ blob, const int64_t* __restrict__ foff, int n,
                           PacWavInfo* __restrict__ info, int hop) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = blob + foff[i];
    const int64_t len = foff[i + 1] - foff[i];
    PacWavInfo w = {0, 0, 0, 0, 0, 0, 0, 0};
    int64_t pos = 12;
    if (len < 12 || !tag_is(p, 'R', 'I', 'F', 'F') || !tag_is(p + 8, 'W', 'A', 'V', 'E')) {
        w.status = PAC_WAV_NOT_RIFF;
        info[i] = w;
        return;
    }
    while (true) {                                   // pcmfile.py:38-42
        if (pos + 4 > len) { w.status = PAC_WAV_NO_FMT; info[i] = w; return; }
        const bool hit = tag_is(p + pos, 'f', 'm', 't', ' ');
        pos += 4;
        if (hit) break;
    }
    if (pos + 20 > len) { w.status = PAC_WAV_NO_FMT; info[i] = w; return; }
    const uint32_t fmt_tag = rd_u16(p + pos + 4), nch = rd_u16(p + pos + 6);
    w.n_channels = (int32_t)nch;
    w.sample_rate = (int32_t)rd_u32(p + pos + 8);
    w.bits_per_sample = (int32_t)rd_u16(p + pos + 18);
    pos += 20;
    if (fmt_tag != 1 || nch == 0) { w.status = PAC_WAV_NOT_PCM; info[i] = w; return; }
    if (w.bits_per_sample != 16) { w.status = PAC_WAV_NOT_16BIT; info[i] = w; return; }
    while (true) {                                   // pcmfile.py:48-52
        if (pos + 4 > len) { w.status = PAC_WAV_NO_DATA; info[i] = w; return; }
        const bool hit = tag_is(p + pos, 'd', 'a', 't', 'a');
        pos += 4;
        if (hit) break;
    }
    if (pos + 4 > len) { w.status = PAC_WAV_NO_DATA; info[i] = w; return; }
    w.num_samples = (int64_t)(rd_u32(p + pos) / (nch * 2u));
    w.data_offset = pos + 4;
    w.frames = w.num_samples;
    // ReadDataBlock stops at the first hop whose read comes back empty
    // (pcmfile.py:69-80, the driver's break at pacfile.py:482): a file that
    // holds fewer data bytes than its header claims (cut short, or a streaming
    // header's 0xFFFFFFFF) is coded up to its last byte, the partial hop
    // zero-padded, and never gets the extra hop
    const int64_t avail = len - w.data_offset > 0 ? len - w.data_offset : 0;
    const int64_t have = (avail + nch * 2 - 1) / (nch * 2);   // frames with at least one byte in the file
    if (have < w.num_samples) {
        w.frames = have;
    } else if (w.num_samples % hop == 0) {           // the extra hop after the data (pacfile.py:240-242)
        const int64_t after = w.data_offset + w.num_samples * nch * 2;
        int64_t ex = len - after;
        ex = ex < 0 ? 0 : (ex > (int64_t)hop * nch * 2 ? (int64_t)hop * nch * 2 : ex);
        w.extra_bytes = ex;
        if (ex > 0) w.frames += hop;
    }
    info[i] = w;
}

#define PAC_WAV_SEG 65536      // output bytes per gather / write workgroup

// out (int16 frames, streams back to back at byte 2 nch fo[s]) <- file bytes
// [data_offset, data_offset + 2 nch frames), zero past the file's end
__global__ __launch_bounds__(256) void k_wav_gather(const uint8_t* __restrict__ blob,
                                                    const int64_t* __restrict__ foff,
                                                    const PacWavInfo* __restrict__ info,
                                                    const int64_t* __restrict__ fo, const int64_t* __restrict__ segb,
                                                    int n, int nch, uint8_t* __restrict__ out) {
    int lo = 0, hi = n;                              // file of this segment: last s with segb[s] <= blockIdx.x
    while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (segb[mid] <= (int64_t)blockIdx.x) lo = mid; else hi = mid; }
    const int s = lo;
    const int64_t nbytes = (fo[s + 1] - fo[s]) * nch * 2;
    const int64_t b0 = ((int64_t)blockIdx.x - segb[s]) * PAC_WAV_SEG;
    const int64_t b1 = b0 + PAC_WAV_SEG < nbytes ? b0 + PAC_WAV_SEG : nbytes;
    const uint8_t* src = blob + foff[s] + info[s].data_offset;
    const int64_t avail = (foff[s + 1] - foff[s]) - info[s].data_offset;    // file bytes from the data start
    uint8_t* dst = out + fo[s] * nch * 2;
    for (int64_t k = b0 + threadIdx.x; k < b1; k += 256) dst[k] = k < avail ? src[k] : (uint8_t)0;
}

// PCMFile.WriteFileHeader (pcmfile.py:103-116) from numSamples, then the frames
__device__ __forceinline__ uint8_t wav_header_byte(int k, int64_t ns, int nch, int fs) {
    const uint32_t data_bytes = (uint32_t)(ns * nch * 2);
    uint32_t v = 0;
    int o = 0;
    if (k < 4) return (uint8_t)"RIFF"[k];
    if (k < 8) { v = 36 + data_bytes; o = k - 4; }
    else if (k < 16) return (uint8_t)"WAVEfmt "[k - 8];
    else if (k < 20) { v = 16; o = k - 16; }
    else if (k < 22) { v = 1; o = k - 20; }
    else if (k < 24) { v = (uint32_t)nch; o = k - 22; }
    else if (k < 28) { v = (uint32_t)fs; o = k - 24; }
    else if (k < 32) { v = (uint32_t)(fs * nch * 2); o = k - 28; }
    else if (k < 34) { v = (uint32_t)(nch * 2); o = k - 32; }
    else if (k < 36) { v = 16; o = k - 34; }
    else if (k < 40) return (uint8_t)"data"[k - 36];
    else { v = data_bytes; o = k - 40; }
    return (uint8_t)(v >> (8 * o));
}

__global__ __launch_bounds__(256) void k_wav_write(const uint8_t* __restrict__ pcm, const int64_t* __restrict__ fo,
                                                   const int64_t* __restrict__ num_samples,
                                                   const int64_t* __restrict__ wo, const int64_t* __restrict__ segb,
                                                   int n, int nch, int fs, uint8_t* __restrict__ out) {
    int lo = 0, hi = n;
    while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (segb[mid] <= (int64_t)blockIdx.x) lo = mid; else hi = mid; }
    const int s = lo;
    const int64_t nbytes = wo[s + 1] - wo[s];
    const int64_t b0 = ((int64_t)blockIdx.x - segb[s]) * PAC_WAV_SEG;
    const int64_t b1 = b0 + PAC_WAV_SEG < nbytes ? b0 + PAC_WAV_SEG : nbytes;
    const uint8_t* src = pcm + fo[s] * nch * 2;
    uint8_t* dst = out + wo[s];
    for (int64_t k = b0 + threadIdx.x; k < b1; k += 256)
        dst[k] = k < 44 ? wav_header_byte((int)k, num_samples[s], nch, fs) : src[k - 44];
}
