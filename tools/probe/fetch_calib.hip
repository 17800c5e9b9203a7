// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access shapes of
// k_master_thr: rocprofv3's FETCH_SIZE is documented
// (MI355X_MICROARCH.md, HBM) to count half the bytes of a 16-B-per-lane
// streaming read; the threshold kernel's row reads and writes are 8 B per
// lane and its spectra reads 4 x 16 B per lane.  Each kernel below touches a
// known byte count once, from a 1 GiB buffer evicted from the Infinity Cache
// by a 512 MiB scratch write between kernels, so its counters can be divided
// by the known bytes.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/fetch_calib tools/probe/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -- ./tools/probe/fetch_calib   (WRITE_SIZE: a second pass)
//
// kernels (names carry the shape):
//   k_rd8      64 lanes x 8 B contiguous per wave instruction (thr's row reads)
//   k_rd16     64 lanes x 16 B contiguous (the guide's calibrated shape)
//   k_rd16x4   each lane 4 consecutive 16 B, lanes 64 B apart (thr's spectra reads)
//   k_wr8      64 lanes x 8 B contiguous stores (thr's row writes)
//   k_wr16     64 lanes x 16 B contiguous stores
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

static constexpr size_t NBYTES = 1ull << 30;      // bytes each kernel touches
static constexpr size_t SCRATCH = 512ull << 20;    // Infinity Cache eviction

__global__ void k_rd8(const double* __restrict__ a, size_t n, double* __restrict__ out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[i];
    if (s == 1.2345) out[0] = s;       // never taken on the zero-filled input: keeps the loads
}
__global__ void k_rd16(const double2* __restrict__ a, size_t n, double* __restrict__ out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 1.2345) out[0] = s;
}
__global__ void k_rd16x4(const double2* __restrict__ a, size_t n4, double* __restrict__ out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const double2* p = a + 4 * i;
#pragma unroll
        for (int k = 0; k < 4; ++k) { const double2 v = p[k]; s += v.x + v.y; }
    }
    if (s == 1.2345) out[0] = s;
}
__global__ void k_wr8(double* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = (double)i;
}
__global__ void k_wr16(double2* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_double2((double)i, 1.0);
}

int main() {
    char *a, *scratch;
    double* out;
    CHK(hipMalloc(&a, NBYTES));
    CHK(hipMalloc(&scratch, SCRATCH));
    CHK(hipMalloc(&out, 64));
    CHK(hipMemset(a, 0, NBYTES));
    const dim3 grid(256 * 8 * 4), block(256);
    auto evict = [&]() { return hipMemset(scratch, 1, SCRATCH); };
    CHK(evict());
    hipLaunchKernelGGL(k_rd8, grid, block, 0, 0, (const double*)a, NBYTES / 8, out);
    CHK(evict());
    hipLaunchKernelGGL(k_rd16, grid, block, 0, 0, (const double2*)a, NBYTES / 16, out);
    CHK(evict());
    hipLaunchKernelGGL(k_rd16x4, grid, block, 0, 0, (const double2*)a, NBYTES / 64, out);
    CHK(evict());
    hipLaunchKernelGGL(k_wr8, grid, block, 0, 0, (double*)a, NBYTES / 8);
    CHK(evict());
    hipLaunchKernelGGL(k_wr16, grid, block, 0, 0, (double2*)a, NBYTES / 16);
    CHK(hipDeviceSynchronize());
    printf("{\"bytes_per_kernel\": %zu}\n", NBYTES);
    CHK(hipFree(a));
    CHK(hipFree(scratch));
    CHK(hipFree(out));
    return 0;
}
