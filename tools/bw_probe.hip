// bw_probe.hip -- the HBM rates this box reaches with hand-written gfx950 kernels, for bench.py's
// roofline.measured_ceiling (torch.copy_ / index_select are not a ceiling).
// Built by __graft_entry__.build() into dlrm.jl_amd/lib/libdlrm_probe.so; bench.py times each
// launch with HIP events on the stream it passes.  Measurement only: nothing in the hot path
// links it.
//   dlrm_probe_copy    dst[i] = src[i], 16 B per lane, grid-stride (read + write)
//   dlrm_probe_read    a contiguous read, 16 B per lane (read only; one float per workgroup out)
//   dlrm_probe_gather  nitems random rows of row_bytes (64..1024) from a table, row_bytes / 16 lanes
//                      per row, each row line-aligned (read only) -- tools/fetch_probe.hip's shape
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void probe_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__global__ __launch_bounds__(256) void probe_read(const u32x4* __restrict__ src, int64_t n, float* __restrict__ out) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const u32x4 v = __builtin_nontemporal_load(src + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = 1.0f;
}

__device__ __forceinline__ uint64_t probe_row(uint32_t item, uint64_t nrows) {
    uint32_t h = item * 0x9E3779B1u;
    h ^= h >> 15;
    h *= 0x85EBCA77u;
    h ^= h >> 13;
    return (uint64_t)h % nrows;
}

template <int R>
__global__ __launch_bounds__(256) void probe_gather(const u32x4* __restrict__ table, uint64_t nrows, int nitems,
                                                    float* __restrict__ out) {
    constexpr int LPR = R / 16;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int item = tid / LPR, v = tid % LPR;
    uint32_t acc = 0;
    if (item < nitems) {
        const u32x4 x = table[probe_row(item, nrows) * LPR + v];
        acc = x.x ^ x.y ^ x.z ^ x.w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = 1.0f;
}

static int grid_for(int64_t n16) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t want = (n16 + 255) / 256;
    const int64_t cap = (int64_t)cus * 16;
    return (int)(want < cap ? (want < 1 ? 1 : want) : cap);
}

extern "C" {

int dlrm_probe_copy(const void* src, void* dst, int64_t bytes, void* stream) {
    const int64_t n = bytes / 16;
    hipLaunchKernelGGL(probe_copy, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src,
                       (u32x4*)dst, n);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int dlrm_probe_read(const void* src, int64_t bytes, float* out, void* stream) {
    const int64_t n = bytes / 16;
    hipLaunchKernelGGL(probe_read, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src, n, out);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int dlrm_probe_gather(const void* table, int64_t table_bytes, int row_bytes, int nitems, float* out, void* stream) {
    const uint64_t nrows = (uint64_t)(table_bytes / row_bytes);
    const int64_t threads = (int64_t)nitems * (row_bytes / 16);
    const unsigned grid = (unsigned)((threads + 255) / 256);
    hipStream_t s = (hipStream_t)stream;
    const u32x4* t = (const u32x4*)table;
    switch (row_bytes) {
        case 64: hipLaunchKernelGGL(probe_gather<64>, dim3(grid), dim3(256), 0, s, t, nrows, nitems, out); break;
        case 128: hipLaunchKernelGGL(probe_gather<128>, dim3(grid), dim3(256), 0, s, t, nrows, nitems, out); break;
        case 256: hipLaunchKernelGGL(probe_gather<256>, dim3(grid), dim3(256), 0, s, t, nrows, nitems, out); break;
        case 512: hipLaunchKernelGGL(probe_gather<512>, dim3(grid), dim3(256), 0, s, t, nrows, nitems, out); break;
        case 1024: hipLaunchKernelGGL(probe_gather<1024>, dim3(grid), dim3(256), 0, s, t, nrows, nitems, out); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
