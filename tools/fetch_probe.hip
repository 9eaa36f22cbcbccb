// fetch_probe.hip -- what FETCH_SIZE reports for reads of known size on gfx950 (VERDICT r2 item 5:
// settle the counter correction for the D = 16 apply's 64-B random rows).
//
// Each kernel reads a known number of bytes and writes one float per workgroup (so nothing is
// optimised away):
//   stream<V>   : a contiguous 256 MB read, 16 B per lane           (the guide's "x2" case)
//   gather<R>   : N random rows of R bytes (R = 64, 128, 256, 512) from a 4 GB table, one row per
//                 R/16 lanes, rows spread so no two share a 128-B line
// Run under `rocprofv3 --pmc FETCH_SIZE` (its own pass); tools/fetch_probe_summary.py divides the
// counter by the bytes each launch requested.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_read(const u32x4* __restrict__ src, int64_t n, float* __restrict__ out) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const u32x4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = 1.0f;
}

// row r of the gather: a hash of the item, times the row stride (256 B), so every row sits in its
// own 128-B line and rows are spread over the whole table
__device__ __forceinline__ uint64_t row_of(uint32_t item, uint64_t nrows) {
    uint32_t h = item * 0x9E3779B1u;
    h ^= h >> 15;
    h *= 0x85EBCA77u;
    h ^= h >> 13;
    return (uint64_t)h % nrows;
}

template <int R>
__global__ __launch_bounds__(256) void gather_rows(const u32x4* __restrict__ table, uint64_t nrows, int nitems,
                                                   float* __restrict__ out) {
    constexpr int LPR = R / 16;        // lanes per row
    constexpr int STRIDE = 512 / 16;   // row stride in 16-B units (512 B: one row per two lines)
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int item = tid / LPR, v = tid % LPR;
    uint32_t acc = 0;
    if (item < nitems) {
        const u32x4 x = table[row_of(item, nrows) * STRIDE + v];
        acc = x.x ^ x.y ^ x.z ^ x.w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = 1.0f;
}

int main() {
    const size_t tbytes = (size_t)4 << 30;
    u32x4* table;
    float* out;
    CHECK(hipMalloc(&table, tbytes));
    CHECK(hipMemset(table, 1, tbytes));
    CHECK(hipMalloc(&out, 1 << 20));
    const uint64_t nrows = tbytes / 512;
    const int64_t sn = ((int64_t)256 << 20) / 16;
    const int nitems = 1 << 18;  // 262,144 rows per launch
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(stream_read, dim3(4096), dim3(256), 0, 0, table, sn, out);
        hipLaunchKernelGGL(gather_rows<64>, dim3((nitems * 4 + 255) / 256), dim3(256), 0, 0, table, nrows, nitems, out);
        hipLaunchKernelGGL(gather_rows<128>, dim3((nitems * 8 + 255) / 256), dim3(256), 0, 0, table, nrows, nitems, out);
        hipLaunchKernelGGL(gather_rows<256>, dim3((nitems * 16 + 255) / 256), dim3(256), 0, 0, table, nrows, nitems, out);
        hipLaunchKernelGGL(gather_rows<512>, dim3((nitems * 32 + 255) / 256), dim3(256), 0, 0, table, nrows, nitems, out);
    }
    CHECK(hipDeviceSynchronize());
    printf("{\"stream_read\": %lld, \"gather_rows<64>\": %lld, \"gather_rows<128>\": %lld, \"gather_rows<256>\": %lld, "
           "\"gather_rows<512>\": %lld}\n",
           (long long)sn * 16, (long long)nitems * 64, (long long)nitems * 128, (long long)nitems * 256,
           (long long)nitems * 512);
    CHECK(hipFree(table));
    CHECK(hipFree(out));
    return 0;
}
