// bitonic_probe: checks dlrm.jl_amd/csrc/bitonic.hpp (one wave sorts 64·R keys in registers)
// against std::sort on random and adversarial keys, for 32- and 64-bit keys, and times it
// (HIP events, many waves in flight as in the wave build).
//   hipcc -O3 --offload-arch=gfx950 -I dlrm.jl_amd/csrc tools/bitonic_probe.hip -o tools/bin/bitonic_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "bitonic.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int R, typename V>
__global__ __launch_bounds__(256) void sort_kernel(const V* in, V* out, int reps) {
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    V a[R];
#pragma unroll
    for (int r = 0; r < R; ++r) a[r] = in[(size_t)wave * 64 * R + r * 64 + lane];
    for (int k = 0; k < reps; ++k) {
        dlrm::wave_bitonic_sort<R>(a);
        if (reps > 1) {  // (timing: re-sort a permuted copy so the compiler cannot drop the loop)
#pragma unroll
            for (int r = 0; r < R; ++r) a[r] = a[r] ^ (V)(k & 1);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) out[(size_t)wave * 64 * R + r * 64 + lane] = a[r];
}

template <int R, typename V>
static int check(int waves, int mode, std::mt19937_64& g) {
    const int n = 64 * R;
    std::vector<V> h((size_t)waves * n), o(h.size());
    for (int w = 0; w < waves; ++w)
        for (int i = 0; i < n; ++i) {
            uint64_t key;
            if (mode == 0) key = g() % 1000003;        // random rows
            else if (mode == 1) key = g() % 3;         // hot rows: three keys
            else if (mode == 2) key = (uint64_t)(n - i);  // descending
            else key = 0xFFFFFFFFull >> 11;            // one row, padding-sized key
            const V pos = (V)i;
            h[(size_t)w * n + i] = (V)((key << 11) | pos);
            if (mode == 3 && i >= n / 2) h[(size_t)w * n + i] = (V)~(V)0;  // padding keys
        }
    V *din, *dout;
    CK(hipMalloc(&din, h.size() * sizeof(V)));
    CK(hipMalloc(&dout, h.size() * sizeof(V)));
    CK(hipMemcpy(din, h.data(), h.size() * sizeof(V), hipMemcpyHostToDevice));
    hipLaunchKernelGGL((sort_kernel<R, V>), dim3(waves / 4), dim3(256), 0, 0, din, dout, 1);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(o.data(), dout, o.size() * sizeof(V), hipMemcpyDeviceToHost));
    int bad = 0;
    for (int w = 0; w < waves; ++w) {
        std::vector<V> ref(h.begin() + (size_t)w * n, h.begin() + (size_t)(w + 1) * n);
        std::sort(ref.begin(), ref.end());
        for (int i = 0; i < n; ++i)
            if (ref[i] != o[(size_t)w * n + i]) {
                if (bad < 3) printf("  mismatch wave %d elem %d: %llx vs %llx\n", w, i, (unsigned long long)o[(size_t)w * n + i],
                                    (unsigned long long)ref[i]);
                ++bad;
            }
    }
    // timing: 416 waves (the metric build's), 1 sort each, back to back; and 64 sorts per wave
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms1 = 0, ms64 = 0;
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(e0));
        for (int it = 0; it < 20; ++it) hipLaunchKernelGGL((sort_kernel<R, V>), dim3(416 / 4), dim3(256), 0, 0, din, dout, 1);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms1, e0, e1));
        CK(hipEventRecord(e0));
        for (int it = 0; it < 20; ++it) hipLaunchKernelGGL((sort_kernel<R, V>), dim3(416 / 4), dim3(256), 0, 0, din, dout, 65);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms64, e0, e1));
    }
    printf("R=%d %2d-bit mode %d: %s (%d mismatches); 416 waves: %.2f us per launch, %.3f us per extra sort\n", R,
           (int)sizeof(V) * 8, mode, bad ? "FAIL" : "ok", bad, ms1 * 1e3 / 20, (ms64 - ms1) * 1e3 / 20 / 64);
    CK(hipFree(din));
    CK(hipFree(dout));
    return bad;
}

int main() {
    std::mt19937_64 g(1);
    int bad = 0;
    for (int mode = 0; mode < 4; ++mode) {
        bad += check<1, uint32_t>(1024, mode, g);
        bad += check<2, uint32_t>(1024, mode, g);
        bad += check<4, uint32_t>(1024, mode, g);
        bad += check<2, uint64_t>(1024, mode, g);
        bad += check<4, uint64_t>(1024, mode, g);
    }
    printf(bad ? "BITONIC FAIL\n" : "BITONIC OK\n");
    return bad ? 1 : 0;
}
