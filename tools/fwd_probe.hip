// Microbenchmark: where does the metric forward's time go?  A standalone replica of the step
// forward's one-hot body (26 tables x 128 fp32 + x, B = 2048, one wave per sample, 16 row loads
// of 16 rows x 64 B in flight per wave, fp32 Gram on v_mfma_f32_16x16x4f32, output staged in
// LDS), with its pieces switched off one at a time:
//   MODE bit 0: the MFMAs (off: the fragments are summed on the VALU)
//   MODE bit 1: the 480-float output row (off: one float per sample)
// and two table layouts: the Kaggle row counts (criteo.jl:350-377: 12 tables < 2048 rows, whose
// rows every sample shares) or every table as large as the largest (all rows random in HBM).
// Build: hipcc -O3 --offload-arch=gfx950 -o fwd_probe tools/fwd_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int T = 26, F = 27, D = 128, B = 2048, W = 128 + 351 + 1, NBATCH = 64;

struct Tabs { const float* p[T]; };

template <int MODE, int WPB>
__global__ __launch_bounds__(64 * WPB) void fwd(Tabs tabs, const int* __restrict__ idx, const float* __restrict__ x,
                                                float* __restrict__ out, const float* __restrict__ zero) {
    __shared__ __attribute__((aligned(16))) float stage_all[WPB][1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 15, q = lane >> 4;
    const int b = blockIdx.x * WPB + w;
    if (b >= B) return;
    if (MODE & 8) {  // empty: one store
        if (lane == 0) out[(size_t)b * W] = 0.f;
        return;
    }
    float* stage = stage_all[w];
    const float* src[2];
    int ri[2];
#pragma unroll
    for (int I = 0; I < 2; ++I) {
        const int row = I * 16 + c;
        ri[I] = (row >= 1 && row < F) ? idx[(row - 1) * B + b] : 0;
    }
#pragma unroll
    for (int I = 0; I < 2; ++I) {
        const int row = I * 16 + c;
        src[I] = row == 0 ? x + (size_t)b * D : (row < F ? tabs.p[row - 1] + (size_t)ri[I] * D : zero);
    }
    if (MODE & 4) {  // index loads only
        if (lane == 0) out[(size_t)b * W] = (float)(ri[0] + ri[1]);
        return;
    }
    __builtin_amdgcn_sched_barrier(0);
    f4 a[8][2];
#pragma unroll
    for (int uu = 0; uu < 8; ++uu)
#pragma unroll
        for (int I = 0; I < 2; ++I) a[uu][I] = *(const f4*)(src[I] + uu * 16 + q * 4);
    __builtin_amdgcn_sched_barrier(0);
    f4 acc[3] = {f4{0, 0, 0, 0}, f4{0, 0, 0, 0}, f4{0, 0, 0, 0}};
    if (MODE & 1) {
#pragma unroll
        for (int uu = 0; uu < 8; ++uu) {
            int ij = 0;
#pragma unroll
            for (int I = 0; I < 2; ++I)
#pragma unroll
                for (int J = 0; J <= I; ++J, ++ij)
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        acc[ij] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[uu][I][k], a[uu][J][k], acc[ij], 0, 0, 0);
        }
    } else {
#pragma unroll
        for (int uu = 0; uu < 8; ++uu) { acc[0] += a[uu][0]; acc[1] += a[uu][1]; }
    }
    float* orow = out + (size_t)b * W;
    if (MODE & 2) {
        if (c == 0)
#pragma unroll
            for (int uu = 0; uu < 8; ++uu) *(f4*)(stage + uu * 16 + q * 4) = a[uu][0];
        int ij = 0;
#pragma unroll
        for (int I = 0; I < 2; ++I)
#pragma unroll
            for (int J = 0; J <= I; ++J, ++ij) {
                const int j = J * 16 + c;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = I * 16 + 4 * q + r;
                    if (i < F && j < i) stage[D + i * (i - 1) / 2 + j] = acc[ij][r];
                }
            }
        if (lane == 0) stage[W - 1] = 0.f;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int e = lane; e < W; e += 64) orow[e] = stage[e];
    } else {
        const f4 s = acc[0] + acc[1] + acc[2];
        if (lane == 0) orow[0] = s.x + s.y + s.z + s.w;
    }
}

template <int MODE, int WPB>
double run(Tabs tabs, const int* idx, const float* x, float* out, const float* zero) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int grid = B / WPB;
    for (int i = 0; i < NBATCH; ++i)
        hipLaunchKernelGGL((fwd<MODE, WPB>), dim3(grid), dim3(64 * WPB), 0, 0, tabs, idx + (size_t)i * T * B, x, out, zero);
    const int reps = 4 * NBATCH;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((fwd<MODE, WPB>), dim3(grid), dim3(64 * WPB), 0, 0, tabs, idx + (size_t)(i % NBATCH) * T * B, x,
                           out, zero);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
}


// Two waves per sample (column halves 0..63 / 64..127): 8 row loads and 48 MFMAs per wave, the
// odd wave's partial Gram tiles added to the even wave's through LDS.
template <int WPB>
__global__ __launch_bounds__(64 * WPB) void fwd2(Tabs tabs, const int* __restrict__ idx, const float* __restrict__ x,
                                                 float* __restrict__ out, const float* __restrict__ zero) {
    __shared__ __attribute__((aligned(16))) float stage_all[WPB / 2][1024];
    __shared__ __attribute__((aligned(16))) f4 part_all[WPB / 2][3][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 15, q = lane >> 4;
    const int h = w & 1;
    const int b = blockIdx.x * (WPB / 2) + (w >> 1);
    float* stage = stage_all[w >> 1];
    f4* part = part_all[w >> 1][0];
    const float* src[2];
    int ri[2];
#pragma unroll
    for (int I = 0; I < 2; ++I) {
        const int row = I * 16 + c;
        ri[I] = (row >= 1 && row < F) ? idx[(row - 1) * B + b] : 0;
    }
#pragma unroll
    for (int I = 0; I < 2; ++I) {
        const int row = I * 16 + c;
        src[I] = row == 0 ? x + (size_t)b * D : (row < F ? tabs.p[row - 1] + (size_t)ri[I] * D : zero);
    }
    __builtin_amdgcn_sched_barrier(0);
    f4 a[4][2];
#pragma unroll
    for (int uu = 0; uu < 4; ++uu)
#pragma unroll
        for (int I = 0; I < 2; ++I) a[uu][I] = *(const f4*)(src[I] + h * 64 + uu * 16 + q * 4);
    __builtin_amdgcn_sched_barrier(0);
    f4 acc[3] = {f4{0, 0, 0, 0}, f4{0, 0, 0, 0}, f4{0, 0, 0, 0}};
#pragma unroll
    for (int uu = 0; uu < 4; ++uu) {
        int ij = 0;
#pragma unroll
        for (int I = 0; I < 2; ++I)
#pragma unroll
            for (int J = 0; J <= I; ++J, ++ij)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    acc[ij] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[uu][I][k], a[uu][J][k], acc[ij], 0, 0, 0);
    }
    if (c == 0)
#pragma unroll
        for (int uu = 0; uu < 4; ++uu) *(f4*)(stage + h * 64 + uu * 16 + q * 4) = a[uu][0];
    if (h == 1)
#pragma unroll
        for (int k = 0; k < 3; ++k) part[k * 64 + lane] = acc[k];
    __syncthreads();
    if (h == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) acc[k] += part[k * 64 + lane];
        int ij = 0;
#pragma unroll
        for (int I = 0; I < 2; ++I)
#pragma unroll
            for (int J = 0; J <= I; ++J, ++ij) {
                const int j = J * 16 + c;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = I * 16 + 4 * q + r;
                    if (i < F && j < i) stage[D + i * (i - 1) / 2 + j] = acc[ij][r];
                }
            }
        if (lane == 0) stage[W - 1] = 0.f;
    }
    __syncthreads();
    float* orow = out + (size_t)b * W;
    for (int e = lane + 64 * h; e < W; e += 128) orow[e] = stage[e];
}

template <int WPB>
double run2(Tabs tabs, const int* idx, const float* x, float* out, const float* zero) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int grid = 2 * B / WPB;
    for (int i = 0; i < NBATCH; ++i)
        hipLaunchKernelGGL((fwd2<WPB>), dim3(grid), dim3(64 * WPB), 0, 0, tabs, idx + (size_t)i * T * B, x, out, zero);
    const int reps = 4 * NBATCH;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((fwd2<WPB>), dim3(grid), dim3(64 * WPB), 0, 0, tabs, idx + (size_t)(i % NBATCH) * T * B, x,
                           out, zero);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
}

int main() {
    static const int64_t kaggle[T] = {1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593, 3194,
                                      27, 14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105, 142572};
    float *x, *out, *zero;
    CK(hipMalloc(&x, (size_t)B * D * 4));
    CK(hipMalloc(&out, (size_t)B * W * 4));
    CK(hipMalloc(&zero, 4096));
    CK(hipMemset(x, 0, (size_t)B * D * 4));
    CK(hipMemset(zero, 0, 4096));
    int* idx;
    CK(hipMalloc(&idx, (size_t)NBATCH * T * B * 4));
    std::mt19937_64 g(1);
    for (int layout = 0; layout < 2; ++layout) {
        // layout 0: Kaggle rows; 1: every table 10.1M rows (all rows random in HBM)
        Tabs tabs;
        std::vector<float*> mem(T);
        std::vector<int64_t> n(T);
        for (int t = 0; t < T; ++t) {
            n[t] = layout == 0 ? kaggle[t] : 10131227;
            CK(hipMalloc(&mem[t], n[t] * D * 4));
            CK(hipMemset(mem[t], 0, n[t] * D * 4));
            tabs.p[t] = mem[t];
        }
        std::vector<int> h((size_t)NBATCH * T * B);
        for (int k = 0; k < NBATCH; ++k)
            for (int t = 0; t < T; ++t)
                for (int b = 0; b < B; ++b) h[((size_t)k * T + t) * B + b] = (int)(g() % n[t]);
        CK(hipMemcpy(idx, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        const char* lname = layout == 0 ? "kaggle rows " : "all 10.1M   ";
        printf("%s empty           wpb4 %7.2f us\n", lname, run<8, 4>(tabs, idx, x, out, zero));
        printf("%s index only      wpb4 %7.2f us\n", lname, run<4, 4>(tabs, idx, x, out, zero));
        printf("%s gather+mfma+out wpb4 %7.2f us\n", lname, run<3, 4>(tabs, idx, x, out, zero));
        printf("%s gather+mfma     wpb4 %7.2f us\n", lname, run<1, 4>(tabs, idx, x, out, zero));
        printf("%s gather+out      wpb4 %7.2f us\n", lname, run<2, 4>(tabs, idx, x, out, zero));
        printf("%s gather          wpb4 %7.2f us\n", lname, run<0, 4>(tabs, idx, x, out, zero));
        printf("%s gather+mfma+out wpb1 %7.2f us\n", lname, run<3, 1>(tabs, idx, x, out, zero));
        printf("%s gather          wpb1 %7.2f us\n", lname, run<0, 1>(tabs, idx, x, out, zero));
        printf("%s gather+mfma+out wpb8 %7.2f us\n", lname, run<3, 8>(tabs, idx, x, out, zero));
        printf("%s 2 waves/sample  wpb4 %7.2f us\n", lname, run2<4>(tabs, idx, x, out, zero));
        printf("%s 2 waves/sample  wpb8 %7.2f us\n", lname, run2<8>(tabs, idx, x, out, zero));
        printf("%s 2 waves/sample  wpb16 %6.2f us\n", lname, run2<16>(tabs, idx, x, out, zero));
        for (int t = 0; t < T; ++t) CK(hipFree(mem[t]));
    }
    return 0;
}
