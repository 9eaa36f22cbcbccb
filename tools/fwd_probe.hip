// Microbenchmark: where does the metric forward's time go?  A standalone replica of the step
// forward's one-hot body (26 tables x 128 fp32 + x, B = 2048, one wave per sample, 16 row loads
// of 16 rows x 64 B in flight per wave, fp32 Gram on v_mfma_f32_16x16x4f32, output staged in
// LDS), with its pieces switched off one at a time:
//   MODE bit 0: the MFMAs (off: the fragments are summed on the VALU)
//   MODE bit 1: the 480-float output row (off: one float per sample)
// and two table layouts: the Kaggle row counts (criteo.jl:350-377: 12 tables < 2048 rows, whose
// rows every sample shares) or every table as large as the largest (all rows random in HBM).
// The library's own forward (dlrm_lookup_interact_fwd, ys = NULL) is timed in the same harness.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/fwd_probe tools/fwd_probe.hip -Ldlrm.jl_amd/lib -ldlrm_hip
//        -Wl,-rpath,'$ORIGIN/../../dlrm.jl_amd/lib'
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <random>

#include "../include/dlrm_hip.h"
#include "../dlrm.jl_amd/csrc/fwd_onehot.hpp"

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

__global__ void fill_random(float* p, int64_t n, uint32_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = ((float)(h & 0xffffff) / 16777216.0f - 0.5f) * 0.01f;
    }
}


// The shipped one-hot body (dlrm.jl_amd/csrc/fwd_onehot.hpp), instantiated here with its knobs.
template <int WPS, bool CONTIG, int WPB, bool TP, bool DEFER>
__global__ __launch_bounds__(64 * WPB, 2) void libbody(int d, int F, int B, const float* __restrict__ x, int64_t x_ld,
                                                      float* __restrict__ out, int64_t out_ld, int padding,
                                                      dlrm::GatherArgs ga, dlrm::TabPtrs tp) {
    __shared__ __attribute__((aligned(16))) float stage_all[WPB * dlrm::kStage];
    dlrm::fwd_body_onehot<float, 2, true, WPB, 128, WPS, CONTIG, TP, DEFER>(
        blockIdx.x, gridDim.x, stage_all, d, F, B, x, x_ld, nullptr, 0, out, out_ld, padding, ga, &tp);
}

template <int WPS, bool CONTIG, int WPB, bool TP = false, bool DEFER = false>
double run_body(const dlrm::TableDesc* dtabs, const int* idx, const float* x, float* out, unsigned* err,
                const dlrm::TableDesc* htabs = nullptr) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int grid = B / (WPB / WPS);
    auto go = [&](int i) {
        dlrm::GatherArgs ga{dtabs, idx + (size_t)(i % NBATCH) * T * B, 0, B, 0, 1, err, nullptr, nullptr};
        dlrm::TabPtrs tp{};
        if (TP) dlrm::fill_tab_ptrs(tp, htabs, T);
        hipLaunchKernelGGL((libbody<WPS, CONTIG, WPB, TP, DEFER>), dim3(grid), dim3(64 * WPB), 0, 0, D, F, B, x,
                           (int64_t)D, out, (int64_t)W, 1, ga, tp);
    };
    for (int i = 0; i < NBATCH; ++i) go(i);
    const int reps = 4 * NBATCH;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) go(i);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
}


// Bisection copy of the shipped body (float, NB = 2, fused, d = 128, two waves per sample), KNOB bits:
//   1: int32 index loaded once (no load_index_if lo/hi pair)   2: table pointers from kernel arguments
//   4: no bounds check (no nrows compare / raise)              8: one __syncthreads fewer (stage only)
template <int KNOB>
__global__ __launch_bounds__(256, 2) void bisect(Tabs tabs, const dlrm::TableDesc* __restrict__ dtabs,
                                                 const int* __restrict__ idx, const float* __restrict__ x,
                                                 float* __restrict__ out, const float* __restrict__ zero,
                                                 unsigned* err) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) float stage_all[2 * 1024 + 2 * 3 * 256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int pair = w >> 1, h = w & 1;
    const int c = lane & 15, q = lane >> 4;
    const int64_t b = (int64_t)blockIdx.x * 2 + pair;
    float* stage = stage_all + pair * 1024;
    f4v* xch = (f4v*)(stage_all + 2 * 1024) + pair * 3 * 64;
    const float* xb = x + b * D;
    float* orow = out + b * W;
    const float* src[2];
    int64_t ri[2];
    dlrm::TableDesc td[2];
#pragma unroll
    for (int I = 0; I < 2; ++I) {
        const int row = I * 16 + c;
        const bool tab = row >= 1 && row < F;
        if (KNOB & 2) td[I] = dlrm::TableDesc{(void*)tabs.p[tab ? row - 1 : 0], 1ll << 40};
        else td[I] = dlrm::load_table(dtabs, tab ? row - 1 : 0);
        if (KNOB & 1) ri[I] = tab ? idx[(row - 1) * B + b] : 0;
        else ri[I] = dlrm::load_index_if(tab, idx, 0, tab ? (int64_t)(row - 1) * B + b : 0);
    }
    bool bad = false;
#pragma unroll
    for (int I = 0; I < 2; ++I) {
        const int row = I * 16 + c;
        const bool tab = row >= 1 && row < F;
        const int64_t r = ri[I];
        const bool ok = (KNOB & 4) ? tab : (tab & (r >= 0) & (r < td[I].nrows));
        bad |= tab & !ok;
        src[I] = row == 0 ? xb : (ok ? (const float*)td[I].data + r * D : nullptr);
    }
    if (!(KNOB & 4) && bad && q == 0 && h == 0) atomicOr(err, 1u);
    f4v acc[3] = {f4v{0, 0, 0, 0}, f4v{0, 0, 0, 0}, f4v{0, 0, 0, 0}};
    __builtin_amdgcn_sched_barrier(0);
    f4v a[4][2];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const int col = (2 * v + h) * 16 + q * 4;
#pragma unroll
        for (int I = 0; I < 2; ++I) a[v][I] = *(const f4v*)(src[I] ? src[I] + col : zero + col);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        int ij = 0;
#pragma unroll
        for (int I = 0; I < 2; ++I)
#pragma unroll
            for (int J = 0; J <= I; ++J, ++ij)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    acc[ij] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[v][I][k], a[v][J][k], acc[ij], 0, 0, 0);
    }
    if (c == 0)
#pragma unroll
        for (int v = 0; v < 4; ++v) *(f4v*)(stage + (2 * v + h) * 16 + q * 4) = a[v][0];
    if (h == 1)
#pragma unroll
        for (int k = 0; k < 3; ++k) xch[k * 64 + lane] = acc[k];
    __syncthreads();
    if (h == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) acc[k] += xch[k * 64 + lane];
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
    for (int e = lane + 64 * h; e < W; e += 128) orow[e] = stage[e];
    if (!(KNOB & 8)) __syncthreads();
}

template <int KNOB>
double run_bisect(Tabs tabs, const dlrm::TableDesc* dtabs, const int* idx, const float* x, float* out, const float* zero,
                  unsigned* err) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto go = [&](int i) {
        hipLaunchKernelGGL((bisect<KNOB>), dim3(B / 2), dim3(256), 0, 0, tabs, dtabs, idx + (size_t)(i % NBATCH) * T * B,
                           x, out, zero, err);
    };
    for (int i = 0; i < NBATCH; ++i) go(i);
    const int reps = 4 * NBATCH;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) go(i);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
}

double run_lib(dlrm_ctx* ctx, dlrm_tables* tb, const int* idx, const float* x, float* out) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto go = [&](int i) {
        const int rc = dlrm_lookup_interact_fwd(ctx, tb, idx + (size_t)(i % NBATCH) * T * B, DLRM_I32, B, 0, B, 1, x, D,
                                                nullptr, 0, out, W, 1);
        if (rc) { printf("lib rc %d: %s\n", rc, dlrm_last_error(ctx)); exit(1); }
    };
    for (int i = 0; i < NBATCH; ++i) go(i);
    const int reps = 4 * NBATCH;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) go(i);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
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

// Software-pipelined forward: SPW samples per wave, every index load of all SPW samples, then
// every row load (sample 0's first), then per sample: MFMAs (even / odd parity partials, the
// shipped order) + staging + stores.  Sample s's MFMAs wait only for its own loads, so they
// run while the later samples' rows are still arriving; only the last sample's tail is exposed.
template <int SPW, int WPB, int OCC>
__global__ __launch_bounds__(64 * WPB, OCC) void fwdp(Tabs tabs, const int* __restrict__ idx, const float* __restrict__ x,
                                                     float* __restrict__ out, const float* __restrict__ zero) {
    __shared__ __attribute__((aligned(16))) float stage_all[WPB][1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 15, q = lane >> 4;
    const int b0 = (blockIdx.x * WPB + w) * SPW;
    float* stage = stage_all[w];
    int ri[SPW][2];
#pragma unroll
    for (int s = 0; s < SPW; ++s)
#pragma unroll
        for (int I = 0; I < 2; ++I) {
            const int row = I * 16 + c;
            ri[s][I] = (row >= 1 && row < F) ? idx[(row - 1) * B + b0 + s] : 0;
        }
    const float* src[SPW][2];
#pragma unroll
    for (int s = 0; s < SPW; ++s)
#pragma unroll
        for (int I = 0; I < 2; ++I) {
            const int row = I * 16 + c;
            src[s][I] = row == 0 ? x + (size_t)(b0 + s) * D : (row < F ? tabs.p[row - 1] + (size_t)ri[s][I] * D : zero);
        }
    __builtin_amdgcn_sched_barrier(0);
    f4 a[SPW][8][2];
#pragma unroll
    for (int s = 0; s < SPW; ++s)
#pragma unroll
        for (int uu = 0; uu < 8; ++uu)
#pragma unroll
            for (int I = 0; I < 2; ++I) a[s][uu][I] = *(const f4*)(src[s][I] + uu * 16 + q * 4);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < SPW; ++s) {
        f4 acc[2][3];
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int k = 0; k < 3; ++k) acc[p][k] = f4{0, 0, 0, 0};
#pragma unroll
        for (int uu = 0; uu < 8; ++uu) {
            int ij = 0;
#pragma unroll
            for (int I = 0; I < 2; ++I)
#pragma unroll
                for (int J = 0; J <= I; ++J, ++ij)
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        acc[uu & 1][ij] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s][uu][I][k], a[s][uu][J][k], acc[uu & 1][ij], 0, 0, 0);
        }
        if (c == 0)
#pragma unroll
            for (int uu = 0; uu < 8; ++uu) *(f4*)(stage + uu * 16 + q * 4) = a[s][uu][0];
        int ij = 0;
#pragma unroll
        for (int I = 0; I < 2; ++I)
#pragma unroll
            for (int J = 0; J <= I; ++J, ++ij) {
                const f4 z = acc[0][ij] + acc[1][ij];
                const int j = J * 16 + c;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = I * 16 + 4 * q + r;
                    if (i < F && j < i) stage[D + i * (i - 1) / 2 + j] = z[r];
                }
            }
        if (lane == 0) stage[W - 1] = 0.f;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        float* orow = out + (size_t)(b0 + s) * W;
        for (int e = lane; e < W; e += 64) orow[e] = stage[e];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

template <int SPW, int WPB, int OCC>
double runp(Tabs tabs, const int* idx, const float* x, float* out, const float* zero) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int grid = B / (WPB * SPW);
    for (int i = 0; i < NBATCH; ++i)
        hipLaunchKernelGGL((fwdp<SPW, WPB, OCC>), dim3(grid), dim3(64 * WPB), 0, 0, tabs, idx + (size_t)i * T * B, x, out, zero);
    const int reps = 4 * NBATCH;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((fwdp<SPW, WPB, OCC>), dim3(grid), dim3(64 * WPB), 0, 0, tabs, idx + (size_t)(i % NBATCH) * T * B,
                           x, out, zero);
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
    dlrm_ctx* ctx = nullptr;
    if (dlrm_ctx_create(0, nullptr, &ctx)) { printf("ctx\n"); return 1; }
    for (int cfg = 1; cfg < 2; ++cfg) {
        const int layout = cfg == 2;       // 0, 1: Kaggle rows; 2: every table 10.1M rows
        const bool randomize = cfg >= 1;   // table contents: zeros (cfg 0) or random
        // layout 0: Kaggle rows; 1: every table 10.1M rows (all rows random in HBM)
        Tabs tabs;
        std::vector<float*> mem(T);
        std::vector<int64_t> n(T);
        for (int t = 0; t < T; ++t) {
            n[t] = layout == 0 ? kaggle[t] : 10131227;
            CK(hipMalloc(&mem[t], n[t] * D * 4));
            if (randomize) hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, mem[t], n[t] * D, (uint32_t)t);
            else CK(hipMemset(mem[t], 0, n[t] * D * 4));
            tabs.p[t] = mem[t];
        }
        std::vector<int> h((size_t)NBATCH * T * B);
        for (int k = 0; k < NBATCH; ++k)
            for (int t = 0; t < T; ++t)
                for (int b = 0; b < B; ++b) h[((size_t)k * T + t) * B + b] = (int)(g() % n[t]);
        CK(hipMemcpy(idx, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        const char* lname = cfg == 0 ? "kaggle, 0s  " : (cfg == 1 ? "kaggle, rnd " : "10.1M, rnd  ");
        hipLaunchKernelGGL(fill_random, dim3(256), dim3(256), 0, 0, x, (int64_t)B * D, 99u);
        CK(hipDeviceSynchronize());
        dlrm_tables* tb = nullptr;
        {
            std::vector<void*> dp(mem.begin(), mem.end());
            if (dlrm_tables_create(ctx, T, D, DLRM_F32, dp.data(), n.data(), &tb)) { printf("tables\n"); return 1; }
        }
        printf("%s LIBRARY fwd          %7.2f us\n", lname, run_lib(ctx, tb, idx, x, out));
        {
            std::vector<dlrm::TableDesc> hd(T);
            for (int t = 0; t < T; ++t) hd[t] = dlrm::TableDesc{mem[t], n[t]};
            dlrm::TableDesc* dtabs;
            unsigned* err;
            CK(hipMalloc(&dtabs, T * sizeof(dlrm::TableDesc)));
            CK(hipMalloc(&err, 16));
            CK(hipMemset(err, 0, 16));
            CK(hipMemcpy(dtabs, hd.data(), T * sizeof(dlrm::TableDesc), hipMemcpyHostToDevice));
            printf("%s body wps2 interleaved %7.2f us\n", lname, run_body<2, false, 4>(dtabs, idx, x, out, err));
            printf("%s body wps2 contiguous  %7.2f us\n", lname, run_body<2, true, 4>(dtabs, idx, x, out, err));
            printf("%s body wps2 TabPtrs     %7.2f us\n", lname, run_body<2, false, 4, true>(dtabs, idx, x, out, err, hd.data()));
            printf("%s body wps2 defer raise %7.2f us\n", lname, run_body<2, false, 4, false, true>(dtabs, idx, x, out, err, hd.data()));
            printf("%s body wps2 TabPtrs+defer%6.2f us\n", lname, run_body<2, false, 4, true, true>(dtabs, idx, x, out, err, hd.data()));
            printf("%s body wps1 TabPtrs+defer%6.2f us\n", lname, run_body<1, false, 4, true, true>(dtabs, idx, x, out, err, hd.data()));
            printf("%s body wps2 contig wpb8 %7.2f us\n", lname, run_body<2, true, 8>(dtabs, idx, x, out, err));
            printf("%s body wps1             %7.2f us\n", lname, run_body<1, false, 4>(dtabs, idx, x, out, err));
            float* zf;
            CK(hipMalloc(&zf, 4096));
            CK(hipMemset(zf, 0, 4096));
            printf("%s bisect 0              %7.2f us\n", lname, run_bisect<0>(tabs, dtabs, idx, x, out, zf, err));
            printf("%s bisect 1 (int32 idx)  %7.2f us\n", lname, run_bisect<1>(tabs, dtabs, idx, x, out, zf, err));
            printf("%s bisect 2 (kernarg tab)%7.2f us\n", lname, run_bisect<2>(tabs, dtabs, idx, x, out, zf, err));
            printf("%s bisect 4 (no bounds)  %7.2f us\n", lname, run_bisect<4>(tabs, dtabs, idx, x, out, zf, err));
            printf("%s bisect 8 (2 barriers) %7.2f us\n", lname, run_bisect<8>(tabs, dtabs, idx, x, out, zf, err));
            printf("%s bisect 15 (all)       %7.2f us\n", lname, run_bisect<15>(tabs, dtabs, idx, x, out, zf, err));
            CK(hipFree(zf));
            CK(hipFree(dtabs)); CK(hipFree(err));
        }
        printf("%s pipelined spw1 wpb4   %7.2f us\n", lname, runp<1, 4, 2>(tabs, idx, x, out, zero));
        printf("%s pipelined spw2 wpb4   %7.2f us\n", lname, runp<2, 4, 1>(tabs, idx, x, out, zero));
        printf("%s pipelined spw2 wpb4 o2%7.2f us\n", lname, runp<2, 4, 2>(tabs, idx, x, out, zero));
        printf("%s pipelined spw2 wpb2   %7.2f us\n", lname, runp<2, 2, 2>(tabs, idx, x, out, zero));
        printf("%s pipelined spw2 wpb1   %7.2f us\n", lname, runp<2, 1, 2>(tabs, idx, x, out, zero));
        printf("%s pipelined spw4 wpb2   %7.2f us\n", lname, runp<4, 2, 1>(tabs, idx, x, out, zero));
        printf("%s pipelined spw4 wpb1   %7.2f us\n", lname, runp<4, 1, 1>(tabs, idx, x, out, zero));
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
        dlrm_tables_destroy(tb);
        for (int t = 0; t < T; ++t) CK(hipFree(mem[t]));
    }
    return 0;
}
