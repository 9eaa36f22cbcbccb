// Microbenchmark: where does the metric backward's time go?  A standalone replica of the step
// backward (interact_bwd_split_kernel<float, 2, 128, 4>: two waves per sample by 64-column
// halves, 4 samples per 512-thread block; lane t < 26 loads table t's index and once-hit flag;
// the packed pair gradients staged in LDS; T re-gathered (8 row loads of 4 rows x 256 B per
// wave); dT = S T on v_mfma_f32_16x16x4f32; once-hit rows updated in place, the others' dt rows
// stored), with pieces switched off:
//   MODE bit 0: MFMAs            bit 1: the output stores (dt rows / row updates / dx)
//   bit 2: the row gather (off: rows read from one L2-resident row)
// Build: hipcc -O3 --offload-arch=gfx950 -o bwd_probe tools/bwd_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <random>
#include <unordered_map>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int T = 26, F = 27, D = 128, B = 2048, W = 128 + 351 + 1, NBATCH = 16, P = 351, PMAX = 32 * 31 / 2;

struct Tabs { float* p[T]; };

template <int MODE, int SPB>
__global__ __launch_bounds__(128 * SPB, 4) void bwd(Tabs tabs, const int* __restrict__ idx, const uint8_t* __restrict__ single,
                                                    const float* __restrict__ x, const float* __restrict__ dout,
                                                    float* __restrict__ dx, float* __restrict__ dt, float lr) {
    __shared__ float pk_all[SPB][PMAX];
    __shared__ __attribute__((aligned(16))) float tt_all[2 * SPB][32 * 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int pair = w / 2, h = w % 2;
    const int c = lane & 15, q = lane >> 4;
    const int b = blockIdx.x * SPB + pair;
    const float* ob = dout + (size_t)b * W;
    float* pk = pk_all[pair];
    float* Tt = tt_all[w];
    const bool tl = lane < T;
    const int myidx = idx[(tl ? lane : 0) * B + b];
    const uint8_t myfl = single[(tl ? lane : 0) * B + b];
    float pv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int p = h * 64 + lane + 128 * k;
        pv[k] = p < P ? ob[128 + p] : 0.f;
    }
    const float xv = ob[64 * h + lane];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int p = h * 64 + lane + 128 * k;
        if (p < PMAX) pk[p] = pv[k];
    }
    __syncthreads();
    const float* rowp[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const int kk = 4 * s + q;
        const int r = __shfl(myidx, kk >= 1 ? kk - 1 : 0, 64);
        rowp[s] = (MODE & 4) ? (kk == 0 ? x + (size_t)b * D : (kk < F ? tabs.p[kk - 1] + (size_t)r * D : x))
                             : x + (size_t)b * D;
    }
    uint32_t urow[2][4];
#pragma unroll
    for (int I = 0; I < 2; ++I)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int f = I * 16 + 4 * q + r;
            const int src = (f >= 1 && f < F) ? f - 1 : 0;
            const int row = __shfl(myidx, src, 64);
            const int fl = __shfl((int)myfl, src, 64);
            urow[I][r] = (f >= 1 && f < F && fl) ? (uint32_t)row : ~0u;
        }
    const int sb = 64 * h;
    const int n0 = sb + 4 * c;
    f4 bv[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const f4 v = *(const f4*)(rowp[s] + n0);
        bv[s] = (4 * s + q < F) ? v : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int s = 0; s < 7; ++s) *(f4*)(Tt + (4 * s + q) * 64 + 4 * c) = bv[s];
    f4 acc[2][4];
#pragma unroll
    for (int I = 0; I < 2; ++I)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[I][e] = f4{0, 0, 0, 0};
    if (MODE & 1) {
#pragma unroll
        for (int s = 0; s < 7; ++s) {
            const int kk = 4 * s + q;
#pragma unroll
            for (int I = 0; I < 2; ++I) {
                const int i = I * 16 + c;
                const int hi = i > kk ? i : kk, lo = i > kk ? kk : i;
                const float av = (i != kk && hi < F) ? pk[hi * (hi - 1) / 2 + lo] : 0.0f;
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[I][e] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[s][e], acc[I][e], 0, 0, 0);
            }
        }
    } else {
#pragma unroll
        for (int s = 0; s < 7; ++s)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[s & 1][e] += bv[s];
    }
    f4 xo;
#pragma unroll
    for (int e = 0; e < 4; ++e) xo[e] = __shfl(xv, 4 * c + e, 64);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (MODE & 2) {
#pragma unroll
        for (int I = 0; I < 2; ++I)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int f = I * 16 + 4 * q + r;
                if (f < F) {
                    const f4 v = f4{acc[I][0][r], acc[I][1][r], acc[I][2][r], acc[I][3][r]};
                    if (urow[I][r] != ~0u) {
                        const f4 tw = *(const f4*)(Tt + f * 64 + 4 * c);
                        f4 wv;
#pragma unroll
                        for (int e = 0; e < 4; ++e) wv[e] = __builtin_fmaf(-lr, 0.0f + v[e], tw[e]);
                        f4* pw = (f4*)(tabs.p[f - 1] + (size_t)urow[I][r] * D + n0);
                        if (MODE & 8) __builtin_nontemporal_store(wv, pw); else *pw = wv;
                    } else {
                        f4* pd = (f4*)(dt + (size_t)b * F * D + (size_t)f * D + n0);
                        if (MODE & 16) __builtin_nontemporal_store(v, pd); else *pd = v;
                    }
                    if (f == 0) *(f4*)(dx + (size_t)b * D + n0) = xo + v;
                }
            }
    } else {
        const f4 s = acc[0][0] + acc[1][1] + acc[0][2] + acc[1][3];
        if (lane == 0) dx[(size_t)b * D + sb] = s.x + s.y + s.z + s.w;
    }
}

template <int MODE, int SPB>
double run(Tabs tabs, const int* idx, const uint8_t* single, const float* x, const float* dout, float* dx, float* dt) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int grid = B / SPB;
    auto go = [&](int i) {
        hipLaunchKernelGGL((bwd<MODE, SPB>), dim3(grid), dim3(128 * SPB), 0, 0, tabs, idx + (size_t)(i % NBATCH) * T * B,
                           single + (size_t)(i % NBATCH) * T * B, x, dout, dx, dt, 0.0f);
    };
    for (int i = 0; i < NBATCH; ++i) go(i);
    const int reps = 16 * NBATCH;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) go(i);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
}

int main() {
    static const int64_t kaggle[T] = {1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593, 3194,
                                      27, 14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105, 142572};
    float *x, *dout, *dx, *dt;
    CK(hipMalloc(&x, (size_t)B * D * 4));
    CK(hipMalloc(&dout, (size_t)B * W * 4));
    CK(hipMalloc(&dx, (size_t)B * D * 4));
    CK(hipMalloc(&dt, (size_t)B * F * D * 4));
    CK(hipMemset(x, 0, (size_t)B * D * 4));
    CK(hipMemset(dout, 0, (size_t)B * W * 4));
    int* idx;
    uint8_t* single;
    CK(hipMalloc(&idx, (size_t)NBATCH * T * B * 4));
    CK(hipMalloc(&single, (size_t)NBATCH * T * B));
    std::mt19937_64 g(1);
    Tabs tabs;
    for (int t = 0; t < T; ++t) {
        CK(hipMalloc(&tabs.p[t], kaggle[t] * D * 4));
        CK(hipMemset(tabs.p[t], 0, kaggle[t] * D * 4));
    }
    std::vector<int> h((size_t)NBATCH * T * B);
    std::vector<uint8_t> hs(h.size());
    long n1 = 0;
    for (int k = 0; k < NBATCH; ++k)
        for (int t = 0; t < T; ++t) {
            std::unordered_map<int, int> cnt;
            for (int b = 0; b < B; ++b) {
                const int r = (int)(g() % kaggle[t]);
                h[((size_t)k * T + t) * B + b] = r;
                cnt[r]++;
            }
            for (int b = 0; b < B; ++b) {
                const bool one = cnt[h[((size_t)k * T + t) * B + b]] == 1;
                hs[((size_t)k * T + t) * B + b] = one;
                n1 += one;
            }
        }
    printf("once-hit positions per batch: %.0f of %d\n", (double)n1 / NBATCH, T * B);
    CK(hipMemcpy(idx, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(single, hs.data(), hs.size(), hipMemcpyHostToDevice));
    printf("full (gather+mfma+stores) spb4 %7.2f us\n", run<7, 4>(tabs, idx, single, x, dout, dx, dt));
    printf("gather+mfma               spb4 %7.2f us\n", run<5, 4>(tabs, idx, single, x, dout, dx, dt));
    printf("gather+stores             spb4 %7.2f us\n", run<6, 4>(tabs, idx, single, x, dout, dx, dt));
    printf("gather                    spb4 %7.2f us\n", run<4, 4>(tabs, idx, single, x, dout, dx, dt));
    printf("no gather, mfma+stores    spb4 %7.2f us\n", run<3, 4>(tabs, idx, single, x, dout, dx, dt));
    printf("no gather, no mfma/stores spb4 %7.2f us\n", run<0, 4>(tabs, idx, single, x, dout, dx, dt));
    printf("full, nt row updates      spb4 %7.2f us\n", run<15, 4>(tabs, idx, single, x, dout, dx, dt));
    printf("full, nt dt               spb4 %7.2f us\n", run<23, 4>(tabs, idx, single, x, dout, dx, dt));
    printf("full, nt both             spb4 %7.2f us\n", run<31, 4>(tabs, idx, single, x, dout, dx, dt));
    printf("no gather, stores, nt both spb4 %6.2f us\n", run<26, 4>(tabs, idx, single, x, dout, dx, dt));
    printf("full                      spb2 %7.2f us\n", run<7, 2>(tabs, idx, single, x, dout, dx, dt));
    printf("full                      spb8 %7.2f us\n", run<7, 8>(tabs, idx, single, x, dout, dx, dt));
    return 0;
}
