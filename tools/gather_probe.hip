// Microbenchmark: read-only gather of random 512-B rows (fp32, D = 128) from a 16 GiB table,
// 53248 rows per launch (Kaggle: 2048 samples x 26 tables), with different per-instruction
// load shapes.  Answers: does the MFMA-operand layout the fused kernels load in (16 rows x 64 B
// per instruction) cost gather bandwidth against full-line (8 rows x 128 B) or full-row
// (2 rows x 512 B) instructions?  Build: hipcc -O3 --offload-arch=gfx950 -o gather_probe gather_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// SHAPE: rows touched per instruction = 64 / (lanes per row); each instruction reads 16 B per lane.
// LPR = lanes per row (4: 64 B, 8: 128 B, 32: 512 B).  RPW rows per wave (all loads in flight).
template <int LPR, int RPW, bool NT>
__global__ __launch_bounds__(256) void gather(const float* __restrict__ tab, const int* __restrict__ idx, int n,
                                              float* __restrict__ out) {
    constexpr int RPI = 64 / LPR;             // rows per instruction
    constexpr int CPI = LPR * 4;              // columns per instruction per row
    constexpr int NI = (RPW / RPI) * (128 / CPI);  // instructions per wave
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int r0 = wave * RPW;
    if (r0 >= n) return;
    int rl, cl;
    if (LPR == 4) { rl = lane & 15; cl = (lane >> 4) * 4; }   // the fused kernels' (c, q) layout
    else { rl = lane / LPR; cl = (lane % LPR) * 4; }
    int64_t rows[RPW / RPI];
#pragma unroll
    for (int g = 0; g < RPW / RPI; ++g) {
        const int r = r0 + g * RPI + rl;
        rows[g] = r < n ? idx[r] : 0;
    }
    f4 v[NI];
#pragma unroll
    for (int g = 0; g < RPW / RPI; ++g)
#pragma unroll
        for (int u = 0; u < 128 / CPI; ++u) {
            const f4* p = (const f4*)(tab + rows[g] * 128 + u * CPI + cl);
            v[g * (128 / CPI) + u] = NT ? __builtin_nontemporal_load(p) : *p;
        }
    f4 s = v[0];
#pragma unroll
    for (int i = 1; i < NI; ++i) s += v[i];
    out[(size_t)wave * 64 + lane] = s.x + s.y + s.z + s.w;
}

template <int LPR, int RPW, bool NT>
void run(const char* name, const float* tab, const int* idx, int n, float* out, int wpb) {
    const int waves = (n + RPW - 1) / RPW;
    const int blocks = (waves + wpb - 1) / wpb;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((gather<LPR, RPW, NT>), dim3(blocks), dim3(64 * wpb), 0, 0, tab, idx, n, out);
    const int reps = 50;
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((gather<LPR, RPW, NT>), dim3(blocks), dim3(64 * wpb), 0, 0, tab, idx + (size_t)(i % 16) * n, n, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / reps;
    printf("%-34s wpb %2d  waves %5d  %7.2f us  %7.0f GB/s (rows read)\n", name, wpb, waves, us,
           (double)n * 512 / (us * 1e3));
}

int main(int argc, char** argv) {
    const int64_t rows = argc > 1 ? atoll(argv[1]) : (int64_t)1 << 25;  // 16 GiB of fp32 x 128
    const int n = 53248;
    float* tab; int* idx; float* out;
    CK(hipMalloc(&tab, rows * 512));
    CK(hipMemset(tab, 0, rows * 512));
    std::vector<int> h((size_t)n * 16);
    std::mt19937_64 g(1);
    for (auto& x : h) x = (int)(g() % rows);
    CK(hipMalloc(&idx, h.size() * 4));
    CK(hipMemcpy(idx, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&out, (size_t)n * 64 * 4));
    printf("table %.2f GiB, %d random rows per launch, 16 index sets rotated\n", rows * 512.0 / (1 << 30), n);
    for (int wpb : {1, 4}) {
        run<4, 16, false>("16 rows x 64 B/instr, 16 rows/wave", tab, idx, n, out, wpb);
        run<4, 32, false>("16 rows x 64 B/instr, 32 rows/wave", tab, idx, n, out, wpb);
        run<8, 16, false>(" 8 rows x 128 B/instr, 16 rows/wave", tab, idx, n, out, wpb);
        run<8, 32, false>(" 8 rows x 128 B/instr, 32 rows/wave", tab, idx, n, out, wpb);
        run<32, 16, false>(" 2 rows x 512 B/instr, 16 rows/wave", tab, idx, n, out, wpb);
        run<32, 32, false>(" 2 rows x 512 B/instr, 32 rows/wave", tab, idx, n, out, wpb);
        run<32, 8, false>(" 2 rows x 512 B/instr,  8 rows/wave", tab, idx, n, out, wpb);
        run<4, 16, true>("16 rows x 64 B/instr, 16/wave, nt", tab, idx, n, out, wpb);
        run<32, 16, true>(" 2 rows x 512 B/instr, 16/wave, nt", tab, idx, n, out, wpb);
    }
    CK(hipFree(tab)); CK(hipFree(idx)); CK(hipFree(out));
    return 0;
}
