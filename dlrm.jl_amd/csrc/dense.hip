// dense.hip — the elementwise + column-reduction seams of the dense MLPs around the hot path
// (SURVEY §8 row f1).  The MLP GEMMs stay on hipBLASLt; these kernels replace the chains of
// small launches between them:
//   bce_head_kernel      sigmoid -> bce_loss -> rrule(bce_loss) -> sigmoid pullback -> Σ over the
//                        batch (the last layer's bias gradient): train.jl:33-64, model.jl:83-89
//   relu_bwd_bias_kernel relu pullback (g .* (y .> 0)) fused with the bias gradient Σ_b g[b, :]
//                        (Flux Dense pullback, model.jl:72-93)
// Both reduce in a fixed order (deterministic: replaying a step gives the same bits).
#include <stdlib.h>

#include "common.hpp"

namespace dlrm {

constexpr int kHeadThreads = 1024;

// One workgroup: B logits -> prob, dLoss/dlogit, loss (mean), Σ dlogit.
__global__ void __launch_bounds__(kHeadThreads)
bce_head_kernel(int B, const float* __restrict__ z, int64_t z_ld, const float* __restrict__ y,
                float* __restrict__ prob, float* __restrict__ dz, float* __restrict__ loss, float* __restrict__ dbias) {
    __shared__ float sl[kHeadThreads / kWave], sg[kHeadThreads / kWave];
    const float eps = 1.1920929e-7f;  // eps(Float32), train.jl:51
    const float inv = 1.0f / (float)B;
    float l = 0.0f, g = 0.0f;
    for (int i = threadIdx.x; i < B; i += kHeadThreads) {
        const float zi = z[(int64_t)i * z_ld], yi = y[i];
        const float p = 1.0f / (1.0f + __expf(-zi));  // Flux.sigmoid in float32
        l += -yi * fmaxf(__logf(p), -100.0f) + (yi - 1.0f) * fmaxf(__logf(1.0f - p), -100.0f);
        const float dp = inv * ((1.0f - yi) / (1.0f - p + eps) - yi / (p + eps));
        const float d = dp * p * (1.0f - p);
        prob[i] = p;
        dz[i] = d;
        g += d;
    }
    // wave sums (fixed butterfly order), then the 16 wave partials in wave order
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        l += __shfl_xor(l, o);
        g += __shfl_xor(g, o);
    }
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) {
        sl[w] = l;
        sg[w] = g;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float L = 0.0f, G = 0.0f;
        for (int k = 0; k < kHeadThreads / kWave; ++k) {
            L += sl[k];
            G += sg[k];
        }
        loss[0] = L * inv;
        if (dbias) dbias[0] = G;
    }
}

constexpr int kReluThreads = 256;  // 4 waves; a lane owns 4 consecutive columns
constexpr int kReluWaveRows = 4;  // rows per wave (grid: B/16 row chunks, enough workgroups to fill the chip)
constexpr int kReluRows = kReluWaveRows * (kReluThreads / kWave);  // rows per workgroup

// Cross-workgroup hand-off without agent-scope fences (a release fence writes back the whole L2,
// which here holds the just-written g): partials stored write-through with agent-scope atomic
// stores (sc1), drained (vmcnt(0)) before the barrier, read back with agent-scope atomic loads
// (the same protocol as update.hip's hot-segment combine, cdna_hip_programming.md Guideline 16).
typedef __attribute__((address_space(1))) unsigned long long dense_gu64_t;

__device__ __forceinline__ void dense_store_wt(float* p, const float4& v) {
    const unsigned long long lo = ((unsigned long long)__float_as_uint(v.y) << 32) | __float_as_uint(v.x);
    const unsigned long long hi = ((unsigned long long)__float_as_uint(v.w) << 32) | __float_as_uint(v.z);
    __hip_atomic_store((dense_gu64_t*)p, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((dense_gu64_t*)(p + 2), hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float4 dense_load_wt(const float* p) {
    const unsigned long long lo = __hip_atomic_load((dense_gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long hi = __hip_atomic_load((dense_gu64_t*)(p + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_float4(__uint_as_float((uint32_t)lo), __uint_as_float((uint32_t)(lo >> 32)),
                       __uint_as_float((uint32_t)hi), __uint_as_float((uint32_t)(hi >> 32)));
}

__device__ __forceinline__ void add4(float4& a, const float4& b) {
    a.x += b.x;
    a.y += b.y;
    a.z += b.z;
    a.w += b.w;
}

// g[b][:] *= (y[b][:] > 0) in place; gb[n] = Σ_b g[b][n].  Grid (ceil(N/256), ceil(B/16)); each
// workgroup writes its 16-row column sums to part[chunk][N] (write-through), and the last workgroup
// of a column group to arrive (agent-scope counter, reset by it for the next launch) adds the chunks: wave w
// takes chunks w, w+4, ... (loads in flight together), then the 4 wave sums in wave order.
__global__ void __launch_bounds__(kReluThreads)
relu_bwd_bias_kernel(int B, int N, const float* __restrict__ yv, int64_t y_ld, float* __restrict__ g, int64_t g_ld,
                     float* __restrict__ gb, float* __restrict__ part, unsigned* __restrict__ counters) {
    __shared__ float4 sacc[kReluThreads / kWave][kWave];
    __shared__ bool last;
    constexpr int U = 4;
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const int c = (blockIdx.x * kWave + lane) * 4;
    const bool col_ok = c < N;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const int r0 = blockIdx.y * kReluRows + w * kReluWaveRows;
    if (col_ok) {
        for (int k0 = 0; k0 < kReluWaveRows; k0 += U) {
            float4 gg[U], yy[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int r = min(r0 + k0 + u, B - 1);
                gg[u] = ldg<float4>(g + (int64_t)r * g_ld + c);
                yy[u] = ldg<float4>(yv + (int64_t)r * y_ld + c);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int r = r0 + k0 + u;
                if (r < B) {
                    gg[u].x = yy[u].x > 0.f ? gg[u].x : 0.f;
                    gg[u].y = yy[u].y > 0.f ? gg[u].y : 0.f;
                    gg[u].z = yy[u].z > 0.f ? gg[u].z : 0.f;
                    gg[u].w = yy[u].w > 0.f ? gg[u].w : 0.f;
                    stg<float4>(g + (int64_t)r * g_ld + c, gg[u]);
                    add4(acc, gg[u]);
                }
            }
        }
    }
    sacc[w][lane] = acc;
    __syncthreads();
    if (w == 0) {
#pragma unroll
        for (int k = 1; k < kReluThreads / kWave; ++k) add4(acc, sacc[k][lane]);
        if (col_ok) dense_store_wt(part + (int64_t)blockIdx.y * N + c, acc);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned n = __hip_atomic_fetch_add(counters + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = n == gridDim.y - 1;
        if (last) __hip_atomic_store(counters + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
    const int nch = (int)gridDim.y;
    constexpr int NW = kReluThreads / kWave, UC = 8;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (col_ok) {
        for (int k0 = w; k0 < nch; k0 += NW * UC) {
            float4 a[UC];
#pragma unroll
            for (int u = 0; u < UC; ++u) {
                const int k = min(k0 + u * NW, nch - 1);
                a[u] = dense_load_wt(part + (int64_t)k * N + c);
            }
#pragma unroll
            for (int u = 0; u < UC; ++u)
                if (k0 + u * NW < nch) add4(s, a[u]);
        }
    }
    __syncthreads();  // sacc reuse
    sacc[w][lane] = s;
    __syncthreads();
    if (w == 0 && col_ok) {
#pragma unroll
        for (int k = 1; k < NW; ++k) add4(s, sacc[k][lane]);
        stg<float4>(gb + c, s);
    }
}

// Two-launch form of the same seam (the default; DLRM_RELU_2PASS=0 selects the one-launch form above): launch A masks
// g and writes the 16-row column sums to part[chunk][N] with plain stores; launch B (after the
// kernel boundary: no fences, no counters) sums the chunks per column in chunk order.
__global__ void __launch_bounds__(kReluThreads)
relu_mask_partial_kernel(int B, int N, const float* __restrict__ yv, int64_t y_ld, float* __restrict__ g,
                         int64_t g_ld, float* __restrict__ part) {
    __shared__ float4 sacc[kReluThreads / kWave][kWave];
    constexpr int U = 4;
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const int c = (blockIdx.x * kWave + lane) * 4;
    const bool col_ok = c < N;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const int r0 = blockIdx.y * kReluRows + w * kReluWaveRows;
    if (col_ok) {
        for (int k0 = 0; k0 < kReluWaveRows; k0 += U) {
            float4 gg[U], yy[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int r = min(r0 + k0 + u, B - 1);
                gg[u] = ldg<float4>(g + (int64_t)r * g_ld + c);
                yy[u] = ldg<float4>(yv + (int64_t)r * y_ld + c);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int r = r0 + k0 + u;
                if (r < B) {
                    gg[u].x = yy[u].x > 0.f ? gg[u].x : 0.f;
                    gg[u].y = yy[u].y > 0.f ? gg[u].y : 0.f;
                    gg[u].z = yy[u].z > 0.f ? gg[u].z : 0.f;
                    gg[u].w = yy[u].w > 0.f ? gg[u].w : 0.f;
                    stg<float4>(g + (int64_t)r * g_ld + c, gg[u]);
                    add4(acc, gg[u]);
                }
            }
        }
    }
    sacc[w][lane] = acc;
    __syncthreads();
    if (w == 0) {
#pragma unroll
        for (int k = 1; k < kReluThreads / kWave; ++k) add4(acc, sacc[k][lane]);
        if (col_ok) stg<float4>(part + (int64_t)blockIdx.y * N + c, acc);
    }
}

// 64 columns per workgroup: 16 column lanes (float4) x 16 chunk lanes; chunk lane q sums chunks
// q, q+16, ... (8 loads in flight), then lane q = 0 adds the 16 partial sums in q order.
__global__ void __launch_bounds__(256)
colsum_chunks_kernel(int nch, int N, const float* __restrict__ part, float* __restrict__ gb) {
    __shared__ float4 s[16][16];
    constexpr int UC = 8;
    const int cq = threadIdx.x & 15, q = threadIdx.x >> 4;
    const int c = blockIdx.x * 64 + cq * 4;
    const bool col_ok = c < N;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (col_ok) {
        for (int k0 = q; k0 < nch; k0 += 16 * UC) {
            float4 a[UC];
#pragma unroll
            for (int u = 0; u < UC; ++u) a[u] = ldg<float4>(part + (int64_t)min(k0 + u * 16, nch - 1) * N + c);
#pragma unroll
            for (int u = 0; u < UC; ++u)
                if (k0 + u * 16 < nch) add4(acc, a[u]);
        }
    }
    s[q][cq] = acc;
    __syncthreads();
    if (q == 0 && col_ok) {
#pragma unroll
        for (int k = 1; k < 16; ++k) add4(acc, s[k][cq]);
        stg<float4>(gb + c, acc);
    }
}

int launch_bce_head(dlrm_ctx* ctx, int B, const float* z, int64_t z_ld, const float* y, float* prob, float* dz,
                    float* loss, float* dbias) {
    hipLaunchKernelGGL(bce_head_kernel, dim3(1), dim3(kHeadThreads), 0, ctx_stream(ctx), B, z, z_ld, y, prob, dz, loss,
                       dbias);
    return ctx_hip(ctx, hipGetLastError(), "bce_head launch");
}

int64_t relu_bwd_chunks(int B) { return (B + kReluRows - 1) / kReluRows; }
int64_t relu_bwd_groups(int N) { return (N + kWave * 4 - 1) / (kWave * 4); }

int launch_relu_bwd_bias(dlrm_ctx* ctx, int B, int N, const float* y, int64_t y_ld, float* g, int64_t g_ld, float* gb,
                         float* part, unsigned* counters) {
    if (B == 0 || N == 0) return DLRM_OK;
    const dim3 grid((unsigned)relu_bwd_groups(N), (unsigned)relu_bwd_chunks(B));
    // default: the two-launch form (full step 483 vs 504-509 us with the last-arriver form on MI355X);
    // DLRM_RELU_2PASS=0 selects the one-launch last-arriver form
    const bool two_pass = !knobs().relu_1pass;
    if (two_pass) {
        hipLaunchKernelGGL(relu_mask_partial_kernel, grid, dim3(kReluThreads), 0, ctx_stream(ctx), B, N, y, y_ld, g,
                           g_ld, part);
        hipLaunchKernelGGL(colsum_chunks_kernel, dim3((unsigned)((N + 63) / 64)), dim3(256), 0, ctx_stream(ctx),
                           (int)relu_bwd_chunks(B), N, (const float*)part, gb);
        return ctx_hip(ctx, hipGetLastError(), "relu_bwd_bias (two-pass) launch");
    }
    hipLaunchKernelGGL(relu_bwd_bias_kernel, grid, dim3(kReluThreads), 0, ctx_stream(ctx), B, N, y, y_ld, g, g_ld, gb,
                       part, counters);
    return ctx_hip(ctx, hipGetLastError(), "relu_bwd_bias launch");
}

}  // namespace dlrm
