// interact.hip — pairwise-dot feature interaction (DotInteraction) on gfx950 MFMA.
//
// Forward  = fast_vcat (src/model/interact.jl:271-281) + process_batches/process_slice!
//            (:449-467, :338-362): per sample Z = T T^T over the feature dim, then the strict
//            lower triangle in triangular_slice_kernel! order (:64-75), after x.
// Backward = process_batches_back (:469-489): S = symmetric zero-diagonal unpack of the
//            incoming gradient (:154-173), dT = S T (gemmavx!, :486), dx = dout_x + dT[0]
//            (sumavx, :434).  dT keeps the x rows, as dt_reshaped does (:428-435).
//
// One wave owns one sample.  T_b is [F][d] (F features padded to 16*NB rows), and the
// 16x16 MFMA tiles that hold the lower triangle of Z are the only ones computed:
//   fp32: v_mfma_f32_16x16x4_f32 — exact fp32 products with an fp32 fmaf chain.  Lane
//         (c = l&15, q = l>>4) loads one float4 of row 16I+c at columns u+4q..u+4q+3, and
//         component `comp` is its operand for k-step comp; since A and B of a Gram tile are
//         the same rows, one load feeds both operands of every tile pair (I, J<=I).
//   bf16: v_mfma_f32_16x16x32_bf16 — lane (c, q) holds 8 consecutive bf16 of row 16I+c at
//         columns 32u+8q.., again the same register for A and B; fp32 accumulate, one
//         rounding to bf16 on store (DotInteraction's scratchpads are Float32).
// The packed output row [x | pairs | 0-padding] is staged in LDS per wave and written
// back as one contiguous, coalesced run.
// Backward: dT (16NB x d) = S (16NB x 16NB) * T, with S built in LDS from the packed
// gradient (row stride = 16 mod 32 banks: conflict-free ds_read_b32 for the A fragments);
// B fragments are rows of T read straight from HBM (16 consecutive floats per 16 lanes).
// The interaction's arithmetic intensity (~11-24 flop/B) is far below the MFMA ridge, so
// these kernels are HBM-bound; MFMA just keeps the VALU free and the operand traffic low.
#include "common.hpp"

namespace dlrm {

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int kStage = 1024;  // floats of output staging per wave

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Writes one packed element (index e of the sample's output row).
template <typename T>
__device__ __forceinline__ void put_out(float* stage, bool staged, T* orow, int e, float v) {
    if (staged) stage[e] = v;
    else orow[e] = from_f32<T>(v);
}

template <typename T, int NB>
__device__ __forceinline__ void scatter_pairs(const f32x4_t (&acc)[NB * (NB + 1) / 2], int F, int d, int lane,
                                              float* stage, bool staged, T* orow) {
    const int c = lane & 15, q = lane >> 4;
    int ij = 0;
#pragma unroll
    for (int I = 0; I < NB; ++I)
#pragma unroll
        for (int J = 0; J <= I; ++J, ++ij) {
            const int j = J * 16 + c;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = I * 16 + 4 * q + r;
                if (i < F && j < i) put_out<T>(stage, staged, orow, d + i * (i - 1) / 2 + j, acc[ij][r]);
            }
        }
}

// ---------------------------------------------------------------------------------- fwd
template <int NB>
__global__ __launch_bounds__(256) void interact_fwd_f32(int d, int F, int B, const float* __restrict__ x,
                                                        int64_t x_ld, float* __restrict__ ys, int64_t ys_ld,
                                                        float* __restrict__ out, int64_t out_ld, int padding) {
    __shared__ float stage_all[4][kStage];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 15, q = lane >> 4;
    const int P = F * (F - 1) / 2;
    const int W = d + P + padding;
    const bool staged = W <= kStage;
    float* stage = stage_all[w];
    for (int64_t b = (int64_t)blockIdx.x * 4 + w; b < B; b += (int64_t)gridDim.x * 4) {
        const float* xb = x + b * x_ld;
        float* yb = ys + b * ys_ld;
        float* orow = out + b * out_ld;
        // fast_vcat: x into the reserved rows of ys; x is also the head of the output row.
        for (int i = lane; i < d; i += 64) {
            const float v = xb[i];
            yb[i] = v;
            put_out<float>(stage, staged, orow, i, v);
        }
        f32x4_t acc[NB * (NB + 1) / 2];
#pragma unroll
        for (int k = 0; k < NB * (NB + 1) / 2; ++k) acc[k] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        // feature 0 is read from x itself (ys rows 0..d-1 were just written by this wave)
        const float* rowp[NB];
#pragma unroll
        for (int I = 0; I < NB; ++I) {
            const int row = I * 16 + c;
            rowp[I] = row >= F ? nullptr : (row == 0 ? xb : yb + (int64_t)row * d);
        }
        for (int u = 0; u < d; u += 16) {
            const int col = u + 4 * q;
            f32x4_t a[NB];
#pragma unroll
            for (int I = 0; I < NB; ++I)
                a[I] = (rowp[I] && col < d) ? *(const f32x4_t*)(rowp[I] + col) : f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int comp = 0; comp < 4; ++comp) {
                int ij = 0;
#pragma unroll
                for (int I = 0; I < NB; ++I)
#pragma unroll
                    for (int J = 0; J <= I; ++J, ++ij)
                        acc[ij] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[I][comp], a[J][comp], acc[ij], 0, 0, 0);
            }
        }
        scatter_pairs<float, NB>(acc, F, d, lane, stage, staged, orow);
        for (int e = d + P + lane; e < W; e += 64) put_out<float>(stage, staged, orow, e, 0.0f);
        if (staged) {
            wave_lds_sync();
            for (int e = lane; e < W; e += 64) orow[e] = stage[e];
            wave_lds_sync();
        }
    }
}

template <int NB>
__global__ __launch_bounds__(256) void interact_fwd_bf16(int d, int F, int B, const uint16_t* __restrict__ x,
                                                         int64_t x_ld, uint16_t* __restrict__ ys, int64_t ys_ld,
                                                         uint16_t* __restrict__ out, int64_t out_ld, int padding) {
    __shared__ float stage_all[4][kStage];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 15, q = lane >> 4;
    const int P = F * (F - 1) / 2;
    const int W = d + P + padding;
    const bool staged = W <= kStage;
    float* stage = stage_all[w];
    for (int64_t b = (int64_t)blockIdx.x * 4 + w; b < B; b += (int64_t)gridDim.x * 4) {
        const uint16_t* xb = x + b * x_ld;
        uint16_t* yb = ys + b * ys_ld;
        uint16_t* orow = out + b * out_ld;
        for (int i = lane; i < d; i += 64) {
            const uint16_t v = xb[i];
            yb[i] = v;
            if (staged) stage[i] = bf16_to_f32(v);
            else orow[i] = v;
        }
        f32x4_t acc[NB * (NB + 1) / 2];
#pragma unroll
        for (int k = 0; k < NB * (NB + 1) / 2; ++k) acc[k] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const uint16_t* rowp[NB];
#pragma unroll
        for (int I = 0; I < NB; ++I) {
            const int row = I * 16 + c;
            rowp[I] = row >= F ? nullptr : (row == 0 ? xb : yb + (int64_t)row * d);
        }
        for (int u = 0; u < d; u += 32) {
            const int col = u + 8 * q;
            bf16x8_t a[NB];
#pragma unroll
            for (int I = 0; I < NB; ++I) {
                if (rowp[I] && col < d) a[I] = *(const bf16x8_t*)(rowp[I] + col);
                else a[I] = bf16x8_t{};
            }
            int ij = 0;
#pragma unroll
            for (int I = 0; I < NB; ++I)
#pragma unroll
                for (int J = 0; J <= I; ++J, ++ij)
                    acc[ij] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[I], a[J], acc[ij], 0, 0, 0);
        }
        // stage holds fp32 values; the final store rounds once to bf16
        int ij = 0;
#pragma unroll
        for (int I = 0; I < NB; ++I)
#pragma unroll
            for (int J = 0; J <= I; ++J, ++ij) {
                const int j = J * 16 + c;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = I * 16 + 4 * q + r;
                    if (i < F && j < i) {
                        const int e = d + i * (i - 1) / 2 + j;
                        if (staged) stage[e] = acc[ij][r];
                        else orow[e] = f32_to_bf16(acc[ij][r]);
                    }
                }
            }
        for (int e = d + P + lane; e < W; e += 64) {
            if (staged) stage[e] = 0.0f;
            else orow[e] = 0;
        }
        if (staged) {
            wave_lds_sync();
            for (int e = lane; e < W; e += 64) orow[e] = f32_to_bf16(stage[e]);
            wave_lds_sync();
        }
    }
}

// ---------------------------------------------------------------------------------- bwd
template <int NB> struct BwdGeom {
    static constexpr int NS = 16 * NB;                          // padded features
    static constexpr int SS = NS + ((NB % 2 == 0) ? 16 : 0);    // row stride = 16 (mod 32)
    static constexpr int WPB = NB <= 2 ? 4 : (NB <= 4 ? 2 : 1); // waves per block
    static constexpr int LDS_FLOATS = NS * SS;                  // per wave
};

template <typename T, int NB>
__global__ __launch_bounds__(256) void interact_bwd_kernel(int d, int F, int B, const T* __restrict__ dout,
                                                           int64_t dout_ld, const T* __restrict__ t, int64_t t_ld,
                                                           float* __restrict__ dx, int64_t dx_ld,
                                                           float* __restrict__ dt, int64_t dt_ld) {
    typedef BwdGeom<NB> G;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (w >= G::WPB) return;
    const int c = lane & 15, q = lane >> 4;
    float* S = smem + w * G::LDS_FLOATS;
    const int P = F * (F - 1) / 2;
    const int ksteps = (F + 3) / 4;
    for (int64_t b = (int64_t)blockIdx.x * G::WPB + w; b < B; b += (int64_t)gridDim.x * G::WPB) {
        const T* ob = dout + b * dout_ld;
        const T* tb = t + b * t_ld;
        // S: zero, then scatter the packed pairs to both triangles (fused unpack + transpose-add)
        for (int e = lane; e < G::NS * G::NS; e += 64) S[(e / G::NS) * G::SS + (e % G::NS)] = 0.0f;
        wave_lds_sync();
        for (int p = lane; p < P; p += 64) {
            int i = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)p)) * 0.5f);
            while (i * (i - 1) / 2 > p) --i;
            while ((i + 1) * i / 2 <= p) ++i;
            const int j = p - i * (i - 1) / 2;
            const float v = to_f32(ob[d + p]);
            S[i * G::SS + j] = v;
            S[j * G::SS + i] = v;
        }
        wave_lds_sync();
        for (int nb = 0; nb < d; nb += 16) {
            const int n = nb + c;
            f32x4_t acc[NB];
#pragma unroll
            for (int I = 0; I < NB; ++I) acc[I] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            for (int s = 0; s < ksteps; ++s) {
                const int kk = 4 * s + q;
                const float bv = (kk < F && n < d) ? to_f32(tb[(int64_t)kk * d + n]) : 0.0f;
#pragma unroll
                for (int I = 0; I < NB; ++I) {
                    const float av = S[kk * G::SS + I * 16 + c];  // = S[16I+c][kk] (symmetric)
                    acc[I] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[I], 0, 0, 0);
                }
            }
            if (n < d) {
#pragma unroll
                for (int I = 0; I < NB; ++I)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int f = I * 16 + 4 * q + r;
                        if (f < F) {
                            dt[b * dt_ld + (int64_t)f * d + n] = acc[I][r];
                            if (f == 0) dx[b * dx_ld + n] = to_f32(ob[n]) + acc[I][r];
                        }
                    }
            }
        }
        wave_lds_sync();
    }
}

// ------------------------------------------------------------------ scalar fallbacks
template <typename T>
__global__ __launch_bounds__(256) void interact_fwd_scalar(int d, int F, int B, const T* __restrict__ x, int64_t x_ld,
                                                           T* __restrict__ ys, int64_t ys_ld, T* __restrict__ out,
                                                           int64_t out_ld, int padding) {
    const int P = F * (F - 1) / 2;
    const int W = d + P + padding;
    const int64_t total = (int64_t)B * W;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = e / W;
        const int k = (int)(e % W);
        const T* xb = x + b * x_ld;
        if (k < d) {
            ys[b * ys_ld + k] = xb[k];
            out[b * out_ld + k] = xb[k];
        } else if (k < d + P) {
            const int p = k - d;
            int i = 1;
            while ((i + 1) * i / 2 <= p) ++i;
            const int j = p - i * (i - 1) / 2;
            const T* ri = i == 0 ? xb : ys + b * ys_ld + (int64_t)i * d;
            const T* rj = j == 0 ? xb : ys + b * ys_ld + (int64_t)j * d;
            float z = 0.0f;
            for (int cc = 0; cc < d; ++cc) z = fmaf(to_f32(ri[cc]), to_f32(rj[cc]), z);
            out[b * out_ld + k] = from_f32<T>(z);
        } else {
            out[b * out_ld + k] = from_f32<T>(0.0f);
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void interact_bwd_scalar(int d, int F, int B, const T* __restrict__ dout,
                                                           int64_t dout_ld, const T* __restrict__ t, int64_t t_ld,
                                                           float* __restrict__ dx, int64_t dx_ld,
                                                           float* __restrict__ dt, int64_t dt_ld) {
    const int64_t total = (int64_t)B * F * d;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = e / ((int64_t)F * d);
        const int rem = (int)(e % ((int64_t)F * d));
        const int f = rem / d, n = rem % d;
        const T* ob = dout + b * dout_ld + d;
        float acc = 0.0f;
        for (int j = 0; j < F; ++j) {
            if (j == f) continue;
            const int hi = j > f ? j : f, lo = j > f ? f : j;
            acc = fmaf(to_f32(t[b * t_ld + (int64_t)j * d + n]), to_f32(ob[hi * (hi - 1) / 2 + lo]), acc);
        }
        dt[b * dt_ld + (int64_t)f * d + n] = acc;
        if (f == 0) dx[b * dx_ld + n] = to_f32(dout[b * dout_ld + n]) + acc;
    }
}

// ------------------------------------------------------------------------ launchers
static unsigned grid_for(int64_t items, int per_block, int cus) {
    int64_t g = (items + per_block - 1) / per_block;
    const int64_t cap = (int64_t)cus * 16;
    if (g > cap) g = cap;
    return (unsigned)(g < 1 ? 1 : g);
}

template <int NB>
static void launch_fwd_nb(hipStream_t s, int cus, int dtype, int d, int F, int B, const void* x, int64_t x_ld,
                          void* ys, int64_t ys_ld, void* out, int64_t out_ld, int padding) {
    const unsigned g = grid_for(B, 4, cus);
    if (dtype == DLRM_F32)
        hipLaunchKernelGGL(interact_fwd_f32<NB>, dim3(g), dim3(256), 0, s, d, F, B, (const float*)x, x_ld,
                           (float*)ys, ys_ld, (float*)out, out_ld, padding);
    else
        hipLaunchKernelGGL(interact_fwd_bf16<NB>, dim3(g), dim3(256), 0, s, d, F, B, (const uint16_t*)x, x_ld,
                           (uint16_t*)ys, ys_ld, (uint16_t*)out, out_ld, padding);
}

template <typename T, int NB>
static void launch_bwd_nb(hipStream_t s, int cus, int d, int F, int B, const void* dout, int64_t dout_ld,
                          const void* t, int64_t t_ld, float* dx, int64_t dx_ld, float* dt, int64_t dt_ld) {
    typedef BwdGeom<NB> G;
    const unsigned g = grid_for(B, G::WPB, cus);
    const size_t lds = sizeof(float) * G::LDS_FLOATS * G::WPB;
    hipLaunchKernelGGL((interact_bwd_kernel<T, NB>), dim3(g), dim3(64 * G::WPB), lds, s, d, F, B, (const T*)dout,
                       dout_ld, (const T*)t, t_ld, dx, dx_ld, dt, dt_ld);
}

int launch_interact_fwd(dlrm_ctx* ctx, int dtype, int d, int F, int B, const void* x, int64_t x_ld, void* ys,
                        int64_t ys_ld, void* out, int64_t out_ld, int padding) {
    if (B == 0) return DLRM_OK;
    hipStream_t s = ctx_stream(ctx);
    const int cus = ctx_num_cus(ctx);
    const int esz = dtype == DLRM_F32 ? 4 : 2;
    const int vec = 16 / esz;
    const bool aligned = (uintptr_t)x % 16 == 0 && (uintptr_t)ys % 16 == 0 && (x_ld % vec) == 0 &&
                         (ys_ld % vec) == 0 && (d % vec) == 0;
    const int NB = (F + 15) / 16;
    if (aligned && NB >= 1 && NB <= 6) {  // NB 7-8 exceed 256 VGPRs: scalar path
        switch (NB) {
            case 1: launch_fwd_nb<1>(s, cus, dtype, d, F, B, x, x_ld, ys, ys_ld, out, out_ld, padding); break;
            case 2: launch_fwd_nb<2>(s, cus, dtype, d, F, B, x, x_ld, ys, ys_ld, out, out_ld, padding); break;
            case 3: launch_fwd_nb<3>(s, cus, dtype, d, F, B, x, x_ld, ys, ys_ld, out, out_ld, padding); break;
            case 4: launch_fwd_nb<4>(s, cus, dtype, d, F, B, x, x_ld, ys, ys_ld, out, out_ld, padding); break;
            case 5: launch_fwd_nb<5>(s, cus, dtype, d, F, B, x, x_ld, ys, ys_ld, out, out_ld, padding); break;
            case 6: launch_fwd_nb<6>(s, cus, dtype, d, F, B, x, x_ld, ys, ys_ld, out, out_ld, padding); break;
        }
    } else {
        const int W = d + F * (F - 1) / 2 + padding;
        const unsigned g = grid_for((int64_t)B * W, 256, cus);
        if (dtype == DLRM_F32)
            hipLaunchKernelGGL(interact_fwd_scalar<float>, dim3(g), dim3(256), 0, s, d, F, B, (const float*)x, x_ld,
                               (float*)ys, ys_ld, (float*)out, out_ld, padding);
        else
            hipLaunchKernelGGL(interact_fwd_scalar<uint16_t>, dim3(g), dim3(256), 0, s, d, F, B, (const uint16_t*)x,
                               x_ld, (uint16_t*)ys, ys_ld, (uint16_t*)out, out_ld, padding);
    }
    return ctx_hip(ctx, hipGetLastError(), "interact_fwd launch");
}

template <typename T>
static void dispatch_bwd(int NB, hipStream_t s, int cus, int d, int F, int B, const void* dout, int64_t dout_ld,
                         const void* t, int64_t t_ld, float* dx, int64_t dx_ld, float* dt, int64_t dt_ld) {
    switch (NB) {
        case 1: launch_bwd_nb<T, 1>(s, cus, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld); break;
        case 2: launch_bwd_nb<T, 2>(s, cus, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld); break;
        case 3: launch_bwd_nb<T, 3>(s, cus, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld); break;
        case 4: launch_bwd_nb<T, 4>(s, cus, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld); break;
        case 5: launch_bwd_nb<T, 5>(s, cus, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld); break;
        case 6: launch_bwd_nb<T, 6>(s, cus, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld); break;
        case 7: launch_bwd_nb<T, 7>(s, cus, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld); break;
    }
}

int launch_interact_bwd(dlrm_ctx* ctx, int dtype, int d, int F, int B, const void* dout, int64_t dout_ld,
                        const void* t, int64_t t_ld, float* dx, int64_t dx_ld, float* dt, int64_t dt_ld) {
    if (B == 0) return DLRM_OK;
    hipStream_t s = ctx_stream(ctx);
    const int cus = ctx_num_cus(ctx);
    const int NB = (F + 15) / 16;
    if (NB >= 1 && NB <= 7) {  // NB = 8 would need > 64 KB of dynamic LDS
        if (dtype == DLRM_F32) dispatch_bwd<float>(NB, s, cus, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld);
        else dispatch_bwd<uint16_t>(NB, s, cus, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld);
    } else {
        const unsigned g = grid_for((int64_t)B * F * d, 256, cus);
        if (dtype == DLRM_F32)
            hipLaunchKernelGGL(interact_bwd_scalar<float>, dim3(g), dim3(256), 0, s, d, F, B, (const float*)dout,
                               dout_ld, (const float*)t, t_ld, dx, dx_ld, dt, dt_ld);
        else
            hipLaunchKernelGGL(interact_bwd_scalar<uint16_t>, dim3(g), dim3(256), 0, s, d, F, B,
                               (const uint16_t*)dout, dout_ld, (const uint16_t*)t, t_ld, dx, dx_ld, dt, dt_ld);
    }
    return ctx_hip(ctx, hipGetLastError(), "interact_bwd launch");
}

}  // namespace dlrm
