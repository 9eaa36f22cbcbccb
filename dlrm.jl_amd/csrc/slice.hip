// slice.hip — the operators of the reference's "Implementation 2" interaction on gfx950.
//
// DLRM.jl's default model builder (dlrm(), src/model/model.jl:180) interacts through
// dot_interaction (src/model/interact.jl:503-517): fast_vcat, then self_batched_mul (OneDNN
// batched matmul, :526-537) for the full Gram Z_b = T_b^T T_b, then triangular_slice (:176-191)
// for its strict triangle.  Their rrules are triangular_slice_back (:193-203, :205-215: the
// upper triangle of Z's cotangent, zeros elsewhere) and self_batched_mul_back (:539-551:
// dT = T (Δ + Δ^T)).  dlrm_interact_fwd / dlrm_interact_bwd compute the composition in one
// launch each; these kernels are the pieces, for callers that compose them as the reference
// does (they are not on the benchmark's path).
//
// Layouts (Julia column-major -> C row-major): Z / Δ (sz, sz, B) = C [B][sz][sz] with
// element [b][col][row]; the slice (ncols, B) = C [B][ld]; T (d, F, B) = C [B][F][d].
// Pair p = col(col-1)/2 + row for row < col (triangular_slice_kernel!, :64-75).
//
// self_batched_mul and its pullback: one workgroup per sample, T staged through LDS in
// 64-column chunks, fp32 accumulation in ascending column order (fmaf).  They are small
// HBM-bound contractions (2·F²·d flop per sample against (F·d + F²)·E bytes), so VALU
// FMAs from LDS keep pace with the loads; MFMA would not change the bound.
#include "common.hpp"

namespace dlrm {

constexpr int kSliceChunk = 64;    // columns of T staged per pass
constexpr int kGramAcc = 16;       // Gram entries per thread (F(F+1)/2 <= 256 * 16)

// (col, row), row < col, of pair p
__device__ __forceinline__ void pair_of(int p, int& col, int& row) {
    int c = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)p)) * 0.5f);
    while (c * (c - 1) / 2 > p) --c;
    while ((c + 1) * c / 2 <= p) ++c;
    col = c;
    row = p - c * (c - 1) / 2;
}

// (i, j), j <= i, of the lower-triangle-with-diagonal index q = i(i+1)/2 + j
__device__ __forceinline__ void lower_of(int q, int& i, int& j) {
    int r = (int)((sqrtf(8.0f * (float)q + 1.0f) - 1.0f) * 0.5f);
    while (r * (r + 1) / 2 > q) --r;
    while ((r + 1) * (r + 2) / 2 <= q) ++r;
    i = r;
    j = q - r * (r + 1) / 2;
}

template <typename T>
__global__ __launch_bounds__(256) void triangular_slice_kernel(int sz, int B, const T* __restrict__ z, int64_t z_bs,
                                                               T* __restrict__ out, int64_t out_ld) {
    const int P = sz * (sz - 1) / 2;
    const int64_t total = (int64_t)B * P;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = e / P;
        const int p = (int)(e - b * P);
        int col, row;
        pair_of(p, col, row);
        out[b * out_ld + p] = z[b * z_bs + (int64_t)col * sz + row];
    }
}

// sym = 0: triangular_slice_back_kernel! (:104-120), upper triangle only;
// sym = 1: triangular_slice_back_fuse_add_transpose_kernel! (:150-171), symmetric, zero diagonal.
template <typename T>
__global__ __launch_bounds__(256) void triangular_slice_back_kernel(int sz, int B, const T* __restrict__ dy,
                                                                    int64_t dy_ld, T* __restrict__ a, int64_t a_bs,
                                                                    int sym) {
    const int64_t per = (int64_t)sz * sz;
    const int64_t total = (int64_t)B * per;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = e / per;
        const int k = (int)(e - b * per);
        const int col = k / sz, row = k % sz;  // element [b][col][row] = Julia a[row, col, b]
        T v = from_f32<T>(0.0f);
        if (row < col) v = dy[b * dy_ld + col * (col - 1) / 2 + row];
        else if (sym && row > col) v = dy[b * dy_ld + row * (row - 1) / 2 + col];
        a[b * a_bs + k] = v;
    }
}

// Z_b[i][j] = sum_n T_b[i][n] T_b[j][n] (full F x F, symmetric), stored in T's dtype.
template <typename T>
__global__ __launch_bounds__(256) void self_batched_mul_kernel(int d, int F, int B, const T* __restrict__ t,
                                                               int64_t t_ld, T* __restrict__ z, int64_t z_bs) {
    __shared__ float ts[90 * kSliceChunk];
    const int npairs = F * (F + 1) / 2;
    for (int b = blockIdx.x; b < B; b += gridDim.x) {
        const T* tb = t + (int64_t)b * t_ld;
        float acc[kGramAcc];
#pragma unroll
        for (int k = 0; k < kGramAcc; ++k) acc[k] = 0.0f;
        for (int n0 = 0; n0 < d; n0 += kSliceChunk) {
            const int nc = min(kSliceChunk, d - n0);
            __syncthreads();
            for (int e = threadIdx.x; e < F * nc; e += blockDim.x) {
                const int f = e / nc, n = e % nc;
                ts[f * kSliceChunk + n] = to_f32(tb[(int64_t)f * d + n0 + n]);
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kGramAcc; ++k) {
                const int q = threadIdx.x + k * 256;
                if (q < npairs) {
                    int i, j;
                    lower_of(q, i, j);
                    const float* ri = ts + i * kSliceChunk;
                    const float* rj = ts + j * kSliceChunk;
                    float s = acc[k];
                    for (int n = 0; n < nc; ++n) s = fmaf(ri[n], rj[n], s);
                    acc[k] = s;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kGramAcc; ++k) {
            const int q = threadIdx.x + k * 256;
            if (q < npairs) {
                int i, j;
                lower_of(q, i, j);
                const T v = from_f32<T>(acc[k]);
                z[(int64_t)b * z_bs + (int64_t)i * F + j] = v;
                z[(int64_t)b * z_bs + (int64_t)j * F + i] = v;
            }
        }
    }
}

// dT_b[f][n] = sum_j (Δ_b[f][j] + Δ_b[j][f]) T_b[j][n]   (fp32 out; j ascending, fmaf)
template <typename T>
__global__ __launch_bounds__(256) void self_batched_mul_back_kernel(int d, int F, int B, const T* __restrict__ t,
                                                                    int64_t t_ld, const T* __restrict__ dz,
                                                                    int64_t dz_bs, float* __restrict__ dt,
                                                                    int64_t dt_ld) {
    __shared__ float ss[90 * 90];
    __shared__ float ts[90 * kSliceChunk];
    for (int b = blockIdx.x; b < B; b += gridDim.x) {
        const T* tb = t + (int64_t)b * t_ld;
        const T* db = dz + (int64_t)b * dz_bs;
        __syncthreads();
        for (int e = threadIdx.x; e < F * F; e += blockDim.x) {
            const int f = e / F, j = e % F;
            ss[e] = to_f32(db[(int64_t)f * F + j]) + to_f32(db[(int64_t)j * F + f]);
        }
        for (int n0 = 0; n0 < d; n0 += kSliceChunk) {
            const int nc = min(kSliceChunk, d - n0);
            __syncthreads();
            for (int e = threadIdx.x; e < F * nc; e += blockDim.x) {
                const int f = e / nc, n = e % nc;
                ts[f * kSliceChunk + n] = to_f32(tb[(int64_t)f * d + n0 + n]);
            }
            __syncthreads();
            for (int e = threadIdx.x; e < F * nc; e += blockDim.x) {
                const int f = e / nc, n = e % nc;
                float s = 0.0f;
                for (int j = 0; j < F; ++j) s = fmaf(ss[f * F + j], ts[j * kSliceChunk + n], s);
                dt[(int64_t)b * dt_ld + (int64_t)f * d + n0 + n] = s;
            }
        }
    }
}

static unsigned slice_grid(int64_t items, int cus) {
    int64_t g = (items + 255) / 256;
    const int64_t cap = (int64_t)cus * 16;
    if (g > cap) g = cap;
    return (unsigned)(g < 1 ? 1 : g);
}

int launch_triangular_slice(dlrm_ctx* ctx, int dtype, int sz, int B, const void* z, int64_t z_bs, void* out,
                            int64_t out_ld) {
    if (B == 0 || sz < 2) return DLRM_OK;
    hipStream_t s = ctx_stream(ctx);
    const unsigned g = slice_grid((int64_t)B * sz * (sz - 1) / 2, ctx_num_cus(ctx));
    if (dtype == DLRM_F32)
        hipLaunchKernelGGL(triangular_slice_kernel<float>, dim3(g), dim3(256), 0, s, sz, B, (const float*)z, z_bs,
                           (float*)out, out_ld);
    else
        hipLaunchKernelGGL(triangular_slice_kernel<uint16_t>, dim3(g), dim3(256), 0, s, sz, B, (const uint16_t*)z,
                           z_bs, (uint16_t*)out, out_ld);
    return ctx_hip(ctx, hipGetLastError(), "triangular_slice launch");
}

int launch_triangular_slice_back(dlrm_ctx* ctx, int dtype, int sz, int B, const void* dy, int64_t dy_ld, void* a,
                                 int64_t a_bs, int sym) {
    if (B == 0 || sz < 1) return DLRM_OK;
    hipStream_t s = ctx_stream(ctx);
    const unsigned g = slice_grid((int64_t)B * sz * sz, ctx_num_cus(ctx));
    if (dtype == DLRM_F32)
        hipLaunchKernelGGL(triangular_slice_back_kernel<float>, dim3(g), dim3(256), 0, s, sz, B, (const float*)dy,
                           dy_ld, (float*)a, a_bs, sym);
    else
        hipLaunchKernelGGL(triangular_slice_back_kernel<uint16_t>, dim3(g), dim3(256), 0, s, sz, B,
                           (const uint16_t*)dy, dy_ld, (uint16_t*)a, a_bs, sym);
    return ctx_hip(ctx, hipGetLastError(), "triangular_slice_back launch");
}

int launch_self_batched_mul(dlrm_ctx* ctx, int dtype, int d, int F, int B, const void* t, int64_t t_ld, void* z,
                            int64_t z_bs) {
    if (B == 0) return DLRM_OK;
    hipStream_t s = ctx_stream(ctx);
    int64_t g = B;
    const int64_t cap = (int64_t)ctx_num_cus(ctx) * 8;
    if (g > cap) g = cap;
    if (dtype == DLRM_F32)
        hipLaunchKernelGGL(self_batched_mul_kernel<float>, dim3((unsigned)g), dim3(256), 0, s, d, F, B, (const float*)t,
                           t_ld, (float*)z, z_bs);
    else
        hipLaunchKernelGGL(self_batched_mul_kernel<uint16_t>, dim3((unsigned)g), dim3(256), 0, s, d, F, B,
                           (const uint16_t*)t, t_ld, (uint16_t*)z, z_bs);
    return ctx_hip(ctx, hipGetLastError(), "self_batched_mul launch");
}

int launch_self_batched_mul_back(dlrm_ctx* ctx, int dtype, int d, int F, int B, const void* t, int64_t t_ld,
                                 const void* dz, int64_t dz_bs, float* dt, int64_t dt_ld) {
    if (B == 0) return DLRM_OK;
    hipStream_t s = ctx_stream(ctx);
    int64_t g = B;
    const int64_t cap = (int64_t)ctx_num_cus(ctx) * 8;
    if (g > cap) g = cap;
    if (dtype == DLRM_F32)
        hipLaunchKernelGGL(self_batched_mul_back_kernel<float>, dim3((unsigned)g), dim3(256), 0, s, d, F, B,
                           (const float*)t, t_ld, (const float*)dz, dz_bs, dt, dt_ld);
    else
        hipLaunchKernelGGL(self_batched_mul_back_kernel<uint16_t>, dim3((unsigned)g), dim3(256), 0, s, d, F, B,
                           (const uint16_t*)t, t_ld, (const uint16_t*)dz, dz_bs, dt, dt_ld);
    return ctx_hip(ctx, hipGetLastError(), "self_batched_mul_back launch");
}

}  // namespace dlrm
