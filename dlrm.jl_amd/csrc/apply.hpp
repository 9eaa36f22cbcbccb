// apply.hpp — the work items of EmbeddingTables.update!(Descent(lr), ...) (sgd_apply_kernel).
//
// Reference: src/train/train.jl:283-290 (update! over the SparseIndexer's grouping), pinned by
// src/validation.jl:125-146.  Work items of the indexer (indexer.hpp):
//   * a chunk: a segment (one table row) of <= kChunk positions, run by one lane group: the grad
//     rows are summed in ascending position order from 0, then w = fmaf(-lr, sum, w);
//   * a slice: <= kHotSlice consecutive positions of a longer (hot) segment, run by a whole
//     256-thread workgroup: each lane group sums its consecutive share of the slice in position
//     order, the groups of a wave are combined by a fixed xor butterfly, the waves in wave order.
//     A one-slice segment then updates its row; otherwise the slice stores its partial row
//     (write-through) and adds to the segment's arrival counter, and the last arriving slice adds
//     the partials in slice order from 0 and updates the row.
// Every touched row is written exactly once with a summation order fixed by its positions alone,
// so the result is bitwise reproducible.
//
// Latency is what bounds these items (a few dependent memory round trips each), so a chunk's
// first kChunkInline positions come with its descriptor, the rest with one load per lane, and up
// to 16 grad rows are in flight per lane group.
#pragma once
#include "indexer.hpp"

namespace dlrm {

constexpr int kApplyThreads = 256;
#ifndef DLRM_SLICE_IF
#define DLRM_SLICE_IF 16
#endif
constexpr int kSliceIF = DLRM_SLICE_IF;  // hot slice: grad rows in flight per lane (16-B rows)
constexpr int kApplyWaves = kApplyThreads / 64;

// Lane-group geometry: D elements = VPR vectors of 16 B of the GRAD dtype; a group of LPR lanes
// owns one row, a wave holds RPW groups.
template <typename GT, int VPR>
struct ApplyGeom {
    typedef Vec<GT> GV;
    static constexpr int NE = GV::N;
    static constexpr int D = VPR * NE;
    static constexpr int LPR = VPR <= 64 ? VPR : 64;
    static constexpr int VPL = VPR <= 64 ? 1 : VPR / 64;
    static constexpr int RPW = 64 / LPR;
    static constexpr int NG = kApplyWaves * RPW;        // lane groups per workgroup
    static constexpr int SIF = NE == 8 ? kSliceIF / 2 : kSliceIF;  // hot slice rows in flight (bf16: 8 per 16 B)
    static constexpr int IF = VPL >= 4 ? 4 : (NE == 8 ? 8 : 16) / VPL;  // grad rows in flight per lane
    // once-hit positions per lane group (a grad and a table row in flight for each)
    static constexpr int SPPG = VPL * NE >= 16 ? 2 : (VPL * NE >= 8 ? 4 : 8);
};

// Cross-workgroup hand-off of slice partials (cdna_hip_programming.md Guideline 16, R1/R2):
// payload stored write-through (agent-scope atomic stores = sc1), the storing wave drains
// (vmcnt(0)) before ONE lane adds to the segment's arrival counter; the last arriver reads every
// partial with sc1 loads (no acquire needed) and resets the counter for the next launch.
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) int gi32_t;

__device__ __forceinline__ void store_sc1(float* p, const f32x4& v) {
    const unsigned long long lo = ((unsigned long long)__float_as_uint(v[1]) << 32) | __float_as_uint(v[0]);
    const unsigned long long hi = ((unsigned long long)__float_as_uint(v[3]) << 32) | __float_as_uint(v[2]);
    __hip_atomic_store((gu64_t*)p, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gu64_t*)(p + 2), hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ f32x4 load_sc1(const float* p) {
    const unsigned long long lo = __hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long hi = __hip_atomic_load((gu64_t*)(p + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return f32x4{__uint_as_float((uint32_t)lo), __uint_as_float((uint32_t)(lo >> 32)), __uint_as_float((uint32_t)hi),
                 __uint_as_float((uint32_t)(hi >> 32))};
}

// The grad row of position p, vector k of this lane (k = v + j*64).
template <typename GT>
__device__ __forceinline__ typename Vec<GT>::type grad_vec(const GT* gbase, int64_t grad_ld, const FastDiv& L, int p, int k) {
    return ldg<typename Vec<GT>::type>((const typename Vec<GT>::type*)(gbase + (int64_t)L(p) * grad_ld) + k);
}

template <typename GT>
__device__ __forceinline__ void add_vec(float* acc, const typename Vec<GT>::type& g) {
    float f[Vec<GT>::N];
    Vec<GT>::to_f32(g, f);
#pragma unroll
    for (int e = 0; e < Vec<GT>::N; ++e) acc[e] += f[e];
}

// ---- a chunk, by one lane group (lane v of LPR; gl0 = the group's first lane in the wave)
template <typename TT, typename GT, int VPR>
__device__ __forceinline__ void run_chunk(const int32_t* __restrict__ perm, const int4& a, const int4& b,
                                          TT* __restrict__ table, const GT* __restrict__ gbase, int64_t grad_ld,
                                          const FastDiv& L, float lr, int v, int gl0) {
    typedef ApplyGeom<GT, VPR> G;
    constexpr int NE = G::NE, D = G::D, LPR = G::LPR;
    constexpr int KX = (kChunk - kChunkInline + LPR - 1) / LPR;  // perm loads per lane (long chunks)
    const int beg = a.x, len = a.y - a.x;
    TT* row = table + (int64_t)(uint32_t)a.z * D;
    float tv[G::VPL][NE];
#pragma unroll
    for (int j = 0; j < G::VPL; ++j) load_row<TT, NE>(row, (v + j * 64) * NE, tv[j]);  // beside the grad rows
    const int inl[kChunkInline] = {a.w, b.x, b.y, b.z, b.w};
    int px[KX];  // positions kChunkInline.. : position kChunkInline + k*LPR + lane
    if (len > kChunkInline) {
#pragma unroll
        for (int k = 0; k < KX; ++k) {
            const int u = kChunkInline + k * LPR + v;
            px[k] = u < len ? perm[beg + u] : 0;
        }
    }
    float acc[G::VPL][NE];
#pragma unroll
    for (int j = 0; j < G::VPL; ++j)
#pragma unroll
        for (int e = 0; e < NE; ++e) acc[j][e] = 0.0f;
    constexpr int IF = G::IF;
#pragma unroll
    for (int u0 = 0; u0 < kChunk; u0 += IF) {
        if (u0 >= len) break;  // uniform over the group
        typename Vec<GT>::type gv[IF][G::VPL];
#pragma unroll
        for (int uu = 0; uu < IF; ++uu) {
            const int u = u0 + uu;
            if (u < len) {
                const int p = u < kChunkInline ? inl[u < kChunkInline ? u : 0]
                                               : __shfl(px[(u - kChunkInline) / LPR], gl0 + (u - kChunkInline) % LPR, 64);
#pragma unroll
                for (int j = 0; j < G::VPL; ++j) gv[uu][j] = grad_vec<GT>(gbase, grad_ld, L, p, v + j * 64);
            }
        }
#pragma unroll
        for (int uu = 0; uu < IF; ++uu)
            if (u0 + uu < len)
#pragma unroll
                for (int j = 0; j < G::VPL; ++j) add_vec<GT>(acc[j], gv[uu][j]);
    }
#pragma unroll
    for (int j = 0; j < G::VPL; ++j) {
#pragma unroll
        for (int e = 0; e < NE; ++e) tv[j][e] = __builtin_fmaf(-lr, acc[j][e], tv[j][e]);
        store_row<TT, NE>(row, (v + j * 64) * NE, tv[j]);
    }
}

// ---- once-hit positions of a split indexer (single[p] = 1: the position's row is hit by no other
// position), SPPG consecutive positions per lane group: w = fmaf(-lr, 0 + g, w), the chunk
// path's arithmetic for a one-position segment, with no descriptor or perm read.
struct SinglesArgs {
    const uint8_t* single;  // [T][cap] (IndexerDev::single); NULL: no singles items
    const void* idx;
    int itype;
    int64_t tstride;
    int base;
    int N;                  // positions per table
};
template <typename TT, typename GT, int VPR>
__device__ __forceinline__ void run_singles(const SinglesArgs& sa, int64_t cap, TT* __restrict__ table, int64_t nrows,
                                            int t, int p0, const GT* __restrict__ gbase, int64_t grad_ld, const FastDiv& L,
                                            float lr, int v, int gl0) {
    typedef ApplyGeom<GT, VPR> G;
    constexpr int NE = G::NE, D = G::D, LPR = G::LPR, PPG = G::SPPG;
    constexpr int KX = (PPG + LPR - 1) / LPR;
    uint32_t pr[KX];  // the row of position p0 + k*LPR + v, ~0u when it is not a single
#pragma unroll
    for (int k = 0; k < KX; ++k) {
        const int u = k * LPR + v;
        const bool ok = u < PPG && p0 + u < sa.N;
        const uint8_t fl = ok ? ldg<uint8_t>(sa.single + (int64_t)t * cap + p0 + u) : (uint8_t)0;
        const int64_t r = load_index_if(ok, sa.idx, sa.itype, (int64_t)t * sa.tstride + p0 + u) - sa.base;
        pr[k] = (fl && r >= 0 && r < nrows) ? (uint32_t)r : ~0u;
    }
    uint32_t ru[PPG];
    typename Vec<GT>::type gv[PPG][G::VPL];
    float tv[PPG][G::VPL][NE];
#pragma unroll
    for (int u = 0; u < PPG; ++u) {
        ru[u] = (uint32_t)__shfl((int)pr[u / LPR], gl0 + u % LPR, 64);
        if (ru[u] != ~0u) {
#pragma unroll
            for (int j = 0; j < G::VPL; ++j) {
                gv[u][j] = grad_vec<GT>(gbase, grad_ld, L, p0 + u, v + j * 64);
                load_row<TT, NE>(table + (int64_t)ru[u] * D, (v + j * 64) * NE, tv[u][j]);
            }
        }
    }
#pragma unroll
    for (int u = 0; u < PPG; ++u)
        if (ru[u] != ~0u)
#pragma unroll
            for (int j = 0; j < G::VPL; ++j) {
                float g[NE];
                Vec<GT>::to_f32(gv[u][j], g);
#pragma unroll
                for (int e = 0; e < NE; ++e) tv[u][j][e] = __builtin_fmaf(-lr, 0.0f + g[e], tv[u][j][e]);
                store_row<TT, NE>(table + (int64_t)ru[u] * D, (v + j * 64) * NE, tv[u][j]);
            }
}

// The NEXT batch's split indexer, built by extra workgroups of this apply launch (the training
// step's pipelined form: dlrm_step_bwd_prepare).  Its bounds errors go to `err` (private: the next
// step's forward gathers the same indices and raises them on the context's flag).
struct PrepArgs {
    IndexerDev ix;
    const TableDesc* tabs;  // the tables (for nrows)
    int T;                  // real tables
    const void* idx;
    int itype;
    int64_t tstride;
    int base;
    int N;
    unsigned* err;
};

// LDS of a hot-slice item (one workgroup)
template <int D>
struct SliceLds {
    f32x4 wsum[kApplyWaves][D / 4];   // per-wave partial rows
    int last;
};

// ---- a slice of a hot segment, by the whole workgroup: pos = its positions (perm entries),
// len of them, `row` the table row, `ns` the slices of its segment, its partial row at
// part_me, the segment's first at part_first (slot spacing pdim), `cnt` the segment's arrival
// counter (zero at rest).
template <typename TT, typename GT, int VPR>
__device__ __forceinline__ void slice_body(const int32_t* __restrict__ pos, int len, TT* __restrict__ row, int ns,
                                           float* part_me, const float* part_first, int64_t pdim, int32_t* cnt_p,
                                           const GT* __restrict__ gbase, int64_t grad_ld, const FastDiv& L, float lr,
                                           SliceLds<ApplyGeom<GT, VPR>::D>& sm) {
    typedef ApplyGeom<GT, VPR> G;
    constexpr int NE = G::NE, D = G::D, LPR = G::LPR, NG = G::NG;
    constexpr int SPG = (kHotSlice + NG - 1) / NG;  // positions per lane group
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int g = lane / LPR, v = lane % LPR, gid = w * G::RPW + g;
    // the table row, loaded now (needed only at the end; no other item writes it in this launch)
    float rw[4];
    if (tid < D / 4) load_row<TT, 4>(row, tid * 4, rw);
    // this group's consecutive share [g0, u1), in position order: lane v of the group loads
    // positions g0 + k LPR + v, and each row's position comes by a shuffle (no LDS staging and no
    // barrier before the grad rows)
    const int g0 = gid * SPG, u1 = min(len, g0 + SPG);  // (SPG = kHotSlice / NG)
    static_assert(SPG <= LPR, "one position per lane of the group");
    const int gl0 = lane - v;
    const int px = g0 + v < u1 ? pos[g0 + v] : 0;
    float acc[G::VPL][NE];
#pragma unroll
    for (int j = 0; j < G::VPL; ++j)
#pragma unroll
        for (int e = 0; e < NE; ++e) acc[j][e] = 0.0f;
    // grad rows in flight per lane: a lane group's whole share at one 16-B vector per row
    // up to kSliceIF, else the chunk items' IF
    constexpr int IFS = G::VPL == 1 ? (SPG < G::SIF ? SPG : G::SIF) : G::IF;
    constexpr int IF = IFS < SPG ? IFS : SPG;
#pragma unroll 1
    for (int r0 = 0; r0 < SPG; r0 += IF) {
        const int u0 = g0 + r0;
        if (u0 >= u1) break;  // uniform over the group
        typename Vec<GT>::type gv[IF][G::VPL];
#pragma unroll
        for (int uu = 0; uu < IF; ++uu) {
            const int p = __shfl(px, gl0 + r0 + uu, 64);
            if (u0 + uu < u1)
#pragma unroll
                for (int j = 0; j < G::VPL; ++j) gv[uu][j] = grad_vec<GT>(gbase, grad_ld, L, p, v + j * 64);
        }
#pragma unroll
        for (int uu = 0; uu < IF; ++uu)
            if (u0 + uu < u1)
#pragma unroll
                for (int j = 0; j < G::VPL; ++j) add_vec<GT>(acc[j], gv[uu][j]);
    }
    // the wave's groups: xor butterfly over the group bits of the lane (fixed order)
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1)
#pragma unroll
        for (int j = 0; j < G::VPL; ++j)
#pragma unroll
            for (int e = 0; e < NE; ++e) acc[j][e] += __shfl_xor(acc[j][e], o, 64);
    if (g == 0)
#pragma unroll
        for (int j = 0; j < G::VPL; ++j)
#pragma unroll
            for (int e = 0; e < NE; e += 4)
                sm.wsum[w][((v + j * 64) * NE + e) / 4] = f32x4{acc[j][e], acc[j][e + 1], acc[j][e + 2], acc[j][e + 3]};
    __syncthreads();
    // the waves, in wave order, by the first D/4 threads (one float4 of the row each)
    f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
    if (tid < D / 4) {
#pragma unroll
        for (int ww = 0; ww < kApplyWaves; ++ww) sum += sm.wsum[ww][tid];
    }
    static_assert(D / 4 <= kApplyThreads, "a float4 of the row per thread");
    if (ns == 1) {
        if (tid < D / 4) {
#pragma unroll
            for (int e = 0; e < 4; ++e) rw[e] = __builtin_fmaf(-lr, sum[e], rw[e]);
            store_row<TT, 4>(row, tid * 4, rw);
        }
        __syncthreads();  // sm reused by this workgroup's next item
        return;
    }
    gi32_t* cnt = (gi32_t*)cnt_p;
    if (tid < D / 4) store_sc1(part_me + tid * 4, sum);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the arrival
    if (D / 4 > 64) __syncthreads();                   // (several storing waves)
    if (tid == 0) sm.last = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ns - 1;
    __syncthreads();
    if (sm.last && tid < D / 4) {
        float* f = rw;
        const float* first = part_first + tid * 4;
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
        constexpr int PB = 16;  // partial rows in flight
        for (int k0 = 0; k0 < ns; k0 += PB) {
            f32x4 q[PB];
#pragma unroll
            for (int u = 0; u < PB; ++u) q[u] = load_sc1(first + (int64_t)(k0 + u < ns ? k0 + u : k0) * pdim);
#pragma unroll
            for (int u = 0; u < PB; ++u)
                if (k0 + u < ns) s += q[u];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) f[e] = __builtin_fmaf(-lr, s[e], f[e]);
        store_row<TT, 4>(row, tid * 4, f);
        if (tid == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();  // sm reused by this workgroup's next item
}

// ---- a slice of a hot segment located by (virtual table vt, local slice sl): sd = {p0, p1,
// row, h}; the segment's descriptor ix.hot[vt][h] = {beg, end, row, first slice}
template <typename TT, typename GT, int VPR>
__device__ __forceinline__ void run_slice(const IndexerDev& ix, int vt, int sl, const int4& sd, TT* __restrict__ table,
                                          const GT* __restrict__ gbase, int64_t grad_ld, const FastDiv& L, float lr,
                                          SliceLds<ApplyGeom<GT, VPR>::D>& sm) {
    constexpr int D = ApplyGeom<GT, VPR>::D;
    const int64_t off = (int64_t)vt * ix.cap;
    const int4 hd = ix.hot[off + sd.w];
    const int ns = (hd.y - hd.x + kHotSlice - 1) / kHotSlice;
    float* pbase = ix.partial + (int64_t)vt * ix.pcap * ix.pdim;
    slice_body<TT, GT, VPR>(ix.perm + off + sd.x, sd.y - sd.x, table + (int64_t)(uint32_t)sd.z * D, ns,
                            pbase + (int64_t)sl * ix.pdim, pbase + (int64_t)hd.w * ix.pdim, ix.pdim,
                            ix.hot_cnt + off + sd.w, gbase, grad_ld, L, lr, sm);
}

// ---- hot slice k of the item map (one 32-B record: IndexerDev::slice_rec); k and its segment's
// first slice `first` count over the sub-lists' slices in order (partial row and counter slots)
template <typename TT, typename GT, int VPR>
__device__ __forceinline__ void run_slice_rec(const IndexerDev& ix, int k, int first, const int4& r0, const int4& r1,
                                              TT* __restrict__ table, const GT* __restrict__ gbase, int64_t grad_ld,
                                              const FastDiv& L, float lr, SliceLds<ApplyGeom<GT, VPR>::D>& sm) {
    constexpr int D = ApplyGeom<GT, VPR>::D;
    slice_body<TT, GT, VPR>(ix.perm + r0.x, r0.y - r0.x, table + (int64_t)(uint32_t)r0.z * D, r1.x,
                            ix.partial + (int64_t)k * ix.pdim, ix.partial + (int64_t)first * ix.pdim, ix.pdim,
                            ix.hot_cnt + first, gbase, grad_ld, L, lr, sm);
}

}  // namespace dlrm
