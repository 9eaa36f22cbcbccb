// lookup.hip — maplookup(PreallocationStrategy(P), tables, sparse) on gfx950.
//
// Reference: EmbeddingTables.maplookup (un-vendored), called at src/model/model.jl:161;
// semantics pinned by test/model/embedding_update.jl:23-33 and the golden
// `concatenated_result` of ref/pytorch_reference_{single,multi}.hdf5.
//
//   out[b][P + t*D + c] = sum_{k<L} table_t[idx_t[b*L + k] - base][c]
//
// HBM-bound row gather.  Each output row (one (sample, table) pair) is D*E bytes; a wave
// splits into RPW row groups of LPR lanes, each lane moving 16 B per access, so every
// wave-instruction reads RPW whole rows (coalesced 16-B lanes) and writes them back as one
// contiguous run (items are ordered b-major so consecutive tables of a sample are adjacent
// in the output).  Every lane keeps U independent row loads in flight before it stores.
// Pooled bags (L > 1) are seeded with the first row and accumulated in k order in fp32
// (an exact copy for L = 1), then rounded once to the table dtype.
#include "common.hpp"

namespace dlrm {

// A wave takes RPW*U consecutive (sample, table) items; per round of KB lookups of a bag every
// index load of its U bags is issued first, then every row load (unmasked: an out-of-range index
// reads the zero row and raises the flag after the stores), then the k-ordered sums -- a lane
// keeps U x KB x VPL 16-B loads in flight, and a bag costs ceil(L / KB) index->row round trips.
// (The branchy form waited on each row load before issuing the next: 23 us for the sharded
// lookup's 65,536 rows of 512 B.)  TP: the table pointers from a TabPtrs argument (T <= 32),
// else one descriptor load per item, issued with the first round's index loads.
#ifndef DLRM_LOOKUP_NT
#define DLRM_LOOKUP_NT 0
#endif
constexpr bool kLookupNT = DLRM_LOOKUP_NT;  // non-temporal output stores (A/B builds)
template <typename T, int VPR, int U, int KB, bool TP>
__global__ __launch_bounds__(256) void maplookup_vec(const TableDesc* __restrict__ tabs, TabPtrs tp, int ntab,
                                                     const void* __restrict__ idx, int itype,
                                                     int64_t tstride, int base, int B, int L,
                                                     T* __restrict__ out, OutMap om, unsigned* __restrict__ err) {
    typedef Vec<T> V;
    typedef typename V::type vt;
    constexpr int NE = V::N;                       // elements per 16-B vector
    constexpr int LPR = VPR <= 64 ? VPR : 64;      // lanes per row
    constexpr int VPL = VPR <= 64 ? 1 : VPR / 64;  // vectors per lane
    constexpr int RPW = 64 / LPR;                  // rows per wave-instruction
    static_assert(VPR * 16 <= kZeroElems * 4, "rows longer than the zero row");
    const int lane = threadIdx.x & 63;
    const int g = lane / LPR, v = lane % LPR;
    if (g >= RPW) return;  // idle lanes when LPR does not divide 64
    const int wave = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int nwaves = (int)(((int64_t)gridDim.x * blockDim.x) >> 6);
    const int total = ntab * B;  // < 2^31 (launch_maplookup_map)
    constexpr int D = VPR * NE;
    const vt* zero = (const vt*)g_zero_row;
    bool bad = false;

    // (64-bit cursor: total < 2^31, but total + a grid stride need not be)
    for (int64_t first = (int64_t)wave * (RPW * U); first < total; first += (int64_t)nwaves * (RPW * U)) {
        int bb[U], tt[U];
        bool live[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t item = first + u * RPW + g;
            live[u] = item < total;
            const int it = live[u] ? (int)item : 0;
            bb[u] = it / ntab;
            tt[u] = it - bb[u] * ntab;
        }
        TableDesc td[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (TP) td[u] = TableDesc{(void*)tp.p[tt[u]], (int64_t)tp.n[tt[u]]};
            else td[u] = load_table(tabs, tt[u]);
        }
        float acc[U][VPL][NE];
        for (int k0 = 0; k0 < L; k0 += KB) {
            int64_t ri[U][KB];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int kk = 0; kk < KB; ++kk)
                    ri[u][kk] = load_index_if(live[u] && k0 + kk < L, idx, itype,
                                              tt[u] * tstride + (int64_t)bb[u] * L + k0 + kk);
            const vt* src[U][KB];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int kk = 0; kk < KB; ++kk) {
                    const bool use = live[u] && k0 + kk < L;
                    const int64_t r = ri[u][kk] - base;
                    const bool ok = use & (r >= 0) & (r < td[u].nrows);
                    bad |= use & !ok;
                    src[u][kk] = ok ? (const vt*)((const T*)td[u].data + r * D) : zero;
                }
            __builtin_amdgcn_sched_barrier(0);
            vt vv[U][KB][VPL];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int kk = 0; kk < KB; ++kk)
#pragma unroll
                    for (int j = 0; j < VPL; ++j) vv[u][kk][j] = ldg<vt>(src[u][kk] + v + j * 64);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int kk = 0; kk < KB; ++kk) {
                    if (k0 + kk >= L) break;
#pragma unroll
                    for (int j = 0; j < VPL; ++j) {
                        float f[NE];
                        V::to_f32(vv[u][kk][j], f);
#pragma unroll
                        for (int e = 0; e < NE; ++e) acc[u][j][e] = (k0 + kk == 0) ? f[e] : acc[u][j][e] + f[e];
                    }
                }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!live[u]) continue;
            T* o = out + om.row(bb[u]) + (int64_t)tt[u] * om.tstride;
#pragma unroll
            for (int j = 0; j < VPL; ++j) {
                if constexpr (kLookupNT) stg_nt<vt>((vt*)o + v + j * 64, V::from_f32(acc[u][j]));
                else stg<vt>((vt*)o + v + j * 64, V::from_f32(acc[u][j]));
            }
        }
    }
    if (bad && v == 0) raise_index_error(err);
}

// Scalar fallback for shapes / alignments the vector kernel does not take.
template <typename T>
__global__ __launch_bounds__(256) void maplookup_scalar(const TableDesc* __restrict__ tabs, int ntab, int D,
                                                        const void* __restrict__ idx, int itype,
                                                        int64_t tstride, int base, int B, int L,
                                                        T* __restrict__ out, OutMap om, unsigned* __restrict__ err) {
    const int64_t total = (int64_t)ntab * B * D;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(e % D);
        const int64_t item = e / D;
        const int64_t b = item / ntab;
        const int t = (int)(item - b * ntab);
        float acc = 0.0f;
        for (int k = 0; k < L; ++k) {
            const int64_t r = load_index(idx, itype, t * tstride + b * L + k) - base;
            float f = 0.0f;
            if (r >= 0 && r < tabs[t].nrows) f = to_f32(((const T*)tabs[t].data)[r * D + c]);
            else if (c == 0) raise_index_error(err);
            acc = (k == 0) ? f : acc + f;
        }
        out[om.row(b) + (int64_t)t * om.tstride + c] = from_f32<T>(acc);
    }
}

template <typename T, int VPR>
static void launch_vec(hipStream_t s, int cus, const TableDesc* tabs, const TabPtrs* tp, int T_, const void* idx,
                       int itype, int64_t tstride, int base, int B, int L, void* out, const OutMap& om, unsigned* err) {
    constexpr int LPR = VPR <= 64 ? VPR : 64;
    constexpr int RPW = 64 / LPR;
    // one-hot: 4 rows per lane group (8 at <= 256-B rows); pooled: 2 bags x 4 lookups
    constexpr int U1 = VPR <= 16 ? 8 : 4;
    const int U = L > 1 ? 2 : U1;
    const int64_t total = (int64_t)T_ * B;
    const int64_t waves = (total + RPW * U - 1) / (RPW * U);
    int64_t blocks = (waves + 3) / 4;
    const int64_t cap = (int64_t)cus * 16;  // grid-stride beyond 16 blocks per CU
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    static const TabPtrs none{};
#define DLRM_LAUNCH(U_, KB_, TP_)                                                                               \
    hipLaunchKernelGGL((maplookup_vec<T, VPR, U_, KB_, TP_>), dim3((unsigned)blocks), dim3(256), 0, s, tabs,       \
                       tp ? *tp : none, T_, idx, itype, tstride, base, B, L, (T*)out, om, err)
    if (L > 1) {
        if (tp) DLRM_LAUNCH(2, 4, true); else DLRM_LAUNCH(2, 4, false);
    } else {
        if (tp) DLRM_LAUNCH(U1, 1, true); else DLRM_LAUNCH(U1, 1, false);
    }
#undef DLRM_LAUNCH
}

template <typename T>
static bool dispatch_vec(int vpr, hipStream_t s, int cus, const TableDesc* tabs, const TabPtrs* tp, int T_,
                         const void* idx, int itype, int64_t tstride, int base, int B, int L, void* out,
                         const OutMap& om, unsigned* err) {
#define DLRM_CASE(N) \
    case N: launch_vec<T, N>(s, cus, tabs, tp, T_, idx, itype, tstride, base, B, L, out, om, err); return true;
    switch (vpr) {
        DLRM_CASE(1) DLRM_CASE(2) DLRM_CASE(4) DLRM_CASE(8) DLRM_CASE(16) DLRM_CASE(32) DLRM_CASE(64)
        DLRM_CASE(128) DLRM_CASE(256)
        default: return false;
    }
#undef DLRM_CASE
}

int launch_maplookup(dlrm_ctx* ctx, const TableDesc* d_tabs, bool tabs_aligned16, int T_, int D, int dtype,
                     const void* idx, int itype, int64_t tstride, int base, int B, int L, void* out,
                     int64_t out_ld, int64_t out_off, const TableDesc* htabs) {
    return launch_maplookup_map(ctx, d_tabs, tabs_aligned16, T_, D, dtype, idx, itype, tstride, base, B, L, out,
                                OutMap{out_ld, out_off, D, B > 0 ? B : 1, 0}, htabs);
}

int launch_maplookup_map(dlrm_ctx* ctx, const TableDesc* d_tabs, bool tabs_aligned16, int T_, int D, int dtype,
                         const void* idx, int itype, int64_t tstride, int base, int B, int L, void* out,
                         const OutMap& om, const TableDesc* htabs) {
    if (T_ == 0 || B == 0) return DLRM_OK;
    hipStream_t s = ctx_stream(ctx);
    unsigned* err = ctx_error_word(ctx);
    const int cus = ctx_num_cus(ctx);
    const int esz = dtype == DLRM_F32 ? 4 : 2;
    const bool aligned = tabs_aligned16 && ((uintptr_t)out % 16 == 0) && ((om.ld * esz) % 16 == 0) &&
                         ((om.off * esz) % 16 == 0) && ((om.tstride * esz) % 16 == 0) &&
                         ((om.bstride * esz) % 16 == 0) && ((D * esz) % 16 == 0);
    bool done = false;
    if (aligned && (int64_t)T_ * B < (1ll << 31)) {
        const int vpr = D * esz / 16;
        TabPtrs tp;
        const TabPtrs* tpp = fill_tab_ptrs(tp, htabs, T_) ? &tp : nullptr;
        done = dtype == DLRM_F32
                   ? dispatch_vec<float>(vpr, s, cus, d_tabs, tpp, T_, idx, itype, tstride, base, B, L, out, om, err)
                   : dispatch_vec<uint16_t>(vpr, s, cus, d_tabs, tpp, T_, idx, itype, tstride, base, B, L, out, om,
                                            err);
    }
    if (!done) {
        const int64_t total = (int64_t)T_ * B * D;
        int64_t blocks = (total + 255) / 256;
        if (blocks > (int64_t)cus * 16) blocks = (int64_t)cus * 16;
        if (dtype == DLRM_F32)
            hipLaunchKernelGGL(maplookup_scalar<float>, dim3((unsigned)blocks), dim3(256), 0, s, d_tabs, T_, D, idx,
                               itype, tstride, base, B, L, (float*)out, om, err);
        else
            hipLaunchKernelGGL(maplookup_scalar<uint16_t>, dim3((unsigned)blocks), dim3(256), 0, s, d_tabs, T_, D, idx,
                               itype, tstride, base, B, L, (uint16_t*)out, om, err);
    }
    return ctx_hip(ctx, hipGetLastError(), "maplookup launch");
}

// ------------------------------------------------------------------------- row scatter
// dst + dbase[t] + b * dld[t]  <-  src + b * src_ld + src_off + t * D   (D elements each): the
// exchange's repack of a [B][T*D] row block into per-destination blocks (sharded.py), one
// launch for every table.  16-B lanes where the geometry allows.
// Work item = one 16-B piece (VEC: the source rows are 16-B aligned and D*esize % 16 == 0) or
// one element.  A destination row that is not 16-B aligned takes the element path.
template <bool VEC>
__global__ __launch_bounds__(256) void scatter_rows_kernel(int T_, int B, int D, int esize, const char* __restrict__ src,
                                                           int64_t src_ld, int64_t src_off, char* __restrict__ dst,
                                                           const int64_t* __restrict__ dbase,
                                                           const int64_t* __restrict__ dld) {
    const int per = VEC ? 16 / esize : 1;  // elements per item
    const int nv = D / per;
    const int64_t total = (int64_t)B * T_ * nv;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int j = (int)(e % nv);
        const int64_t bt = e / nv;
        const int t = (int)(bt % T_);
        const int64_t b = bt / T_;
        const int64_t so = (b * src_ld + src_off + (int64_t)t * D + (int64_t)j * per) * esize;
        const int64_t dof = (dbase[t] + b * dld[t] + (int64_t)j * per) * esize;
        if (VEC && dof % 16 == 0) {
            *(uint4*)(dst + dof) = *(const uint4*)(src + so);
        } else if (esize == 4) {
            for (int k = 0; k < per; ++k) ((uint32_t*)(dst + dof))[k] = ((const uint32_t*)(src + so))[k];
        } else {
            for (int k = 0; k < per; ++k) ((uint16_t*)(dst + dof))[k] = ((const uint16_t*)(src + so))[k];
        }
    }
}

int launch_scatter_rows(dlrm_ctx* ctx, int esize, int T_, int B, int D, const void* src, int64_t src_ld,
                        int64_t src_off, void* dst, const int64_t* dbase, const int64_t* dld, bool vec_ok) {
    if (T_ == 0 || B == 0 || D == 0) return DLRM_OK;
    hipStream_t s = ctx_stream(ctx);
    const int cus = ctx_num_cus(ctx);
    const int64_t items = (int64_t)B * T_ * (vec_ok ? D / (16 / esize) : D);
    int64_t g = (items + 255) / 256;
    if (g > (int64_t)cus * 16) g = (int64_t)cus * 16;
    const dim3 grid((unsigned)(g < 1 ? 1 : g));
    if (vec_ok)
        hipLaunchKernelGGL(scatter_rows_kernel<true>, grid, dim3(256), 0, s, T_, B, D, esize, (const char*)src, src_ld,
                           src_off, (char*)dst, dbase, dld);
    else
        hipLaunchKernelGGL(scatter_rows_kernel<false>, grid, dim3(256), 0, s, T_, B, D, esize, (const char*)src,
                           src_ld, src_off, (char*)dst, dbase, dld);
    return ctx_hip(ctx, hipGetLastError(), "scatter_rows launch");
}

}  // namespace dlrm
