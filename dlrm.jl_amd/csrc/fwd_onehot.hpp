// fwd_onehot.hpp -- the one-hot forward body of the feature interaction (maplookup fused with
// DotInteraction, or the interaction on a materialized ys), shared by interact.hip's kernels and by
// the replica probe tools/fwd_probe.hip (so the probe times exactly the shipped code).
// Reference: src/model/interact.jl:271-281 (fast_vcat), :449-467 / :338-362 (process_batches /
// process_slice!), :64-75 (triangular_slice_kernel! pair order).  See interact.hip's header.
#pragma once
#include "common.hpp"

#ifndef WT
#define WT(kind, slot, b) do {} while (0)
#endif

namespace dlrm {

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int kStage = 1024;  // floats of output staging per wave

// ---------------------------------------------------------------------------------- fwd
// Fragment traits: fp32 -> v_mfma_f32_16x16x4_f32 with float4 loads (16 columns per step, 4
// MFMA k-steps, one per component); bf16 -> v_mfma_f32_16x16x32_bf16 with 8-element loads
// (32 columns per step, one MFMA).
template <typename T> struct Frag;
template <> struct Frag<float> {
    typedef f32x4_t type;
    static constexpr int COLS = 16, PER_LANE = 4;
    __device__ static inline type zero() { return type{0.f, 0.f, 0.f, 0.f}; }
    __device__ static inline void mma(f32x4_t& acc, const type& a, const type& b) {
#pragma unroll
        for (int k = 0; k < 4; ++k) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[k], b[k], acc, 0, 0, 0);
    }
    __device__ static inline void add_to(float* f, const type& v) {
#pragma unroll
        for (int k = 0; k < 4; ++k) f[k] += v[k];
    }
    __device__ static inline void to_f(float* f, const type& v) {
#pragma unroll
        for (int k = 0; k < 4; ++k) f[k] = v[k];
    }
    __device__ static inline type from_f(const float* f) { return type{f[0], f[1], f[2], f[3]}; }
};
template <> struct Frag<uint16_t> {
    typedef bf16x8_t type;
    static constexpr int COLS = 32, PER_LANE = 8;
    __device__ static inline type zero() { return type{}; }
    __device__ static inline void mma(f32x4_t& acc, const type& a, const type& b) {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
    __device__ static inline void to_f(float* f, const type& v) {
        const u16x8 u = __builtin_bit_cast(u16x8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] = bf16_to_f32(u[k]);
    }
    __device__ static inline void add_to(float* f, const type& v) {
        float g[8];
        to_f(g, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] += g[k];
    }
    __device__ static inline type from_f(const float* f) {
        u16x8 u;
#pragma unroll
        for (int k = 0; k < 8; ++k) u[k] = f32_to_bf16(f[k]);
        return __builtin_bit_cast(type, u);
    }
};

// Where the embedding rows come from: the ys buffer (the reference's two-operator form), or
// straight from the tables (maplookup fused into the interaction: every gathered row is read
// once into MFMA fragments and written to ys from registers — ys is never read back).
struct GatherArgs {
    const TableDesc* tabs;
    const void* idx;
    int itype;
    int64_t tstride;
    int base;
    int L;
    unsigned* err;
    // backward: when set, table t's dt row of sample b goes to dt + dtb[t] + b * dtl[t] (device
    // arrays; the sharded exchange's per-owner send layout) and dt's x row is not written
    const int64_t* dtb;
    const int64_t* dtl;
};

// One-hot forward (L = 1): every row load of a column block (all UU x NB fragments) is issued
// before the first MFMA, so a wave keeps its whole share of the sample's rows in flight at once.
// The compiler's own schedule interleaved one load, a wait and its MFMAs (one 1-KB load in flight
// per wave: the row stream ran at 2 TB/s); the sched_barriers pin the order
//   index / table loads | row loads | MFMAs | x staging.
// Row 0 of T is x itself: it arrives with the rows, and the output's x head (fast_vcat) is
// staged from those fragments instead of a second load of x.
// Summation order (every forward kernel, so all forms agree bit for bit): for F <= 32 (NB <= 2)
// the Gram tiles are accumulated as two partials, column steps of even and of odd index (a step =
// FR::COLS columns), each in ascending step order, and Z = even + odd; for larger F one chain in
// ascending step order (registers).  WPS = 2 runs the two partials on two waves
// (wave h takes the steps of parity h: half the loads and MFMAs per wave, twice the waves in
// flight; tools/fwd_probe.hip: 10.2 vs 11.5 us at the metric shape), the odd wave's tiles handed
// to the even wave through LDS.
// The staged output row written 4 elements per lane (16-B fp32 stores: a quarter of the store
// instructions of one element per lane); DLRM_FWD_VEC_OUT=0 keeps the scalar stores.
#ifndef DLRM_FWD_VEC_OUT
#define DLRM_FWD_VEC_OUT 1
#endif
constexpr bool kFwdVecOut = DLRM_FWD_VEC_OUT;
template <typename T>
__device__ __forceinline__ void store4(T* p, const f32x4_t& v) {
    if constexpr (sizeof(T) == 4) {
        stg<f32x4_t>((f32x4_t*)p, v);
    } else {
        typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
        u32x2_t u;
        u[0] = (uint32_t)from_f32<T>(v[0]) | ((uint32_t)from_f32<T>(v[1]) << 16);
        u[1] = (uint32_t)from_f32<T>(v[2]) | ((uint32_t)from_f32<T>(v[3]) << 16);
        stg<u32x2_t>((u32x2_t*)p, u);
    }
}

// Elements [lo, hi) of a staged output row (LDS) to orow, 16-B stores between a head (up to the
// row's first 16-B boundary at or after lo) and a tail; lt = this lane's index among the NL lanes.
template <typename T, int NL>
__device__ __forceinline__ void store_staged(T* orow, const float* stage, int lo, int hi, int lt) {
    const int e0 = lo + (int)((4 - (((uintptr_t)(orow + lo) >> 2) & 3)) & 3);
    const int hend = e0 < hi ? e0 : hi;
    if (lo + lt < hend) stg<T>(orow + lo + lt, from_f32<T>(stage[lo + lt]));
    if (e0 >= hi) return;
    const int nv = (hi - e0) >> 2;
    for (int k = lt; k < nv; k += NL) {
        const int e = e0 + 4 * k;
        stg<f32x4_t>((f32x4_t*)(orow + e), f32x4_t{stage[e], stage[e + 1], stage[e + 2], stage[e + 3]});
    }
    const int et = e0 + 4 * nv + lt;
    if (lt < 4 && et < hi) stg<T>(orow + et, from_f32<T>(stage[et]));
}

template <typename T, int NB> struct FwdPart {
    static constexpr int NT = NB * (NB + 1) / 2;  // lower-triangle tiles
};
// TP: the table pointers / row counts from a TabPtrs kernel argument (else from ga.tabs).
// DEFER: raise the bounds flag after the stores instead of where the index is checked.
template <typename T, int NB, bool FUSED, int WPB, int DC = 0, int WPS = 1, bool CONTIG = false, bool TP = false,
          bool DEFER = false>
__device__ __forceinline__ void fwd_body_onehot(int bid, int nblocks, float* stage_all, int d_, int F, int B,
                                                const T* __restrict__ x, int64_t x_ld, T* __restrict__ ys,
                                                int64_t ys_ld, T* __restrict__ out, int64_t out_ld, int padding,
                                                const GatherArgs& ga, const TabPtrs* tp = nullptr) {
    const int d = DC > 0 ? DC : d_;
    typedef Frag<T> FR;
    typedef typename FR::type frag;
    // column steps whose loads are issued together: 128 columns at the compiled feature size, 64
    // otherwise (keeps the generic kernel's registers -- both parity partials live -- unspilled)
    // (larger F: fewer columns per block, so the NB fragments of every column step stay in registers)
    constexpr int CBLK = NB <= 2 ? (DC > 0 ? 128 : 64) : (NB <= 4 ? 64 : 32);
    constexpr int UU = CBLK / FR::COLS > 0 ? CBLK / FR::COLS : 1;
    constexpr int NT = FwdPart<T, NB>::NT;
    constexpr int SPB = WPB / WPS;       // samples per workgroup (per pass)
    static_assert(WPS == 1 || WPS == 2, "one or two waves per sample");
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int pair = w / WPS, h = w % WPS;
    const int c = lane & 15, q = lane >> 4;
    const int P = F * (F - 1) / 2;
    const int W = d + P + padding;
    const bool staged = W <= kStage;
    float* stage = stage_all + pair * kStage;
    // WPS = 2: the odd wave's partial tiles, [pair][NT][64 lanes] f32x4 after the stages
    f32x4_t* xch = (f32x4_t*)(stage_all + SPB * kStage) + pair * NT * 64;
    const T* zero = (const T*)g_zero_row;
    constexpr int ZMASK = kZeroElems * 4 / (int)sizeof(T) - 1;
    // the staged output row leaves as 16-B stores when every row start is aligned for them (fp32 at
    // d = 128: forward 12.1 -> 11.4 us, r8d; at d = 16 and for bf16 rows no gain: scalar stores)
    constexpr bool VEC_OUT = kFwdVecOut && sizeof(T) == 4 && DC >= 128;
    // fp32 rows whose start is not 16-B aligned (W % 4 != 0): 16-B stores between a head and a tail
#ifndef DLRM_FWD_VEC_ROW
#define DLRM_FWD_VEC_ROW 1
#endif
    constexpr bool VEC_ROW = DLRM_FWD_VEC_ROW && sizeof(T) == 4 && DC >= 128;
    // EARLY: the first Gram tile (pairs i < 16) and x go out while the MFMAs of the other two tiles
    // run: tile-outer MFMA order (each tile's summation order unchanged: bit-identical output)
#ifndef DLRM_FWD_EARLY
#define DLRM_FWD_EARLY 0
#endif
    constexpr bool EARLY = DLRM_FWD_EARLY && VEC_ROW && WPS == 1 && !CONTIG && NB == 2 && DC > 0 && DC == CBLK;
    const int F16 = F < 16 ? F : 16;
    const int E1 = d + F16 * (F16 - 1) / 2;  // EARLY: x + the pairs of tile 00
    const bool vec_out = W % 4 == 0 && out_ld % 4 == 0 && ((uintptr_t)out & (4 * sizeof(T) - 1)) == 0;
    bool bad_any = false;  // an out-of-range index was skipped (zero row) by this lane
    for (int64_t b0 = (int64_t)bid * SPB; b0 < B; b0 += (int64_t)nblocks * SPB) {
        const int64_t bs = b0 + pair;
        const bool live = bs < B;
        const int64_t b = live ? bs : B - 1;  // a padding sample (WPS = 2) re-reads a real one, stores nothing
        if (h == 0) WT(0, 0, b);
        const T* xb = x + b * x_ld;
        T* yb = (ys && live) ? ys + b * ys_ld : nullptr;
        T* orow = out + b * out_ld;
        const T* src[NB];
        if (FUSED) {
            // every index and descriptor load first (one round trip), then the checks
            TableDesc td[NB];
            int64_t ri[NB];
#pragma unroll
            for (int I = 0; I < NB; ++I) {
                const int row = I * 16 + c;
                const bool tab = row >= 1 && row < F;
                if constexpr (TP) td[I] = TableDesc{(void*)tp->p[tab ? row - 1 : 0], (int64_t)tp->n[tab ? row - 1 : 0]};
                else td[I] = load_table(ga.tabs, tab ? row - 1 : 0);
                ri[I] = load_index_if(tab, ga.idx, ga.itype, tab ? (row - 1) * ga.tstride + b : 0);
            }
            bool bad = false;
#pragma unroll
            for (int I = 0; I < NB; ++I) {
                const int row = I * 16 + c;
                const bool tab = row >= 1 && row < F;
                const int64_t r = ri[I] - ga.base;
                const bool ok = tab & (r >= 0) & (r < td[I].nrows);
                bad |= tab & !ok;
                src[I] = row == 0 ? xb : (ok ? (const T*)td[I].data + r * d : nullptr);
            }
            if constexpr (DEFER) bad_any |= bad & (q == 0) & (h == 0) & live;
            else if (bad & (q == 0) & (h == 0) & live) raise_index_error(ga.err);
        } else {
#pragma unroll
            for (int I = 0; I < NB; ++I) {
                const int row = I * 16 + c;
                src[I] = row == 0 ? xb : (row < F ? ys + b * ys_ld + (int64_t)row * d : nullptr);
            }
        }
        // acc[p][ij]: partial p (column-step parity) of tile ij; WPS = 2 keeps only its own
        constexpr int NPART = (WPS == 1 && NB <= 2) ? 2 : 1;  // NB > 2: one chain (registers)
        f32x4_t acc[NPART][NT];
#pragma unroll
        for (int pp = 0; pp < NPART; ++pp)
#pragma unroll
            for (int k = 0; k < NT; ++k) acc[pp][k] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        for (int u0 = 0; u0 < d; u0 += UU * FR::COLS) {
            // this wave's column steps of the block: interleaved uu = WPS * v + h, or CONTIG
            // (contiguous halves) uu = h * UV + v
            constexpr int UV = UU / WPS;
            __builtin_amdgcn_sched_barrier(0);
            frag a[UV][NB];
#pragma unroll
            for (int v = 0; v < UV; ++v) {
                const int uu = CONTIG ? h * UV + v : WPS * v + h;
                const int col = u0 + uu * FR::COLS + q * FR::PER_LANE;
                // column steps wholly past d (small d; wave-uniform) issue no load
                if (DC > 0 ? (uu * FR::COLS < DC) : (u0 + uu * FR::COLS < d)) {
#pragma unroll
                    for (int I = 0; I < NB; ++I) {
                        const bool ok = src[I] && col < d;
                        a[v][I] = ldg<frag>(ok ? src[I] + col : zero + (col & ZMASK));
                    }
                } else {
#pragma unroll
                    for (int I = 0; I < NB; ++I) a[v][I] = FR::zero();
                }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int v = 0; v < UV; ++v) {
                const int uu = CONTIG ? h * UV + v : WPS * v + h;
                if (!(DC > 0 ? (uu * FR::COLS < DC) : (u0 + uu * FR::COLS < d))) continue;  // (wave-uniform)
                int ij = 0;
#pragma unroll
                for (int I = 0; I < NB; ++I)
#pragma unroll
                    for (int J = 0; J <= I; ++J, ++ij)
                        if (!EARLY || ij == 0)
                            FR::mma(acc[NPART == 2 ? (CONTIG ? (((u0 + uu * FR::COLS) >> 6) & 1) : (uu & 1)) : 0][ij],
                                    a[v][I], a[v][J]);
            }
            if constexpr (EARLY) {
                // x (fast_vcat) and tile 00's pairs staged and stored now; tiles 10 and 11 after
#pragma unroll
                for (int v = 0; v < UV; ++v) {
                    const int col = u0 + v * FR::COLS + q * FR::PER_LANE;
                    if (c == 0 && col < d) {
                        float f[FR::PER_LANE];
                        FR::to_f(f, a[v][0]);
#pragma unroll
                        for (int k = 0; k < FR::PER_LANE; k += 4)
                            *(f32x4_t*)(stage + col + k) = f32x4_t{f[k], f[k + 1], f[k + 2], f[k + 3]};
                    }
                }
                const f32x4_t z0 = acc[0][0] + acc[NPART - 1][0];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 4 * q + r;
                    if (i < F && c < i) stage[d + i * (i - 1) / 2 + c] = z0[r];
                }
                wave_lds_sync();
                if (live) store_staged<T, 64>(orow, stage, 0, E1, lane);
#pragma unroll
                for (int v = 0; v < UV; ++v) {
                    const int uu = v;
                    if (!(uu * FR::COLS < DC)) continue;
                    FR::mma(acc[NPART == 2 ? (uu & 1) : 0][1], a[v][1], a[v][0]);
                    FR::mma(acc[NPART == 2 ? (uu & 1) : 0][2], a[v][1], a[v][1]);
                }
            }
            // fast_vcat: x (row 0: lanes c == 0 of I = 0) into the output head, and the lookup
            // output ys rows (FUSED with ys kept), from the fragments (after the MFMAs, so the MFMAs
            // wait for their own loads only)
#pragma unroll
            for (int v = 0; v < UV; ++v) {
                const int uu = CONTIG ? h * UV + v : WPS * v + h;
                const int col = u0 + uu * FR::COLS + q * FR::PER_LANE;
                if (col < d && live) {
                    if (c == 0 && !EARLY) {
                        float f[FR::PER_LANE];
                        FR::to_f(f, a[v][0]);
                        if (staged) {
#pragma unroll
                            for (int k = 0; k < FR::PER_LANE; k += 4)
                                *(f32x4_t*)(stage + col + k) = f32x4_t{f[k], f[k + 1], f[k + 2], f[k + 3]};
                        } else {
#pragma unroll
                            for (int k = 0; k < FR::PER_LANE; ++k) stg<T>(orow + col + k, from_f32<T>(f[k]));
                        }
                    }
                    if (c == 0 && yb) stg<frag>(yb + col, a[v][0]);
                    if (FUSED && yb) {
#pragma unroll
                        for (int I = 0; I < NB; ++I) {
                            const int row = I * 16 + c;
                            if (row >= 1 && row < F) stg<frag>(yb + (int64_t)row * d + col, a[v][I]);
                        }
                    }
                }
            }
        }
        if (h == 0) WT(0, 1, b);
        // Z = even + odd partials
        f32x4_t z[NT];
        if constexpr (WPS == 1 && NPART == 1) {
#pragma unroll
            for (int k = 0; k < NT; ++k) z[k] = acc[0][k];
        } else if constexpr (WPS == 1) {
#pragma unroll
            for (int k = 0; k < NT; ++k) z[k] = acc[0][k] + acc[NPART - 1][k];
        } else {
            if (h == 1)
#pragma unroll
                for (int k = 0; k < NT; ++k) xch[k * 64 + lane] = acc[0][k];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < NT; ++k) z[k] = acc[0][k] + xch[k * 64 + lane];
        }
        // Z[i][j], i > j: triangular_slice_kernel! order (i-major), after x
        if (h == 0 && live) {
            int ij = 0;
#pragma unroll
            for (int I = 0; I < NB; ++I)
#pragma unroll
                for (int J = 0; J <= I; ++J, ++ij) {
                    if (EARLY && ij == 0) continue;  // (staged and stored already)
                    const int j = J * 16 + c;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = I * 16 + 4 * q + r;
                        if (i < F && j < i) {
                            const int e = d + i * (i - 1) / 2 + j;
                            if (staged) stage[e] = z[ij][r];
                            else stg<T>(orow + e, from_f32<T>(z[ij][r]));
                        }
                    }
                }
            for (int e = d + P + lane; e < W; e += 64) {
                if (staged) stage[e] = 0.0f;
                else stg<T>(orow + e, from_f32<T>(0.0f));
            }
        }
        if (staged) {
            if constexpr (WPS == 1) wave_lds_sync(); else __syncthreads();
            if (live && VEC_OUT && vec_out) {
                for (int e = 4 * (lane + 64 * h); e < W; e += 256 * WPS) store4<T>(orow + e, *(const f32x4_t*)(stage + e));
            } else if (live && VEC_ROW) {
                // rows of W = d + P floats start at any 4-B boundary (479 at the metric config): the
                // head elements up to the row's first 16-B boundary, then 16-B stores of the staged
                // row (read from LDS as four floats), then the tail (EARLY: [E1, W) only)
                store_staged<T, 64 * WPS>(orow, stage, EARLY ? E1 : 0, W, lane + 64 * h);
            } else if (live) {
                for (int e = lane + 64 * h; e < W; e += 64 * WPS) stg<T>(orow + e, from_f32<T>(stage[e]));
            }
            if constexpr (WPS == 1) wave_lds_sync(); else __syncthreads();
        } else if constexpr (WPS == 2) {
            __syncthreads();  // xch is rewritten by the next pass
        }
        if (h == 0) WT(0, 2, b);
    }
    if (DEFER && bad_any) raise_index_error(ga.err);
}

}  // namespace dlrm
