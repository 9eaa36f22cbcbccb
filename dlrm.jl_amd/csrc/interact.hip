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
#include <cstdlib>
#include <type_traits>

#include "common.hpp"

#ifdef DLRM_PHASE
// Phase timestamps of the split indexer inside the step forward's launch (table DLRM_PHASE);
// only in the profiling variant of the library (tools/phase_stepfwd.py).
__device__ unsigned long long g_phase_fwd[64];
#define PHASE(k) do { __syncthreads(); if (blockIdx.x == DLRM_PHASE && threadIdx.x == 0) g_phase_fwd[k] = wall_clock64(); } while (0)
extern "C" int dlrm_debug_phase_fwd(unsigned long long* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_fwd), sizeof(g_phase_fwd));
}
extern "C" int dlrm_debug_phase_fwd_reset(void) {
    static unsigned long long z[64];
    for (int k = 0; k < 64; ++k) z[k] = (k == 60 || k == 62) ? ~0ull : 0ull;
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_phase_fwd), z, sizeof(z));
}
#endif
#include "indexer.hpp"

#ifdef DLRM_WTRACE
// Per-sample wave timestamps (wall_clock64, 100 MHz) of the forward (kind 0) and backward
// (kind 1) bodies; only in the tracing build (tools/wave_trace.sh).
__device__ unsigned long long g_wt[2][6][8192];
#define WT(kind, slot, b) do { if ((threadIdx.x & 63) == 0 && (b) < 8192) g_wt[kind][slot][b] = wall_clock64(); } while (0)
extern "C" int dlrm_debug_wtrace(unsigned long long* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wt), sizeof(g_wt));
}
#else
#define WT(kind, slot, b) do {} while (0)
#endif

#include "fwd_onehot.hpp"

namespace dlrm {

// Workgroup `bid` of `nblocks` (WPB waves, one sample per wave); stage_all = WPB * kStage floats of LDS.
// The fused one-hot forward of F <= 32 features reads its table pointers from a TabPtrs kernel
// argument (fwd_onehot.hpp); kDeferRaise: its bounds flag is raised after the stores.
#ifndef DLRM_DEFER_RAISE
#define DLRM_DEFER_RAISE 1
#endif
constexpr bool kDeferRaise = DLRM_DEFER_RAISE;
template <int NB, bool FUSED, bool POOL> constexpr bool fwd_tab_ptrs() { return FUSED && !POOL && NB <= 2; }

template <typename T, int NB, bool FUSED, int WPB, bool POOL = false, int DC = 0>
__device__ __forceinline__ void fwd_body(int bid, int nblocks, float* stage_all, int d_, int F, int B,
                                         const T* __restrict__ x, int64_t x_ld, T* __restrict__ ys, int64_t ys_ld,
                                         T* __restrict__ out, int64_t out_ld, int padding, const GatherArgs& ga,
                                         const TabPtrs* tp = nullptr) {
    // !POOL: one lookup per (table, sample) -- the callers pick the POOL kernel for FUSED, L > 1
    if constexpr (!POOL) {
        // one wave per sample: with the table pointers in the kernel arguments it beats two waves per
        // sample (column halves) at d = 128 -- tools/fwd_probe.hip: 10.5 vs 11.9 us
        constexpr int WPS = 1;
        constexpr bool TP = fwd_tab_ptrs<NB, FUSED, POOL>();
        fwd_body_onehot<T, NB, FUSED, WPB, DC, WPS, false, TP, kDeferRaise && TP>(
            bid, nblocks, stage_all, d_, F, B, x, x_ld, ys, ys_ld, out, out_ld, padding, ga, tp);
        return;
    }
    const int d = DC > 0 ? DC : d_;  // DC: the feature size as a compile-time constant
    typedef Frag<T> FR;
    typedef typename FR::type frag;
    constexpr int UU = 128 / FR::COLS;  // column steps whose loads are issued together (128 columns)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 15, q = lane >> 4;
    const int P = F * (F - 1) / 2;
    const int W = d + P + padding;
    const bool staged = W <= kStage;
    float* stage = stage_all + w * kStage;
    for (int64_t b = (int64_t)bid * WPB + w; b < B; b += (int64_t)nblocks * WPB) {
        WT(0, 0, b);
        const T* xb = x + b * x_ld;
        T* yb = ys ? ys + b * ys_ld : nullptr;  // FUSED: ys may be NULL (not materialized)
        T* orow = out + b * out_ld;
        // fast_vcat: x into the reserved rows of ys; x is also the head of the output row.
        for (int i = lane; i < d; i += 64) {
            const T v = ldg<T>(xb + i);
            if (yb) stg<T>(yb + i, v);
            if (staged) stage[i] = to_f32(v);
            else stg<T>(orow + i, v);
        }
        // row sources: feature 0 is x itself; features 1..F-1 are ys rows or table rows.  Every
        // load below executes unconditionally (invalid slots read x and are masked to zero), so
        // no branch makes the compiler wait for a lane's loads one at a time.
        const T* src[NB];
        int64_t kidx[NB];  // FUSED, pooled: index position of lookup 0 of this (table, sample)
        TableDesc td[NB];
#pragma unroll
        for (int I = 0; I < NB; ++I) {
            const int row = I * 16 + c;
            const bool tab = FUSED && row >= 1 && row < F;
            kidx[I] = tab ? (row - 1) * ga.tstride + b * ga.L : -1;
            td[I] = FUSED ? load_table(ga.tabs, tab ? row - 1 : 0) : TableDesc{};
            const int64_t r = load_index_if(tab, ga.idx, ga.itype, kidx[I]) - ga.base;
            const bool ok = tab & (r >= 0) & (r < td[I].nrows);
            if (tab & !ok & (q == 0)) raise_index_error(ga.err);
            src[I] = row == 0 ? xb
                              : (!FUSED ? (row < F ? yb + (int64_t)row * d : nullptr)
                                        : (ok ? (const T*)td[I].data + r * d : nullptr));
        }
        f32x4_t acc2[NB <= 2 ? 2 : 1][NB * (NB + 1) / 2];  // NB <= 2: parity partials (fwd_body_onehot's order)
#pragma unroll
        for (int k = 0; k < NB * (NB + 1) / 2; ++k) acc2[0][k] = acc2[NB <= 2 ? 1 : 0][k] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        for (int u0 = 0; u0 < d; u0 += UU * FR::COLS) {
            frag a[UU][NB];
#pragma unroll
            for (int uu = 0; uu < UU; ++uu) {
                const int col = u0 + uu * FR::COLS + q * FR::PER_LANE;
#pragma unroll
                for (int I = 0; I < NB; ++I) {
                    const bool ok = src[I] && col < d;
                    // F <= 32, one-hot: column steps past d (small d, wave-uniform) issue no load at all
                    // (D = 16: 9.5 vs 11.0 us).  Not in the pooled or NB > 2 kernels, where the branches
                    // halve the loads kept in flight (the NB = 5 forward: 105 vs 72 us at d = 256).
                    const frag v = (POOL || NB > 2 || u0 + uu * FR::COLS < d)
                                       ? ldg<frag>((ok ? src[I] : xb) + (ok ? col : 0))
                                       : FR::zero();
                    a[uu][I] = ok ? v : FR::zero();
                }
            }
            if (FUSED) {
                // pooled bags: add lookups 1..L-1 in k order (fp32), round once to T
                if (POOL && ga.L > 1) {
#pragma unroll
                    for (int I = 0; I < NB; ++I) {
                        const bool tab = kidx[I] >= 0;
                        float f[UU][FR::PER_LANE];
#pragma unroll
                        for (int uu = 0; uu < UU; ++uu) FR::to_f(f[uu], a[uu][I]);
#pragma unroll 4
                        for (int k = 1; k < ga.L; ++k) {
                            const int64_t r = load_index_if(tab, ga.idx, ga.itype, kidx[I] + k) - ga.base;
                            const bool ok = tab & (r >= 0) & (r < td[I].nrows);
                            if (tab & !ok & (q == 0) & (u0 == 0)) raise_index_error(ga.err);
                            const T* rp = ok ? (const T*)td[I].data + r * d : xb;
#pragma unroll
                            for (int uu = 0; uu < UU; ++uu) {
                                const int col = u0 + uu * FR::COLS + q * FR::PER_LANE;
                                const bool okc = ok && col < d;
                                const frag v = ldg<frag>(rp + (okc ? col : 0));
                                FR::add_to(f[uu], okc ? v : FR::zero());
                            }
                        }
#pragma unroll
                        for (int uu = 0; uu < UU; ++uu) a[uu][I] = FR::from_f(f[uu]);
                    }
                }
                // the lookup output: ys rows 1..F-1 written from the fragments
                if (yb)
#pragma unroll
                for (int uu = 0; uu < UU; ++uu) {
                    const int col = u0 + uu * FR::COLS + q * FR::PER_LANE;
#pragma unroll
                    for (int I = 0; I < NB; ++I) {
                        const int row = I * 16 + c;
                        if (row >= 1 && row < F && col < d) stg<frag>(yb + (int64_t)row * d + col, a[uu][I]);
                    }
                }
            }
#pragma unroll
            for (int uu = 0; uu < UU; ++uu) {
                int ij = 0;
#pragma unroll
                for (int I = 0; I < NB; ++I)
#pragma unroll
                    for (int J = 0; J <= I; ++J, ++ij) FR::mma(acc2[NB <= 2 ? (uu & 1) : 0][ij], a[uu][I], a[uu][J]);
            }
        }
        f32x4_t acc[NB * (NB + 1) / 2];
#pragma unroll
        for (int k = 0; k < NB * (NB + 1) / 2; ++k) acc[k] = NB <= 2 ? acc2[0][k] + acc2[1][k] : acc2[0][k];
        WT(0, 1, b);
        // Z[i][j], i > j: triangular_slice_kernel! order (i-major), after x
        {
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
                            else stg<T>(orow + e, from_f32<T>(acc[ij][r]));
                        }
                    }
                }
        }
        for (int e = d + P + lane; e < W; e += 64) {
            if (staged) stage[e] = 0.0f;
            else stg<T>(orow + e, from_f32<T>(0.0f));
        }
        if (staged) {
            wave_lds_sync();
            for (int e = lane; e < W; e += 64) stg<T>(orow + e, from_f32<T>(stage[e]));
            wave_lds_sync();
        }
        WT(0, 2, b);
    }
}

// POOL: the pooled-bag path (lookups > 1) is compiled in; the one-hot kernel stays lean.
template <typename T, int NB, bool FUSED, bool POOL, int DC = 0, int WPB = 4>
__global__ __launch_bounds__(64 * WPB, 2) void interact_fwd_kernel(int d, int F, int B, const T* __restrict__ x,
                                                                   int64_t x_ld, T* __restrict__ ys, int64_t ys_ld,
                                                                   T* __restrict__ out, int64_t out_ld, int padding,
                                                                   GatherArgs ga, TabPtrs tp) {
    __shared__ __attribute__((aligned(16))) float stage_all[WPB * kStage];
    fwd_body<T, NB, FUSED, WPB, POOL, DC>(blockIdx.x, gridDim.x, stage_all, d, F, B, x, x_ld, ys, ys_ld, out, out_ld, padding,
                                ga, &tp);
}

// The forward of a training step with the SparseIndexer build in the same grid (split form:
// once-hit positions flagged for the backward, the rest listed for the apply): the first
// T << ix.vshift workgroups sort the tables' positions (indexer.hpp, 256 threads; with
// vshift = 1 two per table, one per row parity, which halves the critical path), the rest run
// the fused lookup + interaction without ys.  The indexer depends only on the indices, so it
// streams beside the gather instead of adding a launch.
// (StepLds, kStepIndexEPL: indexer.hpp)
template <typename T, int NB, int DC = 0>
__global__ __launch_bounds__(256, 3) void interact_fwd_index_kernel(int d, int F, int B, const T* __restrict__ x,
                                                                 int64_t x_ld, T* __restrict__ out, int64_t out_ld,
                                                                 int padding, GatherArgs ga, IndexerDev ix,
                                                                 TabPtrs tp) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int T_ = F - 1;
    // vshift >= 2: the wave build (indexer.hpp wave_build_group: 4 parts per workgroup, one wave
    // each, and the flat item map); else the block build, one workgroup per table part
    const bool wave = ix.vshift >= 2;
    const int NI = wave ? (T_ << ix.vshift) / kWaveParts : T_ << ix.vshift;
#ifdef DLRM_PHASE
    // [0] this block's start (the traced indexer block), [60] / [61] first start / last end of any
    // gather block, [62] / [63] first start / last end of any indexer block
    if (threadIdx.x == 0) {
        const unsigned long long t0 = wall_clock64();
        if ((int)blockIdx.x == DLRM_PHASE) g_phase_fwd[0] = t0;
        atomicMin(&g_phase_fwd[(int)blockIdx.x < NI ? 62 : 60], t0);
    }
#endif
    if ((int)blockIdx.x < NI) {
        if (wave) {
            wave_build_group<false>(ix, blockIdx.x, T_, ga.tabs, ga.idx, ga.itype, ga.tstride, ga.base, B * ga.L, ga.err,
                             *(WaveBuildLds*)smem);
        } else {
            StepLds& sl = *(StepLds*)smem;
            const int v = blockIdx.x, t = v >> ix.vshift;
            fast_index_table<256, kStepIndexEPL, true>(ix, v, t, ix.vshift, (uint32_t)ga.tabs[t].nrows, ga.idx,
                                                       ga.itype, ga.tstride, ga.base, B * ga.L, ga.err, sl);
        }
#ifdef DLRM_PHASE
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(&g_phase_fwd[63], wall_clock64());
#endif
        return;
    }
    fwd_body<T, NB, true, 4, false, DC>(blockIdx.x - NI, gridDim.x - NI, smem, d, F, B, x, x_ld, nullptr, 0, out,
                                        out_ld, padding, ga, &tp);
#ifdef DLRM_PHASE
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&g_phase_fwd[61], wall_clock64());
#endif
}

// ---------------------------------------------------------------------------------- bwd
template <int NB> struct BwdGeom {
    static constexpr int NS = 16 * NB;                          // padded features
    static constexpr int SS = NS + ((NB % 2 == 0) ? 16 : 0);    // row stride = 16 (mod 32)
    static constexpr int WPB = NB <= 2 ? 4 : (NB <= 4 ? 2 : 1); // waves per block
    static constexpr int LDS_FLOATS = NS * SS;                  // per wave: S
    // per wave, with the UPD T tile ([NS][64] floats of one super-block) after S
    template <bool UPD> static constexpr int lds_floats() { return NS * SS + (UPD ? NS * 64 : 0); }
};

// 4 consecutive elements of T as fp32 (16-B load for fp32, 8-B for bf16)
__device__ __forceinline__ f32x4_t load4_f32(const float* p) { return ldg<f32x4_t>(p); }
__device__ __forceinline__ f32x4_t load4_f32(const uint16_t* p) {
    const uint2 v = ldg<uint2>(p);
    return f32x4_t{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u), __uint_as_float(v.y << 16),
                   __uint_as_float(v.y & 0xffff0000u)};
}

// dT = S T per sample, in 64-column super-blocks: lane (c, q) loads T[4s+q][64sb+4c .. +3]
// (16 lanes read 256 contiguous bytes of a row), and component e of that float4 is the B
// operand of the MFMA that produces output columns 64sb + 4j + e.  The four accumulators of
// a tile row then hold 4 consecutive output columns per lane -> one float4 store per row.
// All k-step loads of a super-block are issued before its MFMAs (up to 4*NB in flight).
// GATHER: T_b is not read from a materialized ys but rebuilt from x (row 0) and the table
// rows of the sample's one-hot indices (rows 1..F-1): the same values, without ys.
// UPD (training step, split indexer): a table row hit by this sample only (single[] flag of
// the forward's indexer build) gets its SGD step here -- w = fmaf(-lr, 0 + g, w), exactly the
// apply kernel's arithmetic for a one-position segment -- and its dt row is not written.  No
// other sample reads that row, so the in-place update cannot race with another wave's gather.
struct StepUpdate {
    const uint8_t* single;  // [T][cap]
    int64_t cap;
    float lr;
    const unsigned* err;    // the ctx's bounds flag: set -> no table row is written (the row goes to dt)
};

template <typename T, int NB, bool GATHER, bool UPD = false, int SBU_ = 0, int DC = 0>
__device__ __forceinline__ void bwd_body(int bid, int nblocks, float* smem, int d_, int F, int B,
                                         const T* __restrict__ dout, int64_t dout_ld, const T* __restrict__ t,
                                         int64_t t_ld, float* __restrict__ dx, int64_t dx_ld,
                                         float* __restrict__ dt, int64_t dt_ld, const GatherArgs& ga,
                                         const T* __restrict__ x, int64_t x_ld, const StepUpdate& su = StepUpdate{}) {
    const int d = DC > 0 ? DC : d_;  // DC: the feature size as a compile-time constant
    typedef BwdGeom<NB> G;
    constexpr int KS = 4 * NB;          // max k-steps (F <= 16 NB)
    constexpr int SBU = SBU_ > 0 ? SBU_ : (NB <= 2 ? 2 : 1);  // 64-column super-blocks loaded together
    constexpr int KPB = 8;              // packed-gradient values per lane loaded together
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // the table descriptors, once per workgroup, in LDS after the waves' regions: read where
    // used instead of held in registers across the index loads
    TableDesc* tds = (TableDesc*)(smem + G::WPB * G::template lds_floats<UPD>());
    int64_t* dmap = (int64_t*)(tds + (F - 1));  // GATHER + ga.dtb: [2][F-1] row bases / strides of dt
    if (GATHER) {
        for (int t = threadIdx.x; t < F - 1; t += blockDim.x) {
            tds[t] = load_table(ga.tabs, t);
            if (ga.dtb) {
                dmap[t] = ga.dtb[t];
                dmap[F - 1 + t] = ga.dtl[t];
            }
        }
        __syncthreads();
    }
    const bool mapped = GATHER && ga.dtb;
    if (w >= G::WPB) return;
    const int c = lane & 15, q = lane >> 4;
    float* S = smem + w * G::template lds_floats<UPD>();
    float* Tt = S + G::NS * G::SS;  // UPD: the current super-block of T, [NS][64]
    const int P = F * (F - 1) / 2;
    const int ksteps = (F + 3) / 4;
    for (int64_t b = (int64_t)bid * G::WPB + w; b < B; b += (int64_t)nblocks * G::WPB) {
        WT(1, 0, b);
        const T* ob = dout + b * dout_ld;
        const T* tb = GATHER ? nullptr : t + b * t_ld;
        // Independent loads first, so their latencies overlap: the sample's indices (T rows and,
        // UPD, the once-hit flags of its output rows) and the first packed-gradient values.
        const T* rowp[KS];  // GATHER: this lane's T rows kk = 4s + q
        if (GATHER) {
            int64_t ri[KS];
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const int kk = 4 * s + q;
                const bool tab = s < ksteps && kk >= 1 && kk < F;
                ri[s] = load_index_if(tab, ga.idx, ga.itype, (kk - 1) * ga.tstride + b * ga.L);
            }
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const int kk = 4 * s + q;
                const bool tab = s < ksteps && kk >= 1 && kk < F;
                const TableDesc td = tds[tab ? kk - 1 : 0];
                const int64_t r = ri[s] - ga.base;
                const bool ok = tab & (r >= 0) & (r < td.nrows);
                if (tab & !ok & (c == 0)) raise_index_error(ga.err);
                rowp[s] = (s < ksteps && kk == 0) ? x + b * x_ld : (ok ? (const T*)td.data + r * d : nullptr);
            }
        }
        uint32_t urow[NB][4];  // UPD: the once-hit table row of output row f = 16I + 4q + r, else ~0u
        if (UPD) {
            // a bounds error of this step (raised by the forward): the reference's gather throws
            // before update!, so every row goes to dt and the apply (which checks too) writes none
            const bool frozen = *su.err != 0;
            if (b == 0 && lane == 0) snapshot_error(su.err, frozen ? 1u : 0u);
            uint8_t fl[NB][4];
            int64_t ui[NB][4];
#pragma unroll
            for (int I = 0; I < NB; ++I)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int f = I * 16 + 4 * q + r;
                    const bool tab = f >= 1 && f < F;
                    fl[I][r] = ldg<uint8_t>(su.single + (tab ? (int64_t)(f - 1) * su.cap + b : 0));
                    ui[I][r] = load_index_if(tab, ga.idx, ga.itype, (f - 1) * ga.tstride + b);
                }
#pragma unroll
            for (int I = 0; I < NB; ++I)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int f = I * 16 + 4 * q + r;
                    const bool tab = f >= 1 && f < F;
                    const TableDesc td = tds[tab ? f - 1 : 0];
                    const int64_t rr = ui[I][r] - ga.base;
                    urow[I][r] = (tab & !frozen & (fl[I][r] != 0) & (rr >= 0) & (rr < td.nrows)) ? (uint32_t)rr : ~0u;
                }
        }
        // The first super-blocks' T rows (and dout's x part) go out before S is built, so their
        // latency overlaps the packed-gradient loads and the LDS scatter.
        f32x4_t bv[SBU][KS];
        f32x4_t xo[SBU];
        // every lane's T row pointer is valid (ob, the dout row, stands in for a missing row) and
        // `live` masks the values, so the loads are plain base + offset with no selects
        unsigned live = 0;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int kk = 4 * s + q;
            const T* src = GATHER ? rowp[s] : (kk < F ? tb + (int64_t)kk * d : nullptr);
            live |= (s < ksteps && src) ? (1u << s) : 0u;
            rowp[s] = (s < ksteps && src) ? src : ob;
        }
        auto load_batch = [&](int sb0) {
#pragma unroll
            for (int h = 0; h < SBU; ++h) {
                const int n0 = sb0 + 64 * h + 4 * c;
                const int nc = n0 < d ? n0 : 0;
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    const f32x4_t v = load4_f32(rowp[s] + nc);
                    bv[h][s] = ((live >> s) & 1u) && n0 < d ? v : f32x4_t{0.f, 0.f, 0.f, 0.f};
                }
                const int nx = n0 < d ? n0 : 0;  // dout rows need no alignment: scalar reads
                xo[h] = f32x4_t{to_f32(ldg<T>(ob + nx)), to_f32(ldg<T>(ob + nx + 1)), to_f32(ldg<T>(ob + nx + 2)),
                                to_f32(ldg<T>(ob + nx + 3))};
            }
        };
        load_batch(0);
        // S: zero, then scatter the packed pairs to both triangles (fused unpack + transpose-add);
        // KPB values per lane in flight
        for (int e = lane; e < G::NS * G::NS; e += 64) S[(e / G::NS) * G::SS + (e % G::NS)] = 0.0f;
        wave_lds_sync();
        for (int p0 = 0; p0 < P; p0 += 64 * KPB) {
            float dv[KPB];
#pragma unroll
            for (int k = 0; k < KPB; ++k) {
                const int p = p0 + 64 * k + lane;
                const float v = to_f32(ldg<T>(ob + d + (p < P ? p : 0)));
                dv[k] = p < P ? v : 0.0f;
            }
#pragma unroll
            for (int k = 0; k < KPB; ++k) {
                const int p = p0 + 64 * k + lane;
                if (p < P) {
                    int i = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)p)) * 0.5f);
                    while (i * (i - 1) / 2 > p) --i;
                    while ((i + 1) * i / 2 <= p) ++i;
                    const int j = p - i * (i - 1) / 2;
                    S[i * G::SS + j] = dv[k];
                    S[j * G::SS + i] = dv[k];
                }
            }
        }
        wave_lds_sync();
        WT(1, 1, b);
        for (int sb0 = 0; sb0 < d; sb0 += 64 * SBU) {
            if (sb0 > 0) load_batch(sb0);
#pragma unroll
            for (int h = 0; h < SBU; ++h) {
                const int sb = sb0 + 64 * h;
                if (sb >= d) break;
                const int n0 = sb + 4 * c;  // this lane's 4 output columns
                const bool colok = n0 < d;
                if (UPD) {  // stage the super-block's T rows: the update needs row f where dt row f is
                    wave_lds_sync();
#pragma unroll
                    for (int s = 0; s < KS; ++s) {
                        const int kk = 4 * s + q;
                        if (s < ksteps && kk < F) *(f32x4_t*)(Tt + kk * 64 + 4 * c) = bv[h][s];
                    }
                    wave_lds_sync();
                }
                f32x4_t acc[NB][4];
#pragma unroll
                for (int I = 0; I < NB; ++I)
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[I][e] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    if (s < ksteps) {
                        const int kk = 4 * s + q;
#pragma unroll
                        for (int I = 0; I < NB; ++I) {
                            const float av = S[kk * G::SS + I * 16 + c];  // = S[16I+c][kk] (symmetric)
#pragma unroll
                            for (int e = 0; e < 4; ++e)
                                acc[I][e] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[h][s][e], acc[I][e], 0, 0, 0);
                        }
                    }
                }
                if (sb < 128) WT(1, 2 + sb / 64, b);
                if (colok) {
#pragma unroll
                    for (int I = 0; I < NB; ++I)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int f = I * 16 + 4 * q + r;
                            if (f < F) {
                                const f32x4_t v = f32x4_t{acc[I][0][r], acc[I][1][r], acc[I][2][r], acc[I][3][r]};
                                if (UPD && urow[I][r] != ~0u) {
                                    const f32x4_t tw = *(const f32x4_t*)(Tt + f * 64 + 4 * c);
                                    float wv[4];
#pragma unroll
                                    for (int e = 0; e < 4; ++e) wv[e] = __builtin_fmaf(-su.lr, 0.0f + v[e], tw[e]);
                                    store_row<T, 4>((T*)tds[f - 1].data + (int64_t)urow[I][r] * d, n0, wv);
                                } else if (!mapped) {
                                    stg<f32x4_t>(dt + b * dt_ld + (int64_t)f * d + n0, v);
                                } else if (f > 0) {
                                    stg<f32x4_t>(dt + dmap[f - 1] + b * dmap[F - 2 + f] + n0, v);
                                }
                                if (f == 0) stg<f32x4_t>(dx + b * dx_ld + n0, xo[h] + v);
                            }
                        }
                }
            }
        }
        WT(1, 4, b);
        wave_lds_sync();
    }
}

template <typename T, int NB, bool GATHER>
__global__ __launch_bounds__(256, 2) void interact_bwd_kernel(int d, int F, int B, const T* __restrict__ dout,
                                                           int64_t dout_ld, const T* __restrict__ t, int64_t t_ld,
                                                           float* __restrict__ dx, int64_t dx_ld,
                                                           float* __restrict__ dt, int64_t dt_ld, GatherArgs ga,
                                                           const T* __restrict__ x, int64_t x_ld) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    bwd_body<T, NB, GATHER>(blockIdx.x, gridDim.x, smem, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld, ga,
                            x, x_ld);
}

// The backward of a training step with the SparseIndexer build in the same grid: workgroups
// [0, T) each sort one table's positions (indexer.hpp, 256 threads, while the backward's
// workgroups stream), the rest run the re-gathering backward.  Occupancy 3 per SIMD leaves
// room for the indexer's workgroups beside the backward's two per CU.
constexpr int kBwdIndexEPL = 8;  // positions per thread: N <= 2048
template <typename T, int NB>
__global__ __launch_bounds__(256, 3) void interact_bwd_index_kernel(int d, int F, int B, const T* __restrict__ dout,
                                                                    int64_t dout_ld, float* __restrict__ dx,
                                                                    int64_t dx_ld, float* __restrict__ dt,
                                                                    int64_t dt_ld, GatherArgs ga,
                                                                    const T* __restrict__ x, int64_t x_ld,
                                                                    IndexerDev ix) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int T_ = F - 1;
    if ((int)blockIdx.x < T_) {
        FastLds<256, kBwdIndexEPL>& sl = *(FastLds<256, kBwdIndexEPL>*)smem;
        fast_index_table<256, kBwdIndexEPL>(ix, blockIdx.x, blockIdx.x, 0, (uint32_t)ga.tabs[blockIdx.x].nrows,
                                            ga.idx, ga.itype, ga.tstride, ga.base, B * ga.L, ga.err, sl);
        return;
    }
    bwd_body<T, NB, true, false, 1>(blockIdx.x - T_, gridDim.x - T_, smem, d, F, B, dout, dout_ld, nullptr, 0, dx, dx_ld, dt,
                          dt_ld, ga, x, x_ld);
}

// The backward of a training step after interact_fwd_index_kernel: re-gathers T, writes dx
// and the dt rows of positions whose row is hit more than once, and applies the SGD step to
// once-hit rows itself (the apply launch that follows handles the rest).
template <typename T, int NB, int SBU, int DC = 0>
__global__ __launch_bounds__(256, 2) void interact_bwd_update_kernel(int d, int F, int B, const T* __restrict__ dout,
                                                                  int64_t dout_ld, float* __restrict__ dx,
                                                                  int64_t dx_ld, float* __restrict__ dt, int64_t dt_ld,
                                                                  GatherArgs ga, const T* __restrict__ x, int64_t x_ld,
                                                                  StepUpdate su) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    bwd_body<T, NB, true, true, SBU, DC>(blockIdx.x, gridDim.x, smem, d, F, B, dout, dout_ld, nullptr, 0, dx, dx_ld,
                                         dt, dt_ld, ga, x, x_ld, su);
}

// The training step's backward with each sample split over TWO waves by column halves (wave h
// takes the 64-column super-blocks sb = h, h + 2, ...): every wave's dependent chain (indices ->
// rows -> MFMA -> stores) is half as long and needs about half the registers, so four waves per
// SIMD stay resident (B = 2048: all 4096 waves at once) instead of two.  The math per
// super-block is bwd_body's MFMA sequence, so dx, dt and the tables are bit-identical to
// interact_bwd_update_kernel's.
// This path is bound by the vector-memory INSTRUCTION rate of a CU as much as by bytes, so a wave
// issues few loads:
//  - lane t < T loads table t's index and once-hit flag for the sample (one instruction each),
//    validates it and shuffles the row to the lanes that need it (ds_bpermute, not the TA);
//  - the packed pair gradients dout[b][d : d + P] are staged in LDS by the pair's two waves
//    with contiguous loads, and the MFMA A operand S[i][j] is read from there by pair index (no
//    S matrix, no scatter);
//  - dout's x part (dx = dout_x + dt row 0) is one coalesced load of the wave's 64 columns,
//    redistributed by shuffles;
//  - a once-hit row's old value comes from the gathered rows, moved from the B-operand layout
//    (lane (c, q): row 4s + q) to the accumulator layout (row 16I + 4q + r) through the wave's
//    LDS tile, not re-read from HBM.
// One block = SPB samples (WPS·SPB waves; grid = ceil(B / SPB)), one pass: both barriers are
// reached by every wave.  Larger blocks shorten the dispatch ramp (fewer workgroups to place).
// WPS = 1 (d <= 64, one super-block): one wave per sample, the same per-sample load plan --
// the bwd_body kernel's per-lane index / flag loads (KS + 8 NB instructions before the rows)
// are most of a small-d backward's time.
// MAPPED (dlrm_interact_bwd_blocked): table rows' gradients go to the send layout (GatherArgs dtb /
// dtl), none to dt's x row; a separate instantiation, so the step kernels keep their LDS budget.
// CPL = 8 (bf16 rows): a lane loads 8 columns (16 B) of each row and runs 8 MFMAs per k-step, so
// a super-block is 128 columns and one wave takes a d = 128 sample whole (half the load
// instructions per byte of the 4-column form, and more samples resident per CU); the gathered
// rows stay bf16 in the wave's LDS tile.  Every output element is the same MFMA sum over the same
// k-steps as in the 4-column form: dx, dt and the tables are bit-identical.
// YS (dlrm_interact_bwd on a materialized ys, e.g. pooled bags): T row kk of sample b is ys row
// x + b * x_ld + kk * d (x / x_ld carry ys / ys_ld), no index, flag or once-hit update; every dt row
// is written.  Up to 96 features (NB <= 6): the gather-free backward of the pooled workload
// (F = 65), one wave per 64-column super-block.
template <typename T, int NB, int DC, int SPB, int WPS = 2, bool MAPPED = false, int CPL = 4, bool YS = false>
__global__ __launch_bounds__(64 * WPS * SPB, CPL == 8 ? 3 : (NB > 2 ? 2 : 4)) void interact_bwd_split_kernel(int d_, int F, int B, const T* __restrict__ dout,
                                                                   int64_t dout_ld, float* __restrict__ dx,
                                                                   int64_t dx_ld, float* __restrict__ dt,
                                                                   int64_t dt_ld, GatherArgs ga,
                                                                   const T* __restrict__ x, int64_t x_ld,
                                                                   StepUpdate su) {
    static_assert(CPL == 4 || (CPL == 8 && sizeof(T) == 2), "8 columns per lane: bf16 rows");
    constexpr int NS = 16 * NB;
    constexpr int KS = 4 * NB;
    constexpr int PMAX = NS * (NS - 1) / 2;
    constexpr int SBC = 16 * CPL;  // columns per super-block
    // the wave's tile of T: fp32 (CPL = 4) or the rows' own bf16 (CPL = 8)
    typedef typename std::conditional<CPL == 8, uint16_t, float>::type TileT;
    const int d = DC > 0 ? DC : d_;
    __shared__ float pk_all[SPB][PMAX];  // each sample's packed gradient row
    // each wave's tile of T (the once-hit update reads it; YS has none)
    __shared__ __attribute__((aligned(16))) TileT tt_all[YS ? 1 : WPS * SPB][YS ? 4 : NS * SBC];
    __shared__ TableDesc tds[YS ? 1 : NS];
    __shared__ int64_t dmap[MAPPED ? 2 * NS : 1];  // table t's dt rows at dt + dmap[t] + b * dmap[F - 1 + t]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int pair = w / WPS, h = w % WPS;
    constexpr bool mapped = MAPPED;
    const int c = lane & 15, q = lane >> 4;
    const int64_t b = (int64_t)blockIdx.x * SPB + pair;
    const bool live = b < B;
    const int64_t bb = live ? b : 0;  // a padding sample reads sample 0 (and stores nothing)
    const int ksteps = (F + 3) / 4;
    const int P = F * (F - 1) / 2;
    const T* ob = dout + bb * dout_ld;
    float* pk = pk_all[pair];
    TileT* Tt = tt_all[YS ? 0 : w];
    if (h == 0) WT(1, 0, b);
    // the table descriptors (F - 1 <= NS <= 32 < blockDim: one per thread), held in registers and
    // written to LDS after the other independent loads are issued, so no wave waits for them alone
    const bool tdl_ok = !YS && (int)threadIdx.x < F - 1;
    const TableDesc tdl = YS ? TableDesc{nullptr, 0} : load_table(ga.tabs, tdl_ok ? (int)threadIdx.x : 0);
    int64_t dm0 = 0, dm1 = 0;
    if constexpr (MAPPED) {
        dm0 = ldg<int64_t>(ga.dtb + (tdl_ok ? threadIdx.x : 0));
        dm1 = ldg<int64_t>(ga.dtl + (tdl_ok ? threadIdx.x : 0));
    }
    // ---- every independent load first: table `lane`'s index and flag, the packed gradients, x part
    const bool tl = !YS && lane < F - 1;
    const int64_t myidx = YS ? 0 : load_index_if(tl, ga.idx, ga.itype, (int64_t)(tl ? lane : 0) * ga.tstride + bb);
    // su.single NULL (dlrm_interact_bwd_blocked, YS): no once-hit update, every table row goes to dt
    const uint8_t myfl = su.single ? ldg<uint8_t>(su.single + (tl ? (int64_t)lane * su.cap + bb : 0)) : (uint8_t)0;
    constexpr int PPW = (PMAX + 64 * WPS - 1) / (64 * WPS);  // packed values staged per lane
    float pv[PPW];
#pragma unroll
    for (int k = 0; k < PPW; ++k) {
        const int p = h * 64 + lane + 64 * WPS * k;
        const float v = to_f32(ldg<T>(ob + d + (p < P ? p : 0)));
        pv[k] = p < P ? v : 0.0f;
    }
    // super-blocks per wave (CPL = 4, WPS = 2: d <= 512 when not fixed; WPS = 1: d <= 64;
    // CPL = 8: d <= 128, one wave)
    // (DC = 0: WPS = 1 / 2 cover d <= 64 / 512; YS: d = 64 * WPS, one super-block per wave)
    constexpr int SBW = YS ? 1
                           : DC > 0 ? ((DC / SBC + WPS - 1) / WPS > 0 ? (DC / SBC + WPS - 1) / WPS : 1)
                                    : (WPS == 2 ? 4 : 1);
    constexpr int XV = SBC / 64;  // dout x-part values per lane and super-block
    float xv[SBW][XV];
#pragma unroll
    for (int sbi = 0; sbi < SBW; ++sbi)
#pragma unroll
        for (int k = 0; k < XV; ++k) {
            const int n = SBC * h + SBC * WPS * sbi + 64 * k + lane;
            xv[sbi][k] = to_f32(ldg<T>(ob + (n < d ? n : 0)));
        }
    const bool frozen = su.single ? *su.err != 0 : true;  // a bounds error this step: no table row is written
    if (su.single && blockIdx.x == 0 && threadIdx.x == 0) snapshot_error(su.err, frozen ? 1u : 0u);
    if (tdl_ok) {
        tds[threadIdx.x] = tdl;
        if constexpr (MAPPED) {
            dmap[threadIdx.x] = dm0;
            dmap[F - 1 + threadIdx.x] = dm1;
        }
    }
#pragma unroll
    for (int k = 0; k < PPW; ++k) {
        const int p = h * 64 + lane + 64 * WPS * k;
        if (p < PMAX) pk[p] = pv[k];
    }
    __syncthreads();  // tds, pk
    // validate this lane's table index; rows travel as 32-bit (~0u = invalid / no table)
    uint32_t myrow = ~0u;
    if (tl) {
        const int64_t r = myidx - ga.base;
        if (r >= 0 && r < tds[lane].nrows) myrow = (uint32_t)r;
        else if (h == 0 && live) raise_index_error(ga.err);
    }
    const T* rowp[KS];
    unsigned livek = 0;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const int kk = 4 * s + q;
        const uint32_t r = (uint32_t)__shfl((int)myrow, kk >= 1 ? kk - 1 : 0, 64);
        const bool tab = s < ksteps && kk >= 1 && kk < F && r != ~0u;
        const T* src = YS ? ((s < ksteps && kk < F) ? x + bb * x_ld + (int64_t)kk * d : nullptr)
                   : (s < ksteps && kk == 0) ? x + bb * x_ld
                                             : (tab ? (const T*)tds[kk - 1].data + (int64_t)r * d : nullptr);
        livek |= src ? (1u << s) : 0u;
        // (CPL = 8: a masked row reads the zero row -- a 16-B aligned source whatever dout's layout)
        rowp[s] = src ? src : (CPL == 8 ? (const T*)g_zero_row : ob);
    }
    uint32_t urow[NB][4];
#pragma unroll
    for (int I = 0; I < NB; ++I)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int f = I * 16 + 4 * q + r;
            const int src = (f >= 1 && f < F) ? f - 1 : 0;
            const uint32_t row = (uint32_t)__shfl((int)myrow, src, 64);
            const int fl = __shfl((int)myfl, src, 64);
            urow[I][r] = (f >= 1 && f < F && !frozen && fl != 0) ? row : ~0u;
        }
    if (h == 0) WT(1, 1, b);
#pragma unroll
    for (int sbi = 0; sbi < SBW; ++sbi) {
        const int sb = SBC * h + SBC * WPS * sbi;
        if (sb >= d) break;
        const int n0 = sb + CPL * c;  // this lane's CPL output columns
        const bool colok = n0 < d;
        const int nc = colok ? n0 : 0;
        f32x4_t acc[NB][CPL];
#pragma unroll
        for (int I = 0; I < NB; ++I)
#pragma unroll
            for (int e = 0; e < CPL; ++e) acc[I][e] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        if constexpr (CPL == 4) {
            f32x4_t bv[KS];
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const f32x4_t v = load4_f32(rowp[s] + nc);
                bv[s] = ((livek >> s) & 1u) && colok ? v : f32x4_t{0.f, 0.f, 0.f, 0.f};
            }
            if (sbi > 0) wave_lds_sync();  // the previous super-block's tile reads are done
#pragma unroll
            for (int s = 0; s < KS; ++s)
                if (s < ksteps) *(f32x4_t*)(Tt + (4 * s + q) * SBC + 4 * c) = bv[s];
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                if (s < ksteps) {
                    const int kk = 4 * s + q;
#pragma unroll
                    for (int I = 0; I < NB; ++I) {
                        // S[16I+c][kk]: the symmetric zero-diagonal unpack of the pair row
                        const int i = I * 16 + c;
                        const int hi = i > kk ? i : kk, lo = i > kk ? kk : i;
                        const float av = (i != kk && hi < F) ? pk[hi * (hi - 1) / 2 + lo] : 0.0f;
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            acc[I][e] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[s][e], acc[I][e], 0, 0, 0);
                    }
                }
            }
        } else {
            typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
            u32x4_t bv[KS];  // 8 bf16 columns of row 4s+q, packed
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const u32x4_t v = ldg<u32x4_t>(rowp[s] + nc);
                bv[s] = ((livek >> s) & 1u) && colok ? v : u32x4_t{0u, 0u, 0u, 0u};
            }
            if (sbi > 0) wave_lds_sync();  // the previous super-block's tile reads are done
#pragma unroll
            for (int s = 0; s < KS; ++s)
                if (s < ksteps) *(u32x4_t*)(Tt + (4 * s + q) * SBC + 8 * c) = bv[s];
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                if (s < ksteps) {
                    const int kk = 4 * s + q;
#pragma unroll
                    for (int I = 0; I < NB; ++I) {
                        const int i = I * 16 + c;
                        const int hi = i > kk ? i : kk, lo = i > kk ? kk : i;
                        const float av = (i != kk && hi < F) ? pk[hi * (hi - 1) / 2 + lo] : 0.0f;
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            const uint32_t wd = bv[s][e >> 1];
                            const float bvf = __uint_as_float((e & 1) ? (wd & 0xffff0000u) : (wd << 16));
                            acc[I][e] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bvf, acc[I][e], 0, 0, 0);
                        }
                    }
                }
            }
        }
        if (h == 0 && sbi == 0) WT(1, 2, b);
        // dout's x part for this lane's columns (lanes 0..15 hold output row 0)
        float xo[CPL];
#pragma unroll
        for (int e = 0; e < CPL; ++e) {
            const int n = CPL * c + e;  // column within the super-block: lane n & 63 of xv[sbi][n >> 6]
            float xs = __shfl(xv[sbi][0], n & 63, 64);
#pragma unroll
            for (int k = 1; k < XV; ++k) {
                const float t = __shfl(xv[sbi][k], n & 63, 64);
                xs = (n >> 6) == k ? t : xs;
            }
            xo[e] = xs;
        }
        wave_lds_sync();  // the tile of T (written before the MFMAs)
        if (!live || !colok) continue;
#pragma unroll
        for (int I = 0; I < NB; ++I)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int f = I * 16 + 4 * q + r;
                if (f < F) {
                    float v[CPL];
#pragma unroll
                    for (int e = 0; e < CPL; ++e) v[e] = acc[I][e][r];
                    if (urow[I][r] != ~0u) {
                        float wv[CPL];
                        float tw[CPL];  // the row as gathered
                        if constexpr (CPL == 4) {
                            const f32x4_t t4 = *(const f32x4_t*)(Tt + f * SBC + 4 * c);
#pragma unroll
                            for (int e = 0; e < 4; ++e) tw[e] = t4[e];
                        } else {
                            typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
                            const u32x4_t t8 = *(const u32x4_t*)(Tt + f * SBC + 8 * c);
#pragma unroll
                            for (int e = 0; e < 8; ++e)
                                tw[e] = __uint_as_float((e & 1) ? (t8[e >> 1] & 0xffff0000u) : (t8[e >> 1] << 16));
                        }
#pragma unroll
                        for (int e = 0; e < CPL; ++e) wv[e] = __builtin_fmaf(-su.lr, 0.0f + v[e], tw[e]);
                        store_row<T, CPL, true>((T*)tds[f - 1].data + (int64_t)urow[I][r] * d, n0, wv);
                    } else if (!mapped && (f > 0 || !su.single)) {
                        // (the training step (su.single set) leaves dt's x row alone: dx carries it)
                        // (CPL = 8: a lane's two 16-B pieces are 32 B apart, so each store instruction
                        // covers half of every line: plain stores let L2 merge the halves, where
                        // non-temporal ones left as partial-line writes, 95 -> 117 MB per launch)
#pragma unroll
                        for (int e = 0; e < CPL; e += 4) {
                            const f32x4_t pv4 = f32x4_t{v[e], v[e + 1], v[e + 2], v[e + 3]};
                            if constexpr (CPL == 8) stg<f32x4_t>(dt + b * dt_ld + (int64_t)f * d + n0 + e, pv4);
                            else stg_nt<f32x4_t>(dt + b * dt_ld + (int64_t)f * d + n0 + e, pv4);
                        }
                    } else if (f > 0) {
#pragma unroll
                        for (int e = 0; e < CPL; e += 4)
                            stg_nt<f32x4_t>(dt + dmap[f - 1] + b * dmap[F - 2 + f] + n0 + e,
                                            f32x4_t{v[e], v[e + 1], v[e + 2], v[e + 3]});
                    }
                    if (f == 0)
#pragma unroll
                        for (int e = 0; e < CPL; e += 4)
                            stg<f32x4_t>(dx + b * dx_ld + n0 + e, f32x4_t{xo[e] + v[e], xo[e + 1] + v[e + 1],
                                                                         xo[e + 2] + v[e + 2], xo[e + 3] + v[e + 3]});
                }
            }
        if (h == 0 && sbi == 0) {
            WT(1, 3, b);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            WT(1, 4, b);
        }
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

template <typename T, bool GATHER>
__device__ __forceinline__ float t_elem(const T* t, int64_t t_ld, int64_t b, int j, int n, int d, const GatherArgs& ga,
                                        const T* x, int64_t x_ld) {
    if (!GATHER) return to_f32(t[b * t_ld + (int64_t)j * d + n]);
    if (j == 0) return to_f32(x[b * x_ld + n]);
    const int64_t r = load_index(ga.idx, ga.itype, (j - 1) * ga.tstride + b * ga.L) - ga.base;
    if (r < 0 || r >= ga.tabs[j - 1].nrows) {
        raise_index_error(ga.err);
        return 0.0f;
    }
    return to_f32(((const T*)ga.tabs[j - 1].data)[r * d + n]);
}

template <typename T, bool GATHER>
__global__ __launch_bounds__(256) void interact_bwd_scalar(int d, int F, int B, const T* __restrict__ dout,
                                                           int64_t dout_ld, const T* __restrict__ t, int64_t t_ld,
                                                           float* __restrict__ dx, int64_t dx_ld,
                                                           float* __restrict__ dt, int64_t dt_ld, GatherArgs ga,
                                                           const T* __restrict__ x, int64_t x_ld) {
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
            acc = fmaf(t_elem<T, GATHER>(t, t_ld, b, j, n, d, ga, x, x_ld), to_f32(ob[hi * (hi - 1) / 2 + lo]), acc);
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

// samples per 4-wave workgroup of the one-hot forward (fwd_body: one wave per sample)
static int fwd_samples_per_block(int, int) { return 4; }

template <typename T, int NB, bool FUSED>
static void launch_fwd_nb(hipStream_t s, int cus, int d, int F, int B, const void* x, int64_t x_ld, void* ys,
                          int64_t ys_ld, void* out, int64_t out_ld, int padding, const GatherArgs& ga,
                          const TabPtrs& tp) {
    const bool pooled = FUSED && ga.L > 1;
    const unsigned g = grid_for(B, pooled ? 4 : fwd_samples_per_block(d, NB), cus);
    if (FUSED && ga.L > 1)
        hipLaunchKernelGGL((interact_fwd_kernel<T, NB, FUSED, true>), dim3(g), dim3(256), 0, s, d, F, B, (const T*)x,
                           x_ld, (T*)ys, ys_ld, (T*)out, out_ld, padding, ga, tp);
    else if (d == 128)  // the BASELINE feature size, compiled for it
        hipLaunchKernelGGL((interact_fwd_kernel<T, NB, FUSED, false, 128>), dim3(g), dim3(256), 0, s, d, F, B,
                           (const T*)x, x_ld, (T*)ys, ys_ld, (T*)out, out_ld, padding, ga, tp);
    else
        hipLaunchKernelGGL((interact_fwd_kernel<T, NB, FUSED, false>), dim3(g), dim3(256), 0, s, d, F, B, (const T*)x,
                           x_ld, (T*)ys, ys_ld, (T*)out, out_ld, padding, ga, tp);
}

template <typename T, bool FUSED>
static bool dispatch_fwd(int NB, hipStream_t s, int cus, int d, int F, int B, const void* x, int64_t x_ld, void* ys,
                         int64_t ys_ld, void* out, int64_t out_ld, int padding, const GatherArgs& ga,
                         const TabPtrs& tp = TabPtrs{}) {
    switch (NB) {
#define DLRM_CASE(N) \
    case N: launch_fwd_nb<T, N, FUSED>(s, cus, d, F, B, x, x_ld, ys, ys_ld, out, out_ld, padding, ga, tp); return true;
        DLRM_CASE(1) DLRM_CASE(2) DLRM_CASE(3) DLRM_CASE(4) DLRM_CASE(5) DLRM_CASE(6)
#undef DLRM_CASE
        default: return false;
    }
}

static bool fwd_aligned(int dtype, int d, const void* x, int64_t x_ld, const void* ys, int64_t ys_ld) {
    const int vec = dtype == DLRM_F32 ? 4 : 8;  // elements per 16-B fragment load
    return (uintptr_t)x % 16 == 0 && (uintptr_t)ys % 16 == 0 && (x_ld % vec) == 0 && (ys_ld % vec) == 0 &&
           (d % vec) == 0;
}

int launch_interact_fwd(dlrm_ctx* ctx, int dtype, int d, int F, int B, const void* x, int64_t x_ld, void* ys,
                        int64_t ys_ld, void* out, int64_t out_ld, int padding) {
    if (B == 0) return DLRM_OK;
    hipStream_t s = ctx_stream(ctx);
    const int cus = ctx_num_cus(ctx);
    const int NB = (F + 15) / 16;
    GatherArgs ga{};
    bool done = false;
    if (fwd_aligned(dtype, d, x, x_ld, ys, ys_ld))
        done = dtype == DLRM_F32
                   ? dispatch_fwd<float, false>(NB, s, cus, d, F, B, x, x_ld, ys, ys_ld, out, out_ld, padding, ga)
                   : dispatch_fwd<uint16_t, false>(NB, s, cus, d, F, B, x, x_ld, ys, ys_ld, out, out_ld, padding, ga);
    if (!done) {  // NB > 6 would exceed 256 VGPRs; odd alignments
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

// maplookup(PreallocationStrategy(d)) + DotInteraction in one launch.  Returns
// DLRM_E_UNSUPPORTED when the shape/alignment has no fused kernel (the caller then runs
// the two operators separately).
int launch_lookup_interact_fwd(dlrm_ctx* ctx, const TableDesc* tabs, bool tabs_aligned16, int T_, int dtype,
                               const void* idx, int itype, int64_t tstride, int base, int L, int d, int B,
                               const void* x, int64_t x_ld, void* ys, int64_t ys_ld, void* out, int64_t out_ld,
                               int padding,
                    const TableDesc* htabs) {
    if (B == 0) return DLRM_OK;
    const int F = T_ + 1;
    const int NB = (F + 15) / 16;
    if (T_ == 0 || !tabs_aligned16 || !fwd_aligned(dtype, d, x, x_ld, ys, ys_ld) || NB > 6) return DLRM_E_UNSUPPORTED;
    // Pooled bags with ys kept: the many-wave pooled gather (maplookup) + the interaction on ys
    // beat one wave gathering T*L rows per sample (measured 489 vs 701 us at 64 x 256, L = 10);
    // the caller's two-launch fallback gives the same bits.
    if (L > 1 && ys && (int64_t)T_ * L > 64) return DLRM_E_UNSUPPORTED;
    hipStream_t s = ctx_stream(ctx);
    const int cus = ctx_num_cus(ctx);
    GatherArgs ga{tabs, idx, itype, tstride, base, L, ctx_error_word(ctx)};
    TabPtrs tp{};
    if (L == 1 && NB <= 2 && !fill_tab_ptrs(tp, htabs, T_)) return DLRM_E_UNSUPPORTED;  // (the two-launch form)
    const bool ok = dtype == DLRM_F32
                        ? dispatch_fwd<float, true>(NB, s, cus, d, F, B, x, x_ld, ys, ys_ld, out, out_ld, padding, ga, tp)
                        : dispatch_fwd<uint16_t, true>(NB, s, cus, d, F, B, x, x_ld, ys, ys_ld, out, out_ld, padding, ga, tp);
    if (!ok) return DLRM_E_UNSUPPORTED;
    return ctx_hip(ctx, hipGetLastError(), "lookup_interact_fwd launch");
}

template <typename T, int NB, bool GATHER>
static void launch_bwd_nb(hipStream_t s, int cus, int d, int F, int B, const void* dout, int64_t dout_ld,
                          const void* t, int64_t t_ld, float* dx, int64_t dx_ld, float* dt, int64_t dt_ld,
                          const GatherArgs& ga, const void* x, int64_t x_ld) {
    typedef BwdGeom<NB> G;
    const unsigned g = grid_for(B, G::WPB, cus);
    const size_t lds = sizeof(float) * G::LDS_FLOATS * G::WPB + (GATHER ? (sizeof(TableDesc) + 16) * (F - 1) : 0);
    hipLaunchKernelGGL((interact_bwd_kernel<T, NB, GATHER>), dim3(g), dim3(64 * G::WPB), lds, s, d, F, B,
                       (const T*)dout, dout_ld, (const T*)t, t_ld, dx, dx_ld, dt, dt_ld, ga, (const T*)x, x_ld);
}

template <typename T, bool GATHER>
static void dispatch_bwd(int NB, hipStream_t s, int cus, int d, int F, int B, const void* dout, int64_t dout_ld,
                         const void* t, int64_t t_ld, float* dx, int64_t dx_ld, float* dt, int64_t dt_ld,
                         const GatherArgs& ga, const void* x, int64_t x_ld) {
    switch (NB) {
#define DLRM_CASE(N)                                                                                               \
    case N:                                                                                                        \
        launch_bwd_nb<T, N, GATHER>(s, cus, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld, ga, x, x_ld); \
        break;
        DLRM_CASE(1) DLRM_CASE(2) DLRM_CASE(3) DLRM_CASE(4) DLRM_CASE(5) DLRM_CASE(6) DLRM_CASE(7)
#undef DLRM_CASE
    }
}

// dT = S T per sample; T from `t` (materialized ys) or, GATHER, from x + the table rows.
template <bool GATHER>
static int run_interact_bwd(dlrm_ctx* ctx, int dtype, int d, int F, int B, const void* dout, int64_t dout_ld,
                            const void* t, int64_t t_ld, float* dx, int64_t dx_ld, float* dt, int64_t dt_ld,
                            const GatherArgs& ga, bool rows_aligned, const void* x, int64_t x_ld) {
    if (B == 0) return DLRM_OK;
    hipStream_t s = ctx_stream(ctx);
    const int cus = ctx_num_cus(ctx);
    const int NB = (F + 15) / 16;
    const int esz = dtype == DLRM_F32 ? 4 : 2;
    const bool t_ok = GATHER ? (rows_aligned && (uintptr_t)x % (4 * esz) == 0 && (x_ld % 4) == 0)
                             : ((uintptr_t)t % (4 * esz) == 0 && (t_ld % 4) == 0);
    const bool aligned = d % 4 == 0 && t_ok && (uintptr_t)dx % 16 == 0 && (uintptr_t)dt % 16 == 0 && (dx_ld % 4) == 0 &&
                         (dt_ld % 4) == 0;
    // a materialized ys with 33..96 features (pooled bags): the split kernel's load plan, one wave
    // per 64-column super-block (the one-wave-per-sample bwd_body kernel spills at NB = 5 and ran
    // the pooled backward at 145 us); bit-identical (the same MFMA sums).  DLRM_BWD_YS = 0: bwd_body.
    const bool ys_split = !knobs().bwd_ys_body;
    const int wps = d >= 256 ? 4 : (d >= 128 ? 2 : 1);
    if (!GATHER && ys_split && aligned && NB >= 3 && NB <= 6 && d == 64 * wps) {
        const StepUpdate su{nullptr, 0, 0.0f, ctx_error_word(ctx)};
#define DLRM_YS(TY, N_, W_)                                                                                         \
    hipLaunchKernelGGL((interact_bwd_split_kernel<TY, N_, 0, 1, W_, false, 4, true>), dim3((unsigned)B),            \
                       dim3(64 * W_), 0, s, d, F, B, (const TY*)dout, dout_ld, dx, dx_ld, dt, dt_ld, ga,           \
                       (const TY*)t, t_ld, su)
#define DLRM_YS_W(TY, N_) \
    if (wps == 4) DLRM_YS(TY, N_, 4); else if (wps == 2) DLRM_YS(TY, N_, 2); else DLRM_YS(TY, N_, 1);
#define DLRM_YS_NB(TY)                                                                            \
    switch (NB) {                                                                                 \
        case 3: DLRM_YS_W(TY, 3) break;                                                           \
        case 4: DLRM_YS_W(TY, 4) break;                                                           \
        case 5: DLRM_YS_W(TY, 5) break;                                                           \
        default: DLRM_YS_W(TY, 6) break;                                                          \
    }
        if (dtype == DLRM_F32) { DLRM_YS_NB(float) } else { DLRM_YS_NB(uint16_t) }
#undef DLRM_YS_NB
#undef DLRM_YS_W
#undef DLRM_YS
        return ctx_hip(ctx, hipGetLastError(), "interact_bwd(ys, split) launch");
    }
    if (aligned && NB >= 1 && NB <= 7) {  // NB = 8 would need > 64 KB of dynamic LDS
        if (dtype == DLRM_F32)
            dispatch_bwd<float, GATHER>(NB, s, cus, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld, ga, x, x_ld);
        else
            dispatch_bwd<uint16_t, GATHER>(NB, s, cus, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld, ga, x,
                                           x_ld);
    } else {
        const unsigned g = grid_for((int64_t)B * F * d, 256, cus);
        if (dtype == DLRM_F32)
            hipLaunchKernelGGL((interact_bwd_scalar<float, GATHER>), dim3(g), dim3(256), 0, s, d, F, B,
                               (const float*)dout, dout_ld, (const float*)t, t_ld, dx, dx_ld, dt, dt_ld, ga,
                               (const float*)x, x_ld);
        else
            hipLaunchKernelGGL((interact_bwd_scalar<uint16_t, GATHER>), dim3(g), dim3(256), 0, s, d, F, B,
                               (const uint16_t*)dout, dout_ld, (const uint16_t*)t, t_ld, dx, dx_ld, dt, dt_ld, ga,
                               (const uint16_t*)x, x_ld);
    }
    return ctx_hip(ctx, hipGetLastError(), "interact_bwd launch");
}

int launch_interact_bwd(dlrm_ctx* ctx, int dtype, int d, int F, int B, const void* dout, int64_t dout_ld,
                        const void* t, int64_t t_ld, float* dx, int64_t dx_ld, float* dt, int64_t dt_ld) {
    return run_interact_bwd<false>(ctx, dtype, d, F, B, dout, dout_ld, t, t_ld, dx, dx_ld, dt, dt_ld, GatherArgs{},
                                   true, nullptr, 0);
}

int launch_interact_bwd_gather(dlrm_ctx* ctx, const TableDesc* tabs, bool tabs_aligned16, int T_, int dtype,
                               const void* idx, int itype, int64_t tstride, int base, int L, int d, int B,
                               const void* x, int64_t x_ld, const void* dout, int64_t dout_ld, float* dx,
                               int64_t dx_ld, float* dt, int64_t dt_ld, const IndexerDev* ix,
                    const TableDesc* htabs) {
    GatherArgs ga{tabs, idx, itype, tstride, base, L, ctx_error_word(ctx)};
    const int F = T_ + 1;
    const int NB = (F + 15) / 16;
    const int esz = dtype == DLRM_F32 ? 4 : 2;
    if (ix && B > 0 && T_ > 0) {
        const bool aligned = d % 4 == 0 && tabs_aligned16 && (uintptr_t)x % (4 * esz) == 0 && (x_ld % 4) == 0 &&
                             (uintptr_t)dx % 16 == 0 && (uintptr_t)dt % 16 == 0 && (dx_ld % 4) == 0 && (dt_ld % 4) == 0;
        if (aligned && NB <= 2 && (int64_t)B * L <= 256 * kBwdIndexEPL) {
            hipStream_t s = ctx_stream(ctx);
            const int cus = ctx_num_cus(ctx);
            size_t lds = sizeof(FastLds<256, kBwdIndexEPL>);
#define DLRM_LAUNCH_BWDIX(TY, N_)                                                                                 \
    {                                                                                                              \
        typedef BwdGeom<N_> G;                                                                                     \
        const size_t blds = sizeof(float) * G::LDS_FLOATS * G::WPB + sizeof(TableDesc) * T_;                       \
        if (blds > lds) lds = blds;                                                                                \
        const unsigned g = grid_for(B, G::WPB, cus);                                                               \
        hipLaunchKernelGGL((interact_bwd_index_kernel<TY, N_>), dim3(g + T_), dim3(256), lds, s, d, F, B,          \
                           (const TY*)dout, dout_ld, dx, dx_ld, dt, dt_ld, ga, (const TY*)x, x_ld, *ix);           \
    }
            if (dtype == DLRM_F32) {
                if (NB == 1) DLRM_LAUNCH_BWDIX(float, 1) else DLRM_LAUNCH_BWDIX(float, 2)
            } else {
                if (NB == 1) DLRM_LAUNCH_BWDIX(uint16_t, 1) else DLRM_LAUNCH_BWDIX(uint16_t, 2)
            }
#undef DLRM_LAUNCH_BWDIX
            return ctx_hip(ctx, hipGetLastError(), "interact_bwd(+indexer) launch");
        }
        // no fused form for this shape: the indexer's own launch, then the backward
        const int rc = launch_indexer_build(ctx, *ix, tabs, T_, idx, itype, tstride, base, B, L);
        if (rc) return rc;
    }
    return run_interact_bwd<true>(ctx, dtype, d, T_ + 1, B, dout, dout_ld, nullptr, 0, dx, dx_ld, dt, dt_ld, ga,
                                  tabs_aligned16, x, x_ld);
}

// dlrm_interact_bwd_gather with table t's dt rows written to dst + dbase[t] + b * dld[t] (the
// sharded exchange's send layout) by the backward's own stores: no dt buffer, no repack launch.
// Vector kernel shapes only (DLRM_E_UNSUPPORTED otherwise).
int launch_interact_bwd_blocked(dlrm_ctx* ctx, const TableDesc* tabs, bool tabs_aligned16, int T_, int dtype,
                                const void* idx, int itype, int64_t tstride, int base, int L, int d, int B,
                                const void* x, int64_t x_ld, const void* dout, int64_t dout_ld, float* dx,
                                int64_t dx_ld, float* dst, const int64_t* dbase, const int64_t* dld,
                    const TableDesc* htabs) {
    if (B == 0 || T_ == 0) return DLRM_OK;
    const int F = T_ + 1;
    const int NB = (F + 15) / 16;
    const int esz = dtype == DLRM_F32 ? 4 : 2;
    const bool aligned = d % 4 == 0 && tabs_aligned16 && (uintptr_t)x % (4 * esz) == 0 && (x_ld % 4) == 0 &&
                         (uintptr_t)dx % 16 == 0 && (uintptr_t)dst % 16 == 0 && (dx_ld % 4) == 0;
    if (!aligned || NB > 7)
        return ctx_fail(ctx, DLRM_E_UNSUPPORTED, "interact_bwd_blocked: 16-B aligned rows and F <= 112 needed");
    GatherArgs ga{tabs, idx, itype, tstride, base, L, ctx_error_word(ctx), dbase, dld};
    hipStream_t s = ctx_stream(ctx);
    const int cus = ctx_num_cus(ctx);
    if (L == 1 && NB <= 2 && (d == 128 || d <= 64) && fwd_aligned(dtype, d, x, x_ld, nullptr, 0)) {
        // the step backward's kernel (two waves per sample at d = 128, one at d <= 64) with no
        // once-hit update: every table row's gradient goes to the send layout
        const StepUpdate su{nullptr, 0, 0.0f, ctx_error_word(ctx)};
#define DLRM_LAUNCH_BLK(TY, N_)                                                                                    \
    if (d == 128)                                                                                                  \
        hipLaunchKernelGGL((interact_bwd_split_kernel<TY, N_, 128, 4, 2, true>), dim3((unsigned)((B + 3) / 4)),      \
                           dim3(128 * 4), 0, s, d, F, B, (const TY*)dout, dout_ld, dx, dx_ld, dst, 0, ga, (const TY*)x,\
                           x_ld, su);                                                                              \
    else                                                                                                           \
        hipLaunchKernelGGL((interact_bwd_split_kernel<TY, N_, 0, 2, 1, true>), dim3((unsigned)((B + 1) / 2)),        \
                           dim3(64 * 2), 0, s, d, F, B, (const TY*)dout, dout_ld, dx, dx_ld, dst, 0, ga, (const TY*)x, \
                           x_ld, su);
        if (dtype == DLRM_F32) {
            if (NB == 1) { DLRM_LAUNCH_BLK(float, 1) } else { DLRM_LAUNCH_BLK(float, 2) }
        } else {
            if (NB == 1) { DLRM_LAUNCH_BLK(uint16_t, 1) } else { DLRM_LAUNCH_BLK(uint16_t, 2) }
        }
#undef DLRM_LAUNCH_BLK
        return ctx_hip(ctx, hipGetLastError(), "interact_bwd_blocked(split) launch");
    }
    if (dtype == DLRM_F32)
        dispatch_bwd<float, true>(NB, s, cus, d, F, B, dout, dout_ld, nullptr, 0, dx, dx_ld, dst, 0, ga, x, x_ld);
    else
        dispatch_bwd<uint16_t, true>(NB, s, cus, d, F, B, dout, dout_ld, nullptr, 0, dx, dx_ld, dst, 0, ga, x, x_ld);
    return ctx_hip(ctx, hipGetLastError(), "interact_bwd_blocked launch");
}

// Shapes whose backward can take a split indexer (interact_bwd_update_kernel: F <= 32, 16-B
// aligned rows and x), whatever the batch size.
bool step_split_supported(bool tabs_aligned16, int T_, int dtype, int d, const void* x, int64_t x_ld) {
    const int NB = (T_ + 1 + 15) / 16;
    return T_ > 0 && tabs_aligned16 && fwd_aligned(dtype, d, x, x_ld, nullptr, 0) && NB <= 2;
}

// Training-step forward (split indexer in the same grid).  DLRM_E_UNSUPPORTED when the shape
// has no such kernel (the caller then runs the fused forward and the indexer separately).
int launch_step_fwd(dlrm_ctx* ctx, const TableDesc* tabs, bool tabs_aligned16, int T_, int dtype, const void* idx,
                    int itype, int64_t tstride, int base, int d, int B, const void* x, int64_t x_ld, void* out,
                    int64_t out_ld, int padding, const IndexerDev& ix,
                    const TableDesc* htabs) {
    const int F = T_ + 1;
    const int NB = (F + 15) / 16;
    if (B == 0 || T_ == 0 || !tabs_aligned16 || !fwd_aligned(dtype, d, x, x_ld, nullptr, 0) || NB > 2 ||
        B > kStepIndexMaxN)
        return DLRM_E_UNSUPPORTED;
    hipStream_t s = ctx_stream(ctx);
    const int cus = ctx_num_cus(ctx);
    GatherArgs ga{tabs, idx, itype, tstride, base, 1, ctx_error_word(ctx)};
    TabPtrs tp{};
    if (!fill_tab_ptrs(tp, htabs, T_)) return DLRM_E_UNSUPPORTED;
    const bool wave = ix.vshift >= 2;
    size_t lds = wave ? sizeof(WaveBuildLds) : sizeof(StepLds);
    if (lds < sizeof(float) * 4 * kStage) lds = sizeof(float) * 4 * kStage;
    const unsigned g = grid_for(B, fwd_samples_per_block(d, NB), cus) +
                       (wave ? (T_ << ix.vshift) / kWaveParts : (T_ << ix.vshift));
#define DLRM_LAUNCH_FWDIX(TY, N_)                                                                                  \
    if (d == 128)                                                                                                  \
        hipLaunchKernelGGL((interact_fwd_index_kernel<TY, N_, 128>), dim3(g), dim3(256), lds, s, d, F, B,            \
                           (const TY*)x, x_ld, (TY*)out, out_ld, padding, ga, ix, tp);                               \
    else                                                                                                           \
        hipLaunchKernelGGL((interact_fwd_index_kernel<TY, N_>), dim3(g), dim3(256), lds, s, d, F, B, (const TY*)x,   \
                           x_ld, (TY*)out, out_ld, padding, ga, ix, tp);
    if (dtype == DLRM_F32) {
        if (NB == 1) DLRM_LAUNCH_FWDIX(float, 1) else DLRM_LAUNCH_FWDIX(float, 2)
    } else {
        if (NB == 1) DLRM_LAUNCH_FWDIX(uint16_t, 1) else DLRM_LAUNCH_FWDIX(uint16_t, 2)
    }
#undef DLRM_LAUNCH_FWDIX
    return ctx_hip(ctx, hipGetLastError(), "step_fwd launch");
}

// Training-step backward after launch_step_fwd: once-hit rows updated in place, dt rows of the
// others written for the apply.  The caller checked the shape (launch_step_fwd accepted it)
// and the 16-B alignment of dx / dt.
int launch_step_bwd(dlrm_ctx* ctx, const TableDesc* tabs, int T_, int dtype, const void* idx, int itype,
                    int64_t tstride, int base, int d, int B, const void* x, int64_t x_ld, const void* dout,
                    int64_t dout_ld, float* dx, int64_t dx_ld, float* dt, int64_t dt_ld, const IndexerDev& ix,
                    float lr,
                    const TableDesc* htabs) {
    if (B == 0 || T_ == 0) return DLRM_OK;
    const int F = T_ + 1;
    const int NB = (F + 15) / 16;
    hipStream_t s = ctx_stream(ctx);
    const int cus = ctx_num_cus(ctx);
    GatherArgs ga{tabs, idx, itype, tstride, base, 1, ctx_error_word(ctx)};
    StepUpdate su{ix.single, ix.cap, lr, ctx_error_word(ctx)};
    // one super-block of T rows in flight: two (the gather backward's choice) spill here
    const int sbu = knobs().upd_sbu;
    // d = 128 (two 64-column super-blocks): two waves per sample (interact_bwd_split_kernel)
    const bool split = !knobs().bwd_nosplit;
    if (split && d == 128) {
        // samples per block (DLRM_BWD_SPB = 2, 4 or 8 overrides)
        const int spb_env = knobs().bwd_spb >= 8 ? 8 : (knobs().bwd_spb >= 4 ? 4 : (knobs().bwd_spb > 0 ? 2 : 0));
#define DLRM_LAUNCH_SPLIT(TY, N_, S_)                                                                              \
    hipLaunchKernelGGL((interact_bwd_split_kernel<TY, N_, 128, S_>), dim3((unsigned)((B + S_ - 1) / S_)),            \
                       dim3(128 * S_), 0, s, d, F, B, (const TY*)dout, dout_ld, dx, dx_ld, dt, dt_ld, ga, (const TY*)x,  \
                       x_ld, su)
#define DLRM_LAUNCH_SPLIT_S(TY, N_)                 \
    if (spb == 8) DLRM_LAUNCH_SPLIT(TY, N_, 8);     \
    else if (spb == 4) DLRM_LAUNCH_SPLIT(TY, N_, 4); \
    else DLRM_LAUNCH_SPLIT(TY, N_, 2);
        // bf16, B > 2048: 8 columns per lane, one wave per sample, 2 samples per block
        // (kaggle-d128-b8192-bf16: backward 52.2 -> 48.4 us, step 110.9 -> 103.3 us, r6q; at B = 2048
        // the two-wave form keeps the step shorter: Terabyte rows 50.6 vs 48.7 M samples/s, r6s).
        // DLRM_BWD_CPL = 4 / 8 forces either form.
        const int cpl_env = knobs().bwd_cpl;
        const bool cpl8 = dtype != DLRM_F32 && (cpl_env ? cpl_env == 8 : B > 2048);
        const int spb = spb_env ? spb_env : (cpl8 ? 2 : 4);
#define DLRM_LAUNCH_SPLIT8(N_, S_)                                                                                 \
    hipLaunchKernelGGL((interact_bwd_split_kernel<uint16_t, N_, 128, S_, 1, false, 8>),                             \
                       dim3((unsigned)((B + S_ - 1) / S_)), dim3(64 * S_), 0, s, d, F, B, (const uint16_t*)dout,    \
                       dout_ld, dx, dx_ld, dt, dt_ld, ga, (const uint16_t*)x, x_ld, su)
#define DLRM_LAUNCH_SPLIT8_S(N_)                 \
    if (spb == 8) DLRM_LAUNCH_SPLIT8(N_, 8);     \
    else if (spb == 4) DLRM_LAUNCH_SPLIT8(N_, 4); \
    else DLRM_LAUNCH_SPLIT8(N_, 2);
        if (dtype == DLRM_F32) {
            if (NB == 1) { DLRM_LAUNCH_SPLIT_S(float, 1) } else { DLRM_LAUNCH_SPLIT_S(float, 2) }
        } else if (cpl8) {
            if (NB == 1) { DLRM_LAUNCH_SPLIT8_S(1) } else { DLRM_LAUNCH_SPLIT8_S(2) }
        } else {
            if (NB == 1) { DLRM_LAUNCH_SPLIT_S(uint16_t, 1) } else { DLRM_LAUNCH_SPLIT_S(uint16_t, 2) }
        }
#undef DLRM_LAUNCH_SPLIT8_S
#undef DLRM_LAUNCH_SPLIT8
#undef DLRM_LAUNCH_SPLIT_S
#undef DLRM_LAUNCH_SPLIT
        return ctx_hip(ctx, hipGetLastError(), "step_bwd(split) launch");
    }
    // d <= 64: the same kernel with one wave per sample, 8 samples per block
    if (split && d <= 64) {
#define DLRM_LAUNCH_ONE(TY, N_)                                                                                    \
    hipLaunchKernelGGL((interact_bwd_split_kernel<TY, N_, 0, 8, 1>), dim3((unsigned)((B + 7) / 8)), dim3(64 * 8), 0, \
                       s, d, F, B, (const TY*)dout, dout_ld, dx, dx_ld, dt, dt_ld, ga, (const TY*)x, x_ld, su)
        if (dtype == DLRM_F32) {
            if (NB == 1) DLRM_LAUNCH_ONE(float, 1); else DLRM_LAUNCH_ONE(float, 2);
        } else {
            if (NB == 1) DLRM_LAUNCH_ONE(uint16_t, 1); else DLRM_LAUNCH_ONE(uint16_t, 2);
        }
#undef DLRM_LAUNCH_ONE
        return ctx_hip(ctx, hipGetLastError(), "step_bwd(one wave per sample) launch");
    }
#define DLRM_LAUNCH_BWDUP(TY, N_)                                                                                  \
    {                                                                                                              \
        typedef BwdGeom<N_> G;                                                                                     \
        const size_t lds = sizeof(float) * G::template lds_floats<true>() * G::WPB + sizeof(TableDesc) * T_;       \
        const dim3 grid(grid_for(B, G::WPB, cus)), blk(64 * G::WPB);                                               \
        if (d == 128 && sbu == 2)                                                                                  \
            hipLaunchKernelGGL((interact_bwd_update_kernel<TY, N_, 2, 128>), grid, blk, lds, s, d, F, B,             \
                               (const TY*)dout, dout_ld, dx, dx_ld, dt, dt_ld, ga, (const TY*)x, x_ld, su);         \
        else if (d == 128)                                                                                         \
            hipLaunchKernelGGL((interact_bwd_update_kernel<TY, N_, 1, 128>), grid, blk, lds, s, d, F, B,             \
                               (const TY*)dout, dout_ld, dx, dx_ld, dt, dt_ld, ga, (const TY*)x, x_ld, su);         \
        else                                                                                                       \
            hipLaunchKernelGGL((interact_bwd_update_kernel<TY, N_, 1>), grid, blk, lds, s, d, F, B, (const TY*)dout, \
                               dout_ld, dx, dx_ld, dt, dt_ld, ga, (const TY*)x, x_ld, su);                          \
    }
    if (dtype == DLRM_F32) {
        if (NB == 1) DLRM_LAUNCH_BWDUP(float, 1) else DLRM_LAUNCH_BWDUP(float, 2)
    } else {
        if (NB == 1) DLRM_LAUNCH_BWDUP(uint16_t, 1) else DLRM_LAUNCH_BWDUP(uint16_t, 2)
    }
#undef DLRM_LAUNCH_BWDUP
    return ctx_hip(ctx, hipGetLastError(), "step_bwd launch");
}

}  // namespace dlrm
