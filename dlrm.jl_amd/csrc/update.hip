// update.hip — SparseIndexer + EmbeddingTables.update!(Descent(lr), ...) on gfx950.
//
// Reference: src/train/train.jl:274-292 (SparseIndexer per table, update! with num_splits /
// nthreads), checked by src/validation.jl:125-146 against the PyTorch `update_emb_*`.
//
//   table_t[r] -= lr * sum_{(b,k): idx_t[b*L+k] - base == r} grad[b][offset + t*D : +D]
//
// Deterministic design (the default):
//  1. indexer_build (one 1024-thread workgroup per table): the table's B*L indices are read
//     once into LDS, then grouped by row with a stable counting-sort pass on the low row byte
//     (invalid indices go to a 257th bucket that stays last).  When every bucket is small
//     (uniform rows: ~8 per bucket at B = 2048) each bucket is ordered by a direct rank on
//     (row, position); skewed rows fall back to the remaining LSD passes.  Lane groups find
//     equal digits with 64-lane ballots (multi-split), so equal rows keep ascending
//     positions.  The same workgroup then lists the segments (one per distinct row): those of
//     <= kChunk positions as chunks, longer ones (hot rows of small tables: a 3-row table gets
//     ~680 hits per row at B = 2048) as hot segments.
//  2. sgd_apply: lane groups take one chunk each (grad rows summed in ascending position
//     order, 16-B lanes, 8 rows in flight, the table row prefetched meanwhile) and write the
//     row once; each hot segment gets a whole workgroup whose lane groups sum fixed-size
//     sub-chunks into LDS, combined in sub-chunk order before the row is written once.
// Every touched row is written exactly once with a summation order fixed by positions:
// bitwise reproducible, and no inter-workgroup hand-off.  DLRM_UPDATE_ATOMIC instead adds
// -lr*g straight into the table with global_atomic_add_f32 (no sort, non-deterministic
// rounding order).
#include "common.hpp"

#ifdef DLRM_PHASE
// Phase timestamps (wall_clock64, 100 MHz) of one indexer block + start/end of every block;
// built only into the profiling variant of the library (tools/phase_indexer.py).
__device__ unsigned long long g_phase[64];
__device__ unsigned long long g_blk[2][256];
__device__ unsigned long long g_phase2[256][32];  // every block < 256: marks k < 32
#define PHASE(k) do { __syncthreads(); if (threadIdx.x == 0) { const unsigned long long c_ = wall_clock64(); \
    if (blockIdx.x == DLRM_PHASE) g_phase[k] = c_; if (blockIdx.x < 256 && (k) < 32) g_phase2[blockIdx.x][k] = c_; } } while (0)
__device__ unsigned long long g_wph[256][4][16];  // wave build: per block, wave, mark
#define WPH(k) do { if ((threadIdx.x & 63) == 0 && blockIdx.x < 256) g_wph[blockIdx.x][(threadIdx.x >> 6) & 3][k] = wall_clock64(); } while (0)
extern "C" int dlrm_debug_wph(unsigned long long* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wph), sizeof(g_wph));
}
extern "C" int dlrm_debug_phase2(unsigned long long* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase2), sizeof(g_phase2));
}
__device__ unsigned long long g_apply[3][32768];  // start, end, kind of every apply block
#define APPLY_START(kind) do { if (threadIdx.x == 0) { const int blk_ = blockIdx.y * gridDim.x + blockIdx.x; \
    if (blk_ < 32768) { g_apply[0][blk_] = wall_clock64(); g_apply[2][blk_] = (kind); } } } while (0)
#define APPLY_END() do { if ((threadIdx.x & 63) == 0) { const int blk_ = blockIdx.y * gridDim.x + blockIdx.x; \
    if (blk_ < 32768) atomicMax(&g_apply[1][blk_], wall_clock64()); } } while (0)
extern "C" int dlrm_debug_phase(unsigned long long* out) {
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(g_phase));
    return (int)hipMemcpyFromSymbol(out + 64, HIP_SYMBOL(g_blk), sizeof(g_blk));
}
extern "C" int dlrm_debug_apply(unsigned long long* out) {
    hipMemset(g_apply, 0, 0);
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_apply), sizeof(g_apply));
}
extern "C" int dlrm_debug_apply_reset(void) {
    static unsigned long long z[3][32768];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_apply), z, sizeof(z));
}
// per-item log of the apply launch: slot = block * 16 + k (its k-th item): start, end, kind | item << 8
__device__ unsigned long long g_item[3][65536];
#define ITEM_START(kind, k, item) do { const int s_ = (blockIdx.x * 16 + (k)); if (threadIdx.x == 0 && (k) < 16 && s_ < 65536) { \
    g_item[0][s_] = wall_clock64(); g_item[2][s_] = (unsigned long long)(kind) | ((unsigned long long)(item) << 8); } } while (0)
#define ITEM_END(k) do { const int s_ = (blockIdx.x * 16 + (k)); if ((threadIdx.x & 63) == 0 && (k) < 16 && s_ < 65536) \
    atomicMax(&g_item[1][s_], wall_clock64()); } while (0)
extern "C" int dlrm_debug_items(unsigned long long* out, int reset) {
    if (reset) {
        static unsigned long long z[3][65536];
        return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_item), z, sizeof(z));
    }
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_item), sizeof(g_item));
}
#else
#define ITEM_START(kind, k, item) do {} while (0)
#define ITEM_END(k) do {} while (0)
#define PHASE(k) do {} while (0)
#define APPLY_START(kind) do {} while (0)
#define APPLY_END() do {} while (0)
#endif

#include "apply.hpp"

namespace dlrm {

constexpr int kBuildThreads = 1024;
constexpr int kBuildWaves = kBuildThreads / 64;
constexpr int kLdsSortMax = 2048;   // positions per table sorted entirely in LDS
constexpr int kDigits = 257;        // 256 row digits + 1 bucket that keeps invalid indices last

int64_t indexer_slice_cap(int64_t cap) { return cap / kHotSlice + cap / (kMinChunk + 1) + 1; }

template <typename V>
__device__ __forceinline__ V block_scan_excl(V v, V* wtot, V* tot) { return block_scan_nw<kBuildWaves, V>(v, wtot, tot); }

struct SortLds {
    int cnt[kBuildWaves][kDigits + 7];  // per-wave digit counts, then their global offsets
    int hist[kDigits + 7];
    int digit_off[kDigits + 7];
    int bucket_start[kDigits + 8];
    int wtot[2 * kBuildWaves];
    long long wtot64[2 * kBuildWaves];
    int nvalid;
    int maxbucket;
};

// One stable counting-sort pass of (K, V) by digit(key) = low byte at `shift`, or 256 for
// the invalid-index sentinel.  Tiles of 1024 positions in order; the lanes of a wave that
// share a digit are found with 9 ballots, the cross-wave offsets go through LDS.
__device__ void radix_pass(int N, int shift, bool first_pass, uint32_t sentinel, const uint32_t* kin,
                           const int32_t* vin, uint32_t* kout, int32_t* vout, SortLds& sl) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const unsigned long long lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int d = tid; d < kDigits; d += kBuildThreads) sl.hist[d] = 0;
    __syncthreads();
    for (int i = tid; i < N; i += kBuildThreads) {
        const uint32_t key = kin[i];
        atomicAdd(&sl.hist[key == sentinel ? 256 : (key >> shift) & 255u], 1);
    }
    __syncthreads();
    {
        const int v = tid < kDigits ? sl.hist[tid] : 0;
        int tot;
        const int ex = block_scan_excl<int>(v, sl.wtot, &tot);
        PHASE(first_pass ? 3 : 13);
        if (tid < kDigits) {
            sl.digit_off[tid] = ex;
            if (first_pass) sl.bucket_start[tid] = ex;
        }
        if (first_pass) {
            if (tid == 0) {
                sl.bucket_start[kDigits] = N;
                sl.maxbucket = 0;
            }
            // largest valid-row bucket (decides rank sort vs more radix passes)
            int m = tid < 256 ? v : 0;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
            __syncthreads();
            if (lane == 0 && m > 0) atomicMax(&sl.maxbucket, m);
        }
        __syncthreads();
    }
    PHASE(first_pass ? 4 : 14);
    for (int tile = 0; tile < N; tile += kBuildThreads) {
        const int i = tile + tid;
        const bool valid = i < N;
        const uint32_t key = valid ? kin[i] : 0u;
        const int32_t val = valid ? vin[i] : 0;
        const uint32_t digit = key == sentinel ? 256u : (key >> shift) & 255u;
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 9; ++bit) {
            const unsigned long long bb = __ballot(valid && ((digit >> bit) & 1u));
            peers &= ((digit >> bit) & 1u) ? bb : ~bb;
        }
        const int rank = __popcll(peers & lt_mask);
        for (int e = lane; e < kDigits; e += 64) sl.cnt[w][e] = 0;
        __syncthreads();
        if (valid && rank == 0) sl.cnt[w][digit] = __popcll(peers);
        __syncthreads();
        if (tid < kDigits) {
            int run = sl.digit_off[tid];
            for (int ww = 0; ww < kBuildWaves; ++ww) {
                const int c = sl.cnt[ww][tid];
                sl.cnt[ww][tid] = run;
                run += c;
            }
            sl.digit_off[tid] = run;
        }
        __syncthreads();
        if (valid) {
            const int dst = sl.cnt[w][digit] + rank;
            kout[dst] = key;
            vout[dst] = val;
        }
        __syncthreads();
        PHASE(first_pass ? 5 + tile / kBuildThreads : 15);
    }
}

// Segments (one per distinct valid row) from the sorted arrays, then the chunk list
// (segments of <= kChunk positions) and the hot list (longer segments).  sseg/srow are
// scratch of >= N entries (LDS when the sort ran in LDS).
__device__ void build_segments(const IndexerDev& ix, int t, const uint32_t* K, const int32_t* V, int N,
                               uint32_t sentinel, int32_t* sseg, uint32_t* srow, SortLds& sl) {
    const int tid = threadIdx.x;
    const int64_t off = (int64_t)t * ix.cap;
    if (tid == 0) sl.nvalid = 0;
    __syncthreads();
    int32_t* seg_start = ix.seg_start + (int64_t)t * (ix.cap + 1);
    uint32_t* seg_row = ix.seg_row + off;
    int32_t* perm = ix.perm + off;
    int U = 0;
    for (int tile = 0; tile < N; tile += kBuildThreads) {
        const int i = tile + tid;
        const uint32_t k = i < N ? K[i] : sentinel;
        const bool live = i < N && k != sentinel;
        const bool head = live && (i == 0 || K[i - 1] != k);
        if (live) {
            perm[i] = V[i];
            if (i + 1 == N || K[i + 1] == sentinel) sl.nvalid = i + 1;
        }
        int tot;
        const int ex = block_scan_excl<int>(head ? 1 : 0, sl.wtot, &tot);
        if (head) {
            seg_start[U + ex] = i;
            seg_row[U + ex] = k;
            sseg[U + ex] = i;
            srow[U + ex] = k;
        }
        U += tot;
    }
    __syncthreads();
    PHASE(20);
    const int nvalid = sl.nvalid;
    if (tid == 0) seg_start[U] = nvalid;
    int4* chunks = ix.chunks + 2 * off;
    int4* hot = ix.hot + off;
    int4* hot_slice = ix.hot_slice + off;
    long long C = 0, H = 0, S = 0;
    for (int tile = 0; tile < U; tile += kBuildThreads) {
        const int s = tile + tid;
        int beg = 0, end = 0;
        if (s < U) {
            beg = sseg[s];
            end = s + 1 < U ? sseg[s + 1] : nvalid;
        }
        const bool isc = s < U && end - beg <= kChunk;
        const bool ish = s < U && end - beg > kChunk;
        const int ns = ish ? (end - beg + kHotSlice - 1) / kHotSlice : 0;
        long long tot, tots;
        const long long ex = block_scan_excl<long long>((isc ? 1ll : 0ll) | ((ish ? 1ll : 0ll) << 32), sl.wtot64, &tot);
        const long long exs = block_scan_excl<long long>((long long)ns, sl.wtot64, &tots);
        if (isc) write_chunk(chunks, C + (ex & 0xffffffffll), beg, end, (int)srow[s], V);
        if (ish) {
            const int h = (int)(H + (ex >> 32));
            const int s0 = (int)(S + exs);
            hot[h] = make_int4(beg, end, (int)srow[s], s0);
            write_slices(hot_slice, s0, beg, end, (int)srow[s], h);
        }
        C += tot & 0xffffffffll;
        H += tot >> 32;
        S += tots;
    }
    PHASE(21);
    if (tid == 0) {
        int32_t* cnt = ix.counts + (int64_t)t * 8;
        cnt[CNT_U] = U; cnt[CNT_C] = (int)C; cnt[CNT_H] = (int)H; cnt[CNT_S] = (int)S; cnt[CNT_NV] = nvalid;
    }
}

template <bool IN_LDS>
__global__ __launch_bounds__(kBuildThreads) void indexer_build_kernel(
    IndexerDev ix, const TableDesc* __restrict__ tabs, const void* __restrict__ idx, int itype,
    int64_t tstride, int base, int B, int L, unsigned* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    __shared__ SortLds sl;
#ifdef DLRM_PHASE
    if (threadIdx.x == 0) g_blk[0][blockIdx.x] = wall_clock64();
#endif
    PHASE(0);
    const int t = blockIdx.x;
    const int tid = threadIdx.x;
    const int N = B * L;
    const int64_t off = (int64_t)t * ix.cap;
    const uint32_t nrows = (uint32_t)tabs[t].nrows;  // host checks nrows < 2^32 - 1
    const uint32_t sentinel = nrows;
    const int nbits = 32 - __clz(nrows > 0 ? nrows - 1 : 0);  // bits of the largest valid row
    uint32_t* kbuf[2];
    int32_t* vbuf[2];
    if (IN_LDS) {
        kbuf[0] = (uint32_t*)dyn;
        kbuf[1] = kbuf[0] + kLdsSortMax;
        vbuf[0] = (int32_t*)(kbuf[1] + kLdsSortMax);
        vbuf[1] = vbuf[0] + kLdsSortMax;
    } else {
        kbuf[0] = ix.keys0 + off; kbuf[1] = ix.keys1 + off;
        vbuf[0] = ix.vals0 + off; vbuf[1] = ix.vals1 + off;
    }
    // the indices, read once and validated (the reference raises BoundsError)
    for (int i = tid; i < N; i += kBuildThreads) {
        const int64_t r = load_index(idx, itype, t * tstride + i) - base;
        uint32_t key = sentinel;
        if (r >= 0 && r < (int64_t)nrows) key = (uint32_t)r;
        else raise_index_error(err);
        kbuf[0][i] = key;
        vbuf[0][i] = i;
    }
    __syncthreads();
    PHASE(1);
    radix_pass(N, 0, true, sentinel, kbuf[0], vbuf[0], kbuf[1], vbuf[1], sl);
    int cur = 1;
    if (nbits > 8) {
        if (sl.maxbucket <= kRankBucketMax) {
            // every low-byte bucket is small: order each bucket by (row, position) directly.
            // The stable pass left each bucket in position order, so j < i <=> pos_j < pos_i.
            for (int i = tid; i < N; i += kBuildThreads) {
                const uint32_t ki = kbuf[1][i];
                if (ki == sentinel) {  // invalid indices stay in the last bucket, in order
                    kbuf[0][i] = ki;
                    vbuf[0][i] = vbuf[1][i];
                    continue;
                }
                const int d = ki & 255u;
                const int bs = sl.bucket_start[d], be = sl.bucket_start[d + 1];
                int rank = 0;
                for (int j = bs; j < be; ++j) {
                    const uint32_t kj = kbuf[1][j];
                    rank += (kj < ki || (kj == ki && j < i)) ? 1 : 0;
                }
                kbuf[0][bs + rank] = ki;
                vbuf[0][bs + rank] = vbuf[1][i];
            }
            __syncthreads();
            PHASE(10);
            cur = 0;
        } else {
            // skewed rows: the remaining LSD passes (the sentinel keeps digit 256: stays last)
            for (int shift = 8; shift < nbits; shift += 8) {
                radix_pass(N, shift, false, sentinel, kbuf[cur], vbuf[cur], kbuf[cur ^ 1], vbuf[cur ^ 1], sl);
                cur ^= 1;
            }
        }
    }
    build_segments(ix, t, kbuf[cur], vbuf[cur], N, sentinel, vbuf[cur ^ 1], kbuf[cur ^ 1], sl);
    PHASE(22);
#ifdef DLRM_PHASE
    if (threadIdx.x == 0) g_blk[1][blockIdx.x] = wall_clock64();
#endif
}

template <int NT, int EPL, bool SPLIT = false>
__global__ __launch_bounds__(NT) void indexer_fast_kernel(IndexerDev ix, const TableDesc* __restrict__ tabs,
                                                          const void* __restrict__ idx, int itype, int64_t tstride,
                                                          int base, int N, unsigned* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    FastLds<NT, EPL>& sl = *(FastLds<NT, EPL>*)dyn;
    const int v = blockIdx.x, t = v >> ix.vshift;  // vshift > 0: one workgroup per table part
#ifdef DLRM_PHASE
    if (threadIdx.x == 0) g_blk[0][blockIdx.x] = wall_clock64();
#endif
    PHASE(0);
    fast_index_table<NT, EPL, SPLIT>(ix, v, t, ix.vshift, (uint32_t)tabs[t].nrows, idx, itype, tstride, base, N, err, sl);
#ifdef DLRM_PHASE
    if (threadIdx.x == 0) g_blk[1][blockIdx.x] = wall_clock64();
#endif
}

// ------------------------------------------------------------------------------ apply
// Persistent launch, flat over tables (apply.hpp).  Work items: [0, S) = the S slices of every
// table's hot segments (one workgroup each, handed out first: the longest chains), then
// ceil(C / NG) items of NG chunks (one per lane group), then (singles: a split indexer whose
// once-hit rows are this launch's too) T * ceil(N / (NG * SPPG)) items of once-hit
// positions.  Workgroup b takes items b, b + grid, ...: every item is short, so static striding
// balances, and no workgroup is launched past the work.
// MODE 0: chunks + hot slices; 1: + once-hit (singles) items; 2: + the next batch's split indexer
// in the first (pa.T << pa.ix.vshift) / 4 workgroups (PrepArgs); 3: the same for more than 2048
// positions per table in rounds; 5: the same by the scan build.
#ifndef DLRM_BUILD_PRIO
#define DLRM_BUILD_PRIO 3
#endif
constexpr int kBuildPrio = DLRM_BUILD_PRIO;  // s_setprio of the in-apply build's waves (0..3)

// The build of more than 2048 positions per table: 3 = the scan build (indexer.hpp
// wave_build_group_scan; int32 indices, 16-B aligned per table, N % 4 == 0), the default; 1 = rounds
// (wave_build_group<true>, any index type; DLRM_WAVE_ROUNDS=1 forces it).
static int wave_big_kind(const PrepArgs& pa) {
    if (knobs().wave_rounds) return 1;
    const bool vec32 = pa.itype == DLRM_I32 && (uintptr_t)pa.idx % 16 == 0 && (pa.tstride * 4) % 16 == 0 &&
                       pa.N % 4 == 0;
    return vec32 ? 3 : 1;
}
// workgroups of a build (4 parts each)
__host__ __device__ __forceinline__ int prep_groups(const PrepArgs& pa) { return (pa.T << pa.ix.vshift) / kWaveParts; }

template <typename TT, typename GT, int VPR, int MODE>
__global__ __launch_bounds__(kApplyThreads, 3) void sgd_apply_kernel(IndexerDev ix, TableDesc* __restrict__ tabs, int T_,
                                                                  int L, const GT* __restrict__ grad, int64_t grad_ld,
                                                                  int64_t grad_offset, float lr,
                                                                  const unsigned* __restrict__ err, SinglesArgs sa,
                                                                  PrepArgs pa) {
    constexpr bool SG = MODE == 1;
    int bid = blockIdx.x, nblk = gridDim.x;
    if (MODE >= 2) {
        extern __shared__ __attribute__((aligned(16))) unsigned char prep_lds[];
        const int NI = prep_groups(pa);
        if (bid < NI) {  // the next batch's split build: one wave per table part (indexer.hpp)
            // the build's waves first at the issue arbiter: its chain of dependent LDS / VALU steps is
            // the launch's longest, the apply waves beside it mostly wait on memory (A/B on one box:
            // 54.72 / 54.77 -> 54.91 / 55.04 M samples/s, apply 10.58 -> 10.45 us)
            __builtin_amdgcn_s_setprio(kBuildPrio);
            ITEM_START(4, 0, bid);
            // (MODE 3 / 5: the builds of more than 2048 positions per table, in their own
            // instantiations, so the step's MODE 2 kernel keeps its registers)
            if constexpr (MODE == 5)
                wave_build_group_scan<kWaveParts>(pa.ix, bid, pa.T, pa.tabs, pa.idx, pa.tstride, pa.base, pa.N, pa.err,
                                      *(WaveBuildLds*)prep_lds);
            else
                wave_build_group<MODE == 3>(pa.ix, bid, pa.T, pa.tabs, pa.idx, pa.itype, pa.tstride, pa.base,
                                            pa.N, pa.err, *(WaveBuildLds*)prep_lds);
            ITEM_END(0);
            return;
        }
        bid -= NI;
        nblk -= NI;
#ifdef DLRM_PREP_ONLY  // (probe: the build alone in this launch)
        return;
#endif
    }
    // a bounds error raised since the last dlrm_check_bounds (the lookup or the indexer build of
    // this step): the reference's gather throws before update!, so no table row is written.  (The
    // error word is loaded with the item counts, one round trip for both.)
    const FastDiv Ld(L);  // position -> bag
    unsigned err0 = ldg<unsigned>(err);
    if (ix.build_err) {  // a standalone prepared build's out-of-range indices (written by an earlier launch)
        const unsigned be = ldg<unsigned>(ix.build_err);
        if (be && !err0 && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) raise_index_error((unsigned*)err);
        err0 |= be;
    }
    typedef ApplyGeom<GT, VPR> G;
    constexpr int D = G::D, NG = G::NG;
    __shared__ SliceLds<D> sm;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int g = lane / G::LPR, v = lane % G::LPR;
    const int gid = w * G::RPW + g;
    // where this launch's items are: the wave build's flat item map (one load per item), else a
    // wave scan of every virtual table's counts (TableScan) and a lookup in it per item
    const bool mp = ix.has_map != 0;
    TableScan sS{}, sC{};
    int Stot, Ctot;
    // the item map's sub-list counts (indexer.hpp kResLists), kept in LDS: item_tot[0..8) slices,
    // [8..16) chunks
    __shared__ int lcnt[2 * kResLists];
    const int* ls = lcnt;
    const int* lc = lcnt + kResLists;
    int lstride = 0;
    if (mp) {
        if (threadIdx.x < 2 * kResLists) lcnt[threadIdx.x] = ix.item_tot[threadIdx.x];
        __syncthreads();
        Stot = 0;
        Ctot = 0;
#pragma unroll
        for (int j = 0; j < kResLists; ++j) {
            Stot += ls[j];
            Ctot += lc[j];
        }
        lstride = res_stride(T_ / kWaveParts, ix.cap, ix.vshift);
    } else {
        sS = scan_counts(ix, T_, CNT_S);
        sC = scan_counts(ix, T_, CNT_C);
        Stot = sS.total;
        Ctot = sC.total;
    }
    if (err0) return;
    const int citems = Stot + (Ctot + NG - 1) / NG;
    constexpr int SP = NG * G::SPPG;                           // positions per singles item
    const int per_t = SG ? (sa.N + SP - 1) / SP : 0;          // singles items per real table
    const int items = citems + (T_ >> ix.vshift) * per_t;
    // Pooled bags (L > 1): every position of a bag reads the bag's gradient row, so a table's
    // gradient slice ([B][D]: 2 MB at B = 2048, D = 256 fp32) is read about L times.  Workgroups b
    // and b + 8 share an XCD (and its L2): with the plain stride every XCD walks every table and
    // fetches each slice for itself.  Instead each XCD takes one contiguous eighth of each item
    // kind (hot slices, chunk items, once-hit items) -- about an eighth of the tables -- so a slice
    // is fetched by one L2 and re-read there.  (One-hot: each gradient row is read once; plain.)
    //   item = pos + (pos < e0 ? r0 : pos < e1 ? s1 : s2), pos = this workgroup's list position
    int pos0 = bid, step = nblk, npos = items, r0 = 0, e0 = items, s1 = 0, e1 = items, s2 = 0;
    if (L > 1 && (nblk & 7) == 0 && ((blockIdx.x - bid) & 7) == 0) {
        const int x = bid & 7, c1 = citems - Stot, c2 = items - citems;
        const int a0 = (int)((int64_t)Stot * x >> 3), b0 = (int)((int64_t)Stot * (x + 1) >> 3);
        const int a1 = (int)((int64_t)c1 * x >> 3), b1 = (int)((int64_t)c1 * (x + 1) >> 3);
        const int a2 = (int)((int64_t)c2 * x >> 3), b2 = (int)((int64_t)c2 * (x + 1) >> 3);
        r0 = a0;
        e0 = b0 - a0;
        s1 = Stot + a1 - e0;
        e1 = e0 + (b1 - a1);
        s2 = citems + a2 - e1;
        npos = e1 + (b2 - a2);
        pos0 = bid >> 3;
        step = nblk >> 3;
    }
#ifdef DLRM_PHASE
    int kk_ = 0;
#endif
    for (int pos = pos0; pos < npos; pos += step) {
        const int item = pos + (pos < e0 ? r0 : (pos < e1 ? s1 : s2));
        APPLY_START(item >= citems ? 3 : (item >= Stot ? 1 : 2));
#ifdef DLRM_PHASE
        const int k_ = kk_++;
        ITEM_START(item >= citems ? 3 : (item >= Stot ? 1 : 2), k_, item);
#undef APPLY_END
#define APPLY_END() do { ITEM_END(k_); } while (0)
#endif
        if (SG && item >= citems) {  // uniform: once-hit positions of one real table
            const int t = (item - citems) / per_t;
            const int p0 = ((item - citems) - t * per_t) * SP + gid * G::SPPG;
            if (g >= G::RPW) continue;
            const TableDesc td = load_table(tabs, t);
            run_singles<TT, GT, VPR>(sa, ix.cap, (TT*)td.data, td.nrows, t, p0, grad + grad_offset + (int64_t)t * D,
                                     grad_ld, Ld, lr, v, lane - v);
            APPLY_END();
            continue;
        }
        if (item >= Stot) {
            const int fc = (item - Stot) * NG + gid;  // flat chunk of this lane group
            const int32_t* pbase;
            int4 ca, cb;
            int t;
            if (mp) {  // the flat chunk record: perm entries global, the virtual table = beg / cap
                if (g >= G::RPW || fc >= Ctot) continue;
                const int r = res_locate(lc, fc, lstride);
                ca = ix.chunk_rec[2 * (int64_t)r];
                cb = ix.chunk_rec[2 * (int64_t)r + 1];
                pbase = ix.perm;
                t = (int)(ca.x / ix.cap);  // (the compact layout: entries of table t at [t cap, (t + 1) cap))
            } else {
                int tc, cl;
                locate(ix, T_, CNT_C, sC, fc, tc, cl);
                if (g >= G::RPW || tc < 0) continue;
                const int64_t co = 2 * ((int64_t)tc * ix.cap + cl);
                ca = ix.chunks[co];
                cb = ix.chunks[co + 1];
                pbase = ix.perm + (int64_t)tc * ix.cap;
                t = tc >> ix.vshift;
            }
            run_chunk<TT, GT, VPR>(pbase, ca, cb, (TT*)tabs[t].data, grad + grad_offset + (int64_t)t * D, grad_ld, Ld,
                                   lr, v, lane - v);
            APPLY_END();
            continue;
        }
        if (mp) {  // (uniform: the slice's whole record in one 32-B load)
            const int r = res_locate(ls, item, lstride);
            const int4 r0 = ix.slice_rec[2 * (int64_t)r], r1 = ix.slice_rec[2 * (int64_t)r + 1];
            const int t = r0.w >> ix.vshift;
            run_slice_rec<TT, GT, VPR>(ix, item, item - (r - r1.y), r0, r1, (TT*)tabs[t].data, grad + grad_offset + (int64_t)t * D,
                                       grad_ld, Ld, lr, sm);
            APPLY_END();
            continue;
        }
        int th, sl;
        locate(ix, T_, CNT_S, sS, item, th, sl);  // item < S: found, the same for every lane
        const int4 sd = ix.hot_slice[(int64_t)th * ix.cap + sl];
        const int t = th >> ix.vshift;
        run_slice<TT, GT, VPR>(ix, th, sl, sd, (TT*)tabs[t].data, grad + grad_offset + (int64_t)t * D, grad_ld, Ld, lr,
                               sm);
        APPLY_END();
    }
#ifdef DLRM_PHASE
#undef APPLY_END
#define APPLY_END() do {} while (0)
#endif
}

// The step indexer's workgroups alone (PrepArgs), where the apply has no vector kernel to host them.
// KIND 0: one round (N <= 2048); 1: rounds (the scan build has its own kernel below).
template <int KIND>
__global__ __launch_bounds__(256) void step_index_kernel(PrepArgs pa) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    wave_build_group<KIND == 1>(pa.ix, blockIdx.x, pa.T, pa.tabs, pa.idx, pa.itype, pa.tstride, pa.base, pa.N,
                                    pa.err, *(WaveBuildLds*)lds);
}

// The scan build alone (indexer.hpp wave_build_group_scan), NW waves per workgroup: 16 when every
// workgroup is resident at once (one per CU: its ~94 registers allow 20 waves per CU), else 8 (two
// per CU) -- a second round of workgroups would double the build.
template <int NW, int MAXN>
__global__ __launch_bounds__(64 * NW) void step_index_scan_kernel(PrepArgs pa) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    wave_build_group_scan<NW, MAXN>(pa.ix, blockIdx.x, pa.T, pa.tabs, pa.idx, pa.tstride, pa.base, pa.N, pa.err,
                              *(WaveBuildLds*)lds);
}

template <int NW, int MAXN = kWaveApplyMaxN>
static void launch_step_index_scan(hipStream_t s, const PrepArgs& pa) {
    static const hipError_t attr = hipFuncSetAttribute((const void*)step_index_scan_kernel<NW, MAXN>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)sizeof(WaveBuildLds));
    (void)attr;
    hipLaunchKernelGGL((step_index_scan_kernel<NW, MAXN>), dim3((unsigned)prep_groups(pa)), dim3(64 * NW),
                       sizeof(WaveBuildLds), s, pa);
}

static int pa_cus(const PrepArgs&) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    }
    return cus;
}

template <int KIND>
static void launch_step_index_kind(hipStream_t s, const PrepArgs& pa) {
    static const hipError_t attr = hipFuncSetAttribute((const void*)step_index_kernel<KIND>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)sizeof(WaveBuildLds));
    (void)attr;
    hipLaunchKernelGGL(step_index_kernel<KIND>, dim3((unsigned)prep_groups(pa)), dim3(256),
                       sizeof(WaveBuildLds), s, pa);
}

// step_index_kernel's own launch (the next batch's split build when the apply launch cannot carry it)
static void launch_step_index(hipStream_t s, const PrepArgs& pa) {
    const int kind = pa.N <= kStepIndexMaxN ? 0 : wave_big_kind(pa);
    if (kind == 0) launch_step_index_kind<0>(s, pa);
    else if (kind == 1) launch_step_index_kind<1>(s, pa);
    else if (pa.N > kWaveApplyMaxN)  // (pooled bags: 64 tables x 20480; 16 waves keep 8 pieces each in registers)
        launch_step_index_scan<16, kWaveMaxN>(s, pa);
    else if (prep_groups(pa) <= pa_cus(pa)) launch_step_index_scan<16>(s, pa);
    else launch_step_index_scan<8>(s, pa);
}

// ---------------------------------------------------------------- bag build (8192 < N <= 32768)
// dlrm_indexer_build of many positions per table (configs[4]'s pooled bags: 64 tables x 20480,
// p = b L + k) as three short launches, partition first, so no workgroup reads more than its own
// share of the indices (the scan build reads the whole table once per 4 parts: 64 times at 256
// parts, 183 us for configs[4]; the hash build it replaces took 146 us with 13x its algorithmic
// bytes in global atomics).  P = 2^(wave_vshift(N) - 1) parts per table (128 at 20480):
//   1. count: one workgroup per 2048-position chunk of a table: each valid position's part
//      (row & (P - 1)) counted in LDS; the chunk's P counts -> keys0 [T][chunks][P].  Out-of-range
//      indices raise the bounds flag and are left out.
//   2. place: the same chunks again; each workgroup sums its table's count matrix into the parts'
//      sizes and offsets (the compact layout: part q at the table's positions in parts < q) and
//      its chunk's base in every part, groups the chunk by part in LDS (waves take consecutive
//      quarters, tiles of 64 in order, the lanes of one part ranked by ballots -- match_digit --
//      one cursor per (wave, part)), and writes each part's run of (row >> vs, position) pairs to
//      the HBM scratch (wscratch K0 / V0) in position order.  The chunk-0 workgroup of a table also
//      lists its groups (4 parts) for the sort launch, those with a part too big for LDS first
//      (keys1: the group, its parts' sizes and offsets; two global atomics per table).
//   3. sort: the wave build's last step (wave_sort_part), one wave per part, 4 per workgroup, in
//      that order: a part of <= 512 positions is copied into its quarter of the LDS pool and sorted
//      there (in registers up to 256 keys); a larger one is streamed once: its hot row (the mode
//      of a 64-key sample) straight to perm as one segment, the rest to LDS, sorted and written
//      behind it (wave_sort_part's hot prefix); the general HBM sort only if the rest overflows.
//      Then segments, once-hit flags and the flat item lists, exactly as every wave build's.
constexpr int kBagChunk = 2048;    // positions per count / place workgroup
constexpr int kBagLdsPart = 512;   // a part sorted in LDS (its quarter of the pool), else in HBM
constexpr int kBagSlot = 12;       // ints per entry of the sort's group order (keys1): g, 4 sizes, 4 offsets

__global__ __launch_bounds__(256) void bag_count_kernel(PrepArgs pa, int nch) {
    __shared__ int hist[kSegPad];
    const int c = blockIdx.x, t = blockIdx.y, tid = threadIdx.x;
    const int P = 1 << pa.ix.vshift;
    const uint32_t pmask = (uint32_t)P - 1u;
    if (c == 0 && t == 0 && tid < 16) pa.ix.keys1[tid] = 0u;  // (bag_place's group-order counters)
    for (int q = tid; q < P; q += 256) hist[q] = 0;
    __syncthreads();
    const uint64_t nrows = (uint64_t)load_table(pa.tabs, t).nrows;
    const int p0 = c * kBagChunk;
    int64_t x[kBagChunk / 256];
    bool in[kBagChunk / 256];
#pragma unroll
    for (int i = 0; i < kBagChunk / 256; ++i) {  // (every load in flight)
        const int p = p0 + i * 256 + tid;
        in[i] = p < pa.N;
        x[i] = load_index_if(in[i], pa.idx, pa.itype, (int64_t)t * pa.tstride + p) - pa.base;
    }
    bool bad = false;
#pragma unroll
    for (int i = 0; i < kBagChunk / 256; ++i) {
        const bool ok = in[i] && (uint64_t)x[i] < nrows;
        bad |= in[i] && !ok;
        if (ok) atomicAdd(&hist[(uint32_t)x[i] & pmask], 1);
    }
    if (__ballot(bad) && (tid & 63) == 0) raise_index_error(pa.err);
    __syncthreads();
    int32_t* cg = (int32_t*)pa.ix.keys0 + ((int64_t)t * nch + c) * P;
    for (int q = tid; q < P; q += 256) cg[q] = hist[q];
}

__global__ __launch_bounds__(256) void bag_place_kernel(PrepArgs pa, int nch) {
    __shared__ int cw[kWaveParts][kSegPad];  // per-wave counts, then per-wave cursors in the chunk
    __shared__ int cb[kSegPad];              // part q's entries of this chunk start at cb[q] (table)
    __shared__ int cl[kSegPad];              // ... and at cl[q] in the chunk's staging
    __shared__ uint32_t sx[kBagChunk];       // the chunk grouped by part: rows, positions
    __shared__ int32_t sp[kBagChunk];
    __shared__ int wtot[8];
    const IndexerDev& ix = pa.ix;
    const int c = blockIdx.x, t = blockIdx.y, tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    const int vs = ix.vshift, P = 1 << vs;
    const uint32_t pmask = (uint32_t)P - 1u;
    // this wave's quarter of the chunk (kept in registers), loaded first: its latency overlaps the
    // count matrix's
    const uint64_t nrows = (uint64_t)load_table(pa.tabs, t).nrows;
    constexpr int IT = kBagChunk / 256;  // tiles of 64 per wave
    constexpr uint32_t kBad = 0xffffffffu;
    const int pw = c * kBagChunk + w * (kBagChunk / kWaveParts);
    int64_t xl[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        const int p = pw + i * 64 + lane;
        xl[i] = load_index_if(p < pa.N, pa.idx, pa.itype, (int64_t)t * pa.tstride + p) - pa.base;
    }
    // part q = tid: its size over the table's chunks and the positions of earlier chunks in it
    const int32_t* cg = (const int32_t*)ix.keys0 + (int64_t)t * nch * P;
    int nq = 0, bef = 0, here = 0;
    if (tid < P) {
        int k[kWaveMaxN / kBagChunk];
#pragma unroll
        for (int cc = 0; cc < kWaveMaxN / kBagChunk; ++cc)  // (every load in flight: nch <= 16)
            k[cc] = cc < nch ? cg[(int64_t)cc * P + tid] : 0;
#pragma unroll
        for (int cc = 0; cc < kWaveMaxN / kBagChunk; ++cc) {
            nq += k[cc];
            bef += cc < c ? k[cc] : 0;
            here = cc == c ? k[cc] : here;
        }
    }
    int total;
    const int toff = block_scan_nw<kWaveParts, int>(tid < P ? nq : 0, wtot, &total);
    const int loff = block_scan_nw<kWaveParts, int>(tid < P ? here : 0, wtot, &total);
    if (tid < P) {
        cb[tid] = toff + bef;
        cl[tid] = loff;
    }
    for (int q = tid; q < kWaveParts * kSegPad; q += 256) (&cw[0][0])[q] = 0;
    __syncthreads();
    if (c == 0) {
        // the sort launch's order of this table's groups (4 parts each): those holding a part sorted
        // in HBM (a hot row: its wave's chain is several times a normal part's) go to the front of
        // the order list (keys1 from entry 2 on), the others to the back, so the long chains start first
        // (two global atomics per table reserve its ranges; ranks within the table by a block scan).
        // A slot's entry (kBagSlot ints) carries the group and its parts' sizes and offsets, so the
        // sort's workgroup finds its parts with one load.
        if (tid < P) {
            cw[0][tid] = nq > kBagLdsPart ? 1 : 0;
            cw[2][tid] = nq;
            cw[3][tid] = toff;
        }
        __syncthreads();
        const int G4 = P / kWaveParts;
        bool hot = false;
        if (tid < G4) {
            const int* f = &cw[0][kWaveParts * tid];
            hot = (f[0] | f[1] | f[2] | f[3]) != 0;
        }
        int nhot;
        const int hrank = block_scan_nw<kWaveParts, int>(hot ? 1 : 0, wtot, &nhot);
        // Slots by XCD (T % 8 == 0): the tables of eighth j take the slots g = 8 i + j, i.e. the
        // workgroups on XCD j, whose reservations fill flat sub-list j (indexer.hpp: sub-list = g mod
        // 8).  The apply splits each item kind into eighths by XCD (pooled bags), so each XCD then
        // updates an eighth of the tables and reads their bag gradients into its own L2 only.
        const bool by8 = pa.T % kResLists == 0;
        const int j8 = by8 ? t / (pa.T / kResLists) : 0;
        if (tid == 0) {
            cw[1][0] = (int)atomicAdd(&ix.keys1[2 * j8], (unsigned)nhot);
            cw[1][1] = (int)atomicAdd(&ix.keys1[2 * j8 + 1], (unsigned)(G4 - nhot));
        }
        __syncthreads();
        if (tid < G4) {
            const int groups = (pa.T << vs) / kWaveParts, g = (t << vs) / kWaveParts + tid;
            const int n8 = by8 ? groups / kResLists : groups;  // (slots of this table's eighth)
            const int li = hot ? cw[1][0] + hrank : n8 - 1 - (cw[1][1] + (tid - hrank));
            const int at = by8 ? kResLists * li + j8 : li;
            uint4* e = (uint4*)(ix.keys1 + kBagSlot * (2 + at));
            const int q = kWaveParts * tid;
            e[0] = make_uint4((unsigned)g, 0u, 0u, 0u);
            e[1] = make_uint4(cw[2][q], cw[2][q + 1], cw[2][q + 2], cw[2][q + 3]);
            e[2] = make_uint4(cw[3][q], cw[3][q + 1], cw[3][q + 2], cw[3][q + 3]);
        }
        __syncthreads();
        if (tid < P) cw[0][tid] = cw[2][tid] = cw[3][tid] = 0;
        if (tid < 2) cw[1][tid] = 0;
        __syncthreads();
    }
    // pass 1: this wave's positions per part
    uint32_t xr[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i)
        xr[i] = pw + i * 64 + lane < pa.N && (uint64_t)xl[i] < nrows ? (uint32_t)xl[i] : kBad;
#pragma unroll
    for (int i = 0; i < IT; ++i)
        if (xr[i] != kBad) atomicAdd(&cw[w][xr[i] & pmask], 1);
    __syncthreads();
    if (tid < P) {  // cursors: part q's start in the staging, then the earlier waves' shares
        int run = cl[tid];
#pragma unroll
        for (int ww = 0; ww < kWaveParts; ++ww) {
            const int k = cw[ww][tid];
            cw[ww][tid] = run;
            run += k;
        }
    }
    __syncthreads();
    // pass 2: the chunk into the staging, grouped by part, position order within a part (tiles in
    // order, the lanes of one part ranked by lane)
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        const bool ok = xr[i] != kBad;
        const uint32_t q = xr[i] & pmask;
        const unsigned long long peers = match_digit(q, ok, vs);
        const int rank = __popcll(peers & lanes_below());
        const int base = ok ? cw[w][q] : 0;
        if (ok && rank == 0) cw[w][q] = base + __popcll(peers);
        if (ok) {
            sx[base + rank] = xr[i];
            sp[base + rank] = pw + i * 64 + lane;
        }
    }
    __syncthreads();
    // out: consecutive staged entries of one part go to consecutive slots of its region
    uint32_t* K0 = ix.wscratch + (int64_t)t * ix.cap;
    int32_t* V0 = (int32_t*)ix.wscratch + ix.wstride + (int64_t)t * ix.cap;
    const int m = cw[kWaveParts - 1][P - 1];  // entries staged (the last wave's cursor of the last part)
    for (int i = tid; i < m; i += 256) {
        const uint32_t x = sx[i];
        const uint32_t q = x & pmask;
        const int dst = cb[q] + (i - cl[q]);
        K0[dst] = x >> vs;
        V0[dst] = sp[i];
    }
}

__global__ __launch_bounds__(256) void bag_sort_kernel(PrepArgs pa) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    WaveBuildLds& sl = *(WaveBuildLds*)lds;
    const IndexerDev& ix = pa.ix;
    // (launch slot -> group: the groups with a part sorted in HBM first; the flat lists' sub-list
    // is the launch slot's, so every sub-list still takes its fixed share of the waves)
    const int g = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint4* e = (const uint4*)(ix.keys1 + kBagSlot * (2 + g));
    const uint4 e0 = e[0], e1 = e[1], e2 = e[2];
    const int gg = (int)e0.x;
    const int vs = ix.vshift, gpt = (1 << vs) / kWaveParts;
    const int t = gg / gpt, q0 = (gg - t * gpt) * kWaveParts;
    const int v = (t << vs) + q0 + w;
    const int groups = (pa.T << vs) / kWaveParts;
    const uint32_t nrows = (uint32_t)load_table(pa.tabs, t).nrows;
    const int n = (int)(w == 0 ? e1.x : w == 1 ? e1.y : w == 2 ? e1.z : e1.w);
    const int toff = (int)(w == 0 ? e2.x : w == 1 ? e2.y : w == 2 ? e2.z : e2.w);
    const int64_t S = ix.wstride, o = (int64_t)t * ix.cap + toff;
    uint32_t* K0 = ix.wscratch + o;
    int32_t* V0 = (int32_t*)ix.wscratch + S + o;
    const uint32_t kmax = nrows > 0 ? (nrows - 1) >> vs : 0u;
    const int nbits = 32 - __clz(kmax);
    if (n <= kBagLdsPart) {
        const int pb = w * (kBagLdsPart + 4);  // (16-B aligned quarters of the pool)
        uint32_t* LK0 = sl.K[0] + pb;
        int32_t* LV0 = sl.V[0] + pb;
        uint32_t kk[kBagLdsPart / 64];
        int32_t vv[kBagLdsPart / 64];
#pragma unroll
        for (int j = 0; j < kBagLdsPart / 64; ++j) {  // (every load in flight)
            const int i = 64 * j + lane;
            kk[j] = i < n ? K0[i] : 0u;
            vv[j] = i < n ? V0[i] : 0;
        }
#pragma unroll
        for (int j = 0; j < kBagLdsPart / 64; ++j)
            if (64 * j + lane < n) {
                LK0[64 * j + lane] = kk[j];
                LV0[64 * j + lane] = vv[j];
            }
        wave_lds_sync();
        if (n > kRegSortMax && nbits > 0 && bag_hot_sort<false>(n, nbits, LK0, LV0, sl.K[1] + pb, sl.V[1] + pb))
            wave_sort_part<false, false, true>(ix, v, t, vs, nrows, n, toff, LK0, LV0, sl.K[1] + pb, sl.V[1] + pb,
                                               sl.R + pb, sl.cnt[w], g, groups);
        else
            wave_sort_part<false>(ix, v, t, vs, nrows, n, toff, LK0, LV0, sl.K[1] + pb, sl.V[1] + pb, sl.R + pb,
                                  sl.cnt[w], g, groups);
    } else {
        // A part too big for LDS is nearly always one hot row plus a few hundred others (Zipf rows).
        // The wave streams it once, 512 entries per round trip: the most frequent key of a 64-key
        // sample is taken as the hot row, its positions go straight to perm (one segment, in position
        // order, once-hit flags 0), the others to its LDS quarter; those are then sorted and written
        // as a part with a hot prefix.  If the others overflow the quarter, or the row is not hot
        // after all, the part is sorted in HBM the general way (which rewrites perm and the flags).
        const int pb = w * (kBagLdsPart + 4);
        uint32_t* LK1 = sl.K[1] + pb;
        int32_t* LV1 = sl.V[1] + pb;
        const uint32_t mine = K0[(int64_t)lane * n / 64];
        int cmode = 0;
        for (int j = 0; j < 64; ++j) cmode += __shfl(mine, j, 64) == mine ? 1 : 0;
        int best = (cmode << 6) | lane;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) best = max(best, __shfl_xor(best, d, 64));
        const uint32_t hkey = __shfl(mine, best & 63, 64);
        int32_t* perm = ix.perm + o;
        uint8_t* single = ix.single + (int64_t)t * ix.cap;
        const unsigned long long below = lanes_below();
        int hrun = 0, rrun = 0;
        for (int c0 = 0; c0 < n; c0 += kBagLdsPart) {
            uint32_t kk[kBagLdsPart / 64];
            int32_t vv[kBagLdsPart / 64];
#pragma unroll
            for (int j = 0; j < kBagLdsPart / 64; ++j) {  // (every load of the round in flight)
                const int i = c0 + 64 * j + lane;
                kk[j] = i < n ? K0[i] : ~hkey;
                vv[j] = i < n ? V0[i] : 0;
            }
#pragma unroll
            for (int j = 0; j < kBagLdsPart / 64; ++j) {
                const bool ok = c0 + 64 * j + lane < n;
                const bool hot = ok && kk[j] == hkey;
                const unsigned long long hb = __ballot(hot), rb = __ballot(ok && !hot);
                if (hot) {
                    perm[hrun + __popcll(hb & below)] = vv[j];
                    single[vv[j]] = 0;
                } else if (ok) {
                    const int at = rrun + __popcll(rb & below);
                    if (at < kBagLdsPart) {
                        LK1[at] = kk[j];
                        LV1[at] = vv[j];
                    }
                }
                hrun += __popcll(hb);
                rrun += __popcll(rb);
            }
        }
        if (rrun <= kBagLdsPart && hrun > kChunk && nbits > 0) {
            wave_lds_sync();
            wave_sort_part<false>(ix, v, t, vs, nrows, n, toff, LK1, LV1, sl.K[0] + pb, sl.V[0] + pb, sl.R + pb,
                                  sl.cnt[w], g, groups, hrun, hkey);
        } else {
            uint32_t* K1 = ix.wscratch + 2 * S + o;
            int32_t* V1 = (int32_t*)ix.wscratch + 3 * S + o;
            int32_t* R = (int32_t*)ix.wscratch + 4 * S + o;
            wave_sort_part<true>(ix, v, t, vs, nrows, n, toff, K0, V0, K1, V1, R, sl.cnt[w], g, groups);
        }
    }
}
static_assert(kWaveParts * (kBagLdsPart + 4) <= kStepIndexMaxN + 16, "bag sort: four quarters of the pool");

int launch_bag_build(dlrm_ctx* ctx, const IndexerDev& ix, const TableDesc* tabs, int T_, const void* idx, int itype,
                     int64_t tstride, int base, int N, unsigned* err) {
    if (T_ == 0 || N == 0) return DLRM_OK;
    const int nch = (N + kBagChunk - 1) / kBagChunk;
    if (ix.vshift < 2 || ix.vshift > kWaveMaxVshift || ix.wstride <= 0 || (int64_t)nch * (1 << ix.vshift) > ix.cap ||
        (int64_t)kBagSlot * ((T_ << ix.vshift) / kWaveParts + 2) > (int64_t)T_ * ix.cap)
        return ctx_fail(ctx, DLRM_E_UNSUPPORTED, "bag build: N %d, vshift %d, capacity %lld", N, ix.vshift,
                        (long long)ix.cap);
    const PrepArgs pa{ix, tabs, T_, idx, itype, tstride, base, N, err};
    hipStream_t s = ctx_stream(ctx);
    hipLaunchKernelGGL(bag_count_kernel, dim3((unsigned)nch, (unsigned)T_), dim3(256), 0, s, pa, nch);
    hipLaunchKernelGGL(bag_place_kernel, dim3((unsigned)nch, (unsigned)T_), dim3(256), 0, s, pa, nch);
    static const hipError_t attr = hipFuncSetAttribute((const void*)bag_sort_kernel,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)sizeof(WaveBuildLds));
    (void)attr;
    hipLaunchKernelGGL(bag_sort_kernel, dim3((unsigned)prep_groups(pa)), dim3(256), sizeof(WaveBuildLds), s, pa);
    return ctx_hip(ctx, hipGetLastError(), "bag build launch");
}

// The step's split build alone (dlrm_indexer_prepare): the wave build + item lists, 4 parts per
// workgroup, on the ctx's stream (a caller's side stream: it depends on the indices only).
int launch_step_prepare(dlrm_ctx* ctx, const IndexerDev& ix, const TableDesc* tabs, int T_, const void* idx, int itype,
                        int64_t tstride, int base, int N, unsigned* err) {
    if (T_ == 0 || N == 0) return DLRM_OK;
    const PrepArgs pa{ix, tabs, T_, idx, itype, tstride, base, N, err};
    launch_step_index(ctx_stream(ctx), pa);
    return ctx_hip(ctx, hipGetLastError(), "step_index launch");
}

// Generic (any D) versions: one thread per element column.
template <typename TT, typename GT>
__global__ __launch_bounds__(256) void sgd_chunks_scalar(IndexerDev ix, TableDesc* __restrict__ tabs, int D, int L,
                                                         const GT* __restrict__ grad, int64_t grad_ld,
                                                         int64_t grad_offset, float lr, const unsigned* __restrict__ err) {
    if (ix.build_err && *ix.build_err) {  // (a prepared build's bounds error: raised here, before hot / singles)
        if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) raise_index_error((unsigned*)err);
        return;
    }
    if (*err) return;
    const int t = blockIdx.y;
    const int nchunks = ix.counts[(int64_t)t * 8 + CNT_C];
    const int64_t off = ix.part_off(t);
    const int64_t total = (int64_t)nchunks * D;
    TT* table = (TT*)tabs[t >> ix.vshift].data;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int cid = (int)(e / D), c = (int)(e % D);
        const int4 cd = ix.chunks[2 * (off + cid)];
        float acc = 0.0f;
        for (int i = cd.x; i < cd.y; ++i)
            acc += to_f32(grad[(int64_t)(ix.perm[off + i] / L) * grad_ld + grad_offset + (int64_t)(t >> ix.vshift) * D + c]);
        TT* row = table + (int64_t)(uint32_t)cd.z * D;
        row[c] = from_f32<TT>(__builtin_fmaf(-lr, acc, to_f32(row[c])));
    }
}

template <typename TT, typename GT>
__global__ __launch_bounds__(256) void sgd_hot_scalar(IndexerDev ix, TableDesc* __restrict__ tabs, int D, int L,
                                                      const GT* __restrict__ grad, int64_t grad_ld,
                                                      int64_t grad_offset, float lr, const unsigned* __restrict__ err) {
    if (*err) return;
    const int t = blockIdx.y;
    const int nhot = ix.counts[(int64_t)t * 8 + CNT_H];
    const int64_t off = ix.part_off(t);
    const int64_t total = (int64_t)nhot * D;
    TT* table = (TT*)tabs[t >> ix.vshift].data;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int h = (int)(e / D), c = (int)(e % D);
        const int4 hd = ix.hot[off + h];
        float acc = 0.0f;
        for (int i = hd.x; i < hd.y; ++i)
            acc += to_f32(grad[(int64_t)(ix.perm[off + i] / L) * grad_ld + grad_offset + (int64_t)(t >> ix.vshift) * D + c]);
        TT* row = table + (int64_t)(uint32_t)hd.z * D;
        row[c] = from_f32<TT>(__builtin_fmaf(-lr, acc, to_f32(row[c])));
    }
}

template <typename TT, typename GT>
__global__ __launch_bounds__(256) void sgd_singles_scalar(SinglesArgs sa, int64_t cap, TableDesc* __restrict__ tabs,
                                                          int D, int L, const GT* __restrict__ grad, int64_t grad_ld,
                                                          int64_t grad_offset, float lr,
                                                          const unsigned* __restrict__ err) {
    if (*err) return;
    const int t = blockIdx.y;
    const int64_t total = (int64_t)sa.N * D;
    TT* table = (TT*)tabs[t].data;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(e / D), c = (int)(e % D);
        if (!sa.single[(int64_t)t * cap + p]) continue;
        const int64_t r = load_index(sa.idx, sa.itype, (int64_t)t * sa.tstride + p) - sa.base;
        if (r < 0 || r >= tabs[t].nrows) continue;
        const float g = to_f32(grad[(int64_t)(p / L) * grad_ld + grad_offset + (int64_t)t * D + c]);
        TT* row = table + r * D;
        row[c] = from_f32<TT>(__builtin_fmaf(-lr, 0.0f + g, to_f32(row[c])));
    }
}

// Non-deterministic: every lookup adds -lr * grad straight into its row (fp32 tables).
template <typename GT>
__global__ __launch_bounds__(256) void sgd_atomic_kernel(TableDesc* __restrict__ tabs, int ntab, int D,
                                                         const void* __restrict__ idx, int itype, int64_t tstride,
                                                         int base, int B, int L, const GT* __restrict__ grad,
                                                         int64_t grad_ld, int64_t grad_offset, float lr,
                                                         unsigned* __restrict__ err) {
    if (*err) return;  // raised by validate_indices_kernel (launched first) or an earlier launch
    const int64_t N = (int64_t)B * L;
    const int64_t total = (int64_t)ntab * N * D;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(e % D);
        const int64_t item = e / D;
        const int t = (int)(item / N);
        const int64_t p = item - (int64_t)t * N;
        const int64_t r = load_index(idx, itype, t * tstride + p) - base;
        if (r < 0 || r >= tabs[t].nrows) continue;  // (cannot happen: validated before the launch)
        const float gval = to_f32(grad[(p / L) * grad_ld + grad_offset + (int64_t)t * D + c]);
        unsafeAtomicAdd((float*)tabs[t].data + r * D + c, -lr * gval);
    }
}

// Bounds check of every index before the atomic update (which must not write a row when any
// index of the step is out of range).
__global__ __launch_bounds__(256) void validate_indices_kernel(const TableDesc* __restrict__ tabs, int ntab,
                                                               const void* __restrict__ idx, int itype,
                                                               int64_t tstride, int base, int64_t N,
                                                               unsigned* __restrict__ err) {
    const int64_t total = (int64_t)ntab * N;
    bool bad = false;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int t = (int)(e / N);
        const int64_t r = load_index(idx, itype, t * tstride + (e - (int64_t)t * N)) - base;
        bad |= r < 0 || r >= tabs[t].nrows;
    }
    if (__ballot(bad) && (threadIdx.x & 63) == 0) raise_index_error(err);
}

// ------------------------------------------------------------------------ launchers
size_t indexer_lds_bytes() { return sizeof(uint32_t) * 2 * kLdsSortMax + sizeof(int32_t) * 2 * kLdsSortMax; }

template <int NT, int EPL, bool SPLIT>
static void launch_fast(hipStream_t s, const IndexerDev& ix, const TableDesc* tabs, int T_, const void* idx, int itype,
                        int64_t tstride, int base, int N, unsigned* err) {
    static const hipError_t attr = hipFuncSetAttribute((const void*)indexer_fast_kernel<NT, EPL, SPLIT>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)sizeof(FastLds<NT, EPL>));
    (void)attr;
    hipLaunchKernelGGL((indexer_fast_kernel<NT, EPL, SPLIT>), dim3(T_ << ix.vshift), dim3(NT), sizeof(FastLds<NT, EPL>),
                       s, ix, tabs, idx, itype, tstride, base, N, err);
}

// split: the form dlrm_step_bwd consumes (once-hit positions flagged, their rows left to the
// backward).  stream: NULL = the context's stream.
int launch_indexer_build(dlrm_ctx* ctx, const IndexerDev& ix, const TableDesc* tabs, int T_, const void* idx,
                         int itype, int64_t tstride, int base, int B, int L, bool split, hipStream_t stream) {
    if (T_ == 0) return DLRM_OK;
    hipStream_t s = stream ? stream : ctx_stream(ctx);
    const int64_t N = (int64_t)B * L;
    unsigned* err = ctx_error_word(ctx);
    if (ix.vshift > 0) {  // the caller chose the parts build (kFastMaxN < N <= kPartsMaxN, split)
        if (!split || N > kPartsMaxN)
            return ctx_fail(ctx, DLRM_E_ARG, "indexer parts build: N=%lld split=%d", (long long)N, (int)split);
        launch_fast<1024, 8, true>(s, ix, tabs, T_, idx, itype, tstride, base, (int)N, err);
    } else if (N <= 1024 * 2) {
        if (split) launch_fast<1024, 2, true>(s, ix, tabs, T_, idx, itype, tstride, base, (int)N, err);
        else launch_fast<1024, 2, false>(s, ix, tabs, T_, idx, itype, tstride, base, (int)N, err);
    } else if (N <= kFastMaxN) {  // (8 positions per thread, one workgroup per table: slower than the hash
                                  // build at N = 8192; in 4 parts per table it is the faster one)
        if (split) launch_fast<1024, 4, true>(s, ix, tabs, T_, idx, itype, tstride, base, (int)N, err);
        else launch_fast<1024, 4, false>(s, ix, tabs, T_, idx, itype, tstride, base, (int)N, err);
    } else if (ix.hsize && N <= kHixMaxN) {
        return launch_hix_build(ctx, ix, tabs, T_, idx, itype, tstride, base, (int)N, split, s);
    } else if (split) {
        return ctx_fail(ctx, DLRM_E_UNSUPPORTED, "split indexer build: %lld positions per table", (long long)N);
    } else {
        hipLaunchKernelGGL(indexer_build_kernel<false>, dim3(T_), dim3(kBuildThreads), 0, s, ix, tabs, idx, itype,
                           tstride, base, B, L, err);
    }
    return ctx_hip(ctx, hipGetLastError(), "indexer_build launch");
}

// the apply launch that also carries the next batch's build (MODE >= 2): build workgroups first
template <typename TT, typename GT, int VPR, int MODE>
static void launch_apply_build(hipStream_t s, unsigned grid, const IndexerDev& ix, TableDesc* tabs, int T_, int L,
                               const void* grad, int64_t grad_ld, int64_t grad_offset, float lr, const unsigned* err,
                               const SinglesArgs& sa, const PrepArgs& pa) {
    static const hipError_t attr = hipFuncSetAttribute((const void*)sgd_apply_kernel<TT, GT, VPR, MODE>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)sizeof(WaveBuildLds));
    (void)attr;
    hipLaunchKernelGGL((sgd_apply_kernel<TT, GT, VPR, MODE>), dim3(grid), dim3(kApplyThreads), sizeof(WaveBuildLds), s,
                       ix, tabs, T_, L, (const GT*)grad, grad_ld, grad_offset, lr, err, sa, pa);
}

template <typename TT, typename GT, int VPR>
static void launch_apply_vec(hipStream_t s, const IndexerDev& ix, TableDesc* tabs, int T_, int L, const void* grad,
                             int64_t grad_ld, int64_t grad_offset, float lr, int64_t N, const unsigned* err,
                             const SinglesArgs& sa, const PrepArgs* pa) {
    typedef ApplyGeom<GT, VPR> G;
    // persistent grid: resident workgroups only (never more than the worst-case item count per
    // table: N / kHotSlice + N / (kChunk + 1) + 1 hot slices, N / NG chunk items, singles items)
    const int64_t SP = G::NG * G::SPPG;
    const int64_t ib = (int64_t)T_ * (N / kHotSlice + N / (kMinChunk + 1) + 1 + (N + G::NG - 1) / G::NG) +
                       (sa.single ? (int64_t)(T_ >> ix.vshift) * ((N + SP - 1) / SP) : 0);
    static int per_cu = 0;
    if (!per_cu) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sgd_apply_kernel<TT, GT, VPR, 0>, kApplyThreads,
                                                         0) != hipSuccess || per_cu < 1)
            per_cu = 1;
    }
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    int64_t grid = (int64_t)per_cu * (cus > 0 ? cus : 256);
    if (grid > ib) grid = ib;
    if (grid < 1) grid = 1;
    // (the once-hit items and the next batch's indexer are separate instantiations: the step's
    // apply stays lean)
    if (pa && !sa.single) {
        // MODE 2: <= 2048 positions per table; above, 2 + wave_big_kind (3 rounds, 5 scan)
        const int mode = pa->N <= kStepIndexMaxN ? 2 : 2 + wave_big_kind(*pa);
        const unsigned g2 = (unsigned)(grid + prep_groups(*pa));
        if (mode == 2) launch_apply_build<TT, GT, VPR, 2>(s, g2, ix, tabs, T_, L, grad, grad_ld, grad_offset, lr, err, sa, *pa);
        else if (mode == 5) launch_apply_build<TT, GT, VPR, 5>(s, g2, ix, tabs, T_, L, grad, grad_ld, grad_offset, lr, err, sa, *pa);
        else launch_apply_build<TT, GT, VPR, 3>(s, g2, ix, tabs, T_, L, grad, grad_ld, grad_offset, lr, err, sa, *pa);
    } else if (sa.single) {
        hipLaunchKernelGGL((sgd_apply_kernel<TT, GT, VPR, 1>), dim3((unsigned)grid), dim3(kApplyThreads), 0, s, ix,
                           tabs, T_, L, (const GT*)grad, grad_ld, grad_offset, lr, err, sa, PrepArgs{});
        // MODE 2 has no once-hit items: the next batch's build (if any) gets its own launch
        if (pa) launch_step_index(s, *pa);
    } else {
        hipLaunchKernelGGL((sgd_apply_kernel<TT, GT, VPR, 0>), dim3((unsigned)grid), dim3(kApplyThreads), 0, s, ix,
                           tabs, T_, L, (const GT*)grad, grad_ld, grad_offset, lr, err, sa, PrepArgs{});
    }
}

template <typename TT, typename GT>
static bool dispatch_apply(int vpr, hipStream_t s, const IndexerDev& ix, TableDesc* tabs, int T_, int L,
                           const void* grad, int64_t grad_ld, int64_t grad_offset, float lr, int64_t N,
                           const unsigned* err, const SinglesArgs& sa, const PrepArgs* pa) {
#define DLRM_CASE(V) \
    case V: launch_apply_vec<TT, GT, V>(s, ix, tabs, T_, L, grad, grad_ld, grad_offset, lr, N, err, sa, pa); return true;
    switch (vpr) {
        DLRM_CASE(1) DLRM_CASE(2) DLRM_CASE(4) DLRM_CASE(8) DLRM_CASE(16) DLRM_CASE(32) DLRM_CASE(64) DLRM_CASE(128)
        default: return false;
    }
#undef DLRM_CASE
}

int launch_sgd_apply(dlrm_ctx* ctx, const IndexerDev& ix, TableDesc* tabs, bool tabs_aligned16, int T_, int D,
                     int tdtype, int L, int64_t N, const void* grad, int gdtype, int64_t grad_ld, int64_t grad_offset,
                     float lr, const SinglesArgs& sa, const PrepArgs* pa) {
    if (T_ == 0 || N == 0) return DLRM_OK;
    T_ <<= ix.vshift;  // virtual tables (row-parity halves) of a forward-launch build
    hipStream_t s = ctx_stream(ctx);
    const unsigned* err = ctx_error_word(ctx);
    const int gesz = gdtype == DLRM_F32 ? 4 : 2;
    const int tesz = tdtype == DLRM_F32 ? 4 : 2;
    const bool aligned = tabs_aligned16 && (uintptr_t)grad % 16 == 0 && (grad_ld * gesz) % 16 == 0 &&
                         (grad_offset * gesz) % 16 == 0 && (D * gesz) % 16 == 0 && (D * tesz) % 16 == 0 && D % 4 == 0;
    bool done = false;
    const int64_t slots = (int64_t)T_ * (N + 1);  // (item counts stay in int)
    if (aligned && slots < (1ll << 31)) {
        const int vpr = D * gesz / 16;
        if (tdtype == DLRM_F32 && gdtype == DLRM_F32)
            done = dispatch_apply<float, float>(vpr, s, ix, tabs, T_, L, grad, grad_ld, grad_offset, lr, N, err, sa, pa);
        else if (tdtype == DLRM_BF16 && gdtype == DLRM_F32)
            done = dispatch_apply<uint16_t, float>(vpr, s, ix, tabs, T_, L, grad, grad_ld, grad_offset, lr, N, err, sa, pa);
        else if (tdtype == DLRM_F32 && gdtype == DLRM_BF16)
            done = dispatch_apply<float, uint16_t>(vpr, s, ix, tabs, T_, L, grad, grad_ld, grad_offset, lr, N, err, sa, pa);
        else
            done = dispatch_apply<uint16_t, uint16_t>(vpr, s, ix, tabs, T_, L, grad, grad_ld, grad_offset, lr, N,
                                                      err, sa, pa);
    }
    if (!done && pa) launch_step_index(s, *pa);
    if (!done) {
        const int64_t gx0 = (N * D + 255) / 256;
        const unsigned gx = (unsigned)(gx0 < 1 ? 1 : (gx0 > 4096 ? 4096 : gx0));
        const int64_t hx0 = ((N / (kChunk + 1)) * D + 255) / 256;
        const unsigned hx = (unsigned)(hx0 < 1 ? 1 : (hx0 > 1024 ? 1024 : hx0));
#define DLRM_SCALAR(TT, GT)                                                                                         \
    hipLaunchKernelGGL((sgd_chunks_scalar<TT, GT>), dim3(gx, T_), dim3(256), 0, s, ix, tabs, D, L, (const GT*)grad, \
                       grad_ld, grad_offset, lr, err);                                                              \
    hipLaunchKernelGGL((sgd_hot_scalar<TT, GT>), dim3(hx, T_), dim3(256), 0, s, ix, tabs, D, L, (const GT*)grad,    \
                       grad_ld, grad_offset, lr, err);                                                              \
    if (sa.single)                                                                                                  \
        hipLaunchKernelGGL((sgd_singles_scalar<TT, GT>), dim3(gx, T_ >> ix.vshift), dim3(256), 0, s, sa, ix.cap,    \
                           tabs, D, L, (const GT*)grad, grad_ld, grad_offset, lr, err);
        if (tdtype == DLRM_F32 && gdtype == DLRM_F32) { DLRM_SCALAR(float, float) }
        else if (tdtype == DLRM_BF16 && gdtype == DLRM_F32) { DLRM_SCALAR(uint16_t, float) }
        else if (tdtype == DLRM_F32 && gdtype == DLRM_BF16) { DLRM_SCALAR(float, uint16_t) }
        else { DLRM_SCALAR(uint16_t, uint16_t) }
#undef DLRM_SCALAR
    }
    return ctx_hip(ctx, hipGetLastError(), "sgd_apply launch");
}

int launch_sgd_atomic(dlrm_ctx* ctx, TableDesc* tabs, int T_, int D, const void* idx, int itype, int64_t tstride,
                      int base, int B, int L, const void* grad, int gdtype, int64_t grad_ld, int64_t grad_offset,
                      float lr) {
    if (T_ == 0 || B == 0) return DLRM_OK;
    hipStream_t s = ctx_stream(ctx);
    const int64_t cap = (int64_t)ctx_num_cus(ctx) * 16;
    {
        int64_t gv = ((int64_t)T_ * B * L + 255) / 256;
        if (gv > cap) gv = cap;
        hipLaunchKernelGGL(validate_indices_kernel, dim3((unsigned)gv), dim3(256), 0, s, tabs, T_, idx, itype, tstride,
                           base, (int64_t)B * L, ctx_error_word(ctx));
    }
    const int64_t total = (int64_t)T_ * B * L * D;
    int64_t g = (total + 255) / 256;
    if (g > cap) g = cap;
    if (gdtype == DLRM_F32)
        hipLaunchKernelGGL(sgd_atomic_kernel<float>, dim3((unsigned)g), dim3(256), 0, s, tabs, T_, D, idx, itype, tstride,
                           base, B, L, (const float*)grad, grad_ld, grad_offset, lr, ctx_error_word(ctx));
    else
        hipLaunchKernelGGL(sgd_atomic_kernel<uint16_t>, dim3((unsigned)g), dim3(256), 0, s, tabs, T_, D, idx, itype,
                           tstride, base, B, L, (const uint16_t*)grad, grad_ld, grad_offset, lr, ctx_error_word(ctx));
    return ctx_hip(ctx, hipGetLastError(), "sgd_atomic launch");
}

}  // namespace dlrm
