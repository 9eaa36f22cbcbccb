// update.hip — SparseIndexer + EmbeddingTables.update!(Descent(lr), ...) on gfx950.
//
// Reference: src/train/train.jl:274-292 (SparseIndexer per table, update! with num_splits /
// nthreads), checked by src/validation.jl:125-146 against the PyTorch `update_emb_*`.
//
//   table_t[r] -= lr * sum_{(b,k): idx_t[b*L+k] - base == r} grad[b][offset + t*D : +D]
//
// Deterministic design (the default):
//  1. indexer_build (one 1024-thread workgroup per table): stable LSD radix sort of the
//     table's B*L lookup positions by row (8-bit digits, only ceil(log2(nrows+1)) key bits,
//     so a 3-row table sorts in one 2-bit pass), keys/values kept in LDS when they fit.
//     Wave-level ranking uses 64-lane ballots (multi-split), cross-wave offsets go through
//     LDS, so equal rows keep ascending positions.  Then, still in the workgroup: unique
//     segments (one per touched row), and a CHUNK work list — segments longer than kChunk
//     positions (hot rows of small tables: a 3-row table gets ~680 hits per row at B=2048)
//     are split so that no wave serialises on a hot row.
//  2. sgd_chunks (grid over all chunks): one lane group per chunk streams its grad rows in
//     ascending position order (fp32 sum, 16-B lanes, 8 rows in flight), then either
//     read-modify-writes the table row once (single-chunk segment) or publishes a partial
//     sum; the last chunk of a hot segment to arrive (agent-scope ticket) adds the
//     partials in chunk order and writes the row once.
// Every touched row is written exactly once, with a summation order fixed by positions:
// bitwise reproducible.  DLRM_UPDATE_ATOMIC instead adds -lr*g straight into the table
// with global_atomic_add_f32 (no sort, non-deterministic rounding order).
#include "common.hpp"

namespace dlrm {

constexpr int kBuildThreads = 1024;
constexpr int kBuildWaves = kBuildThreads / 64;
constexpr int kChunk = 32;          // positions per chunk
constexpr int kLdsSortMax = 2048;   // positions per table sorted entirely in LDS

enum { CNT_U = 0, CNT_C = 1, CNT_H = 2, CNT_HC = 3, CNT_NV = 4 };

// Exclusive scan over the 1024 threads of the block; returns this thread's prefix, total in *tot.
__device__ __forceinline__ int block_scan_excl(int v, int* wtot, int* tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) wtot[w] = x;
    __syncthreads();
    if (w == 0) {
        int t = lane < kBuildWaves ? wtot[lane] : 0;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(t, off, 64);
            if (lane >= off) t += y;
        }
        if (lane < kBuildWaves) wtot[kBuildWaves + lane] = t;  // inclusive wave totals
    }
    __syncthreads();
    const int before = w ? wtot[kBuildWaves + w - 1] : 0;
    *tot = wtot[2 * kBuildWaves - 1];
    __syncthreads();  // wtot reusable after return
    return before + x - v;
}

constexpr int kDigits = 257;        // 256 row digits + 1 bucket that keeps invalid indices last
constexpr int kRankBucketMax = 64;  // within-bucket rank sort when every bucket is this small

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

// Exclusive scan of a 64-bit value over the 1024 threads (three packed 21-bit counters).
__device__ __forceinline__ long long block_scan_excl64(long long v, long long* wtot, long long* tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    long long x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const long long y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) wtot[w] = x;
    __syncthreads();
    if (w == 0) {
        long long t = lane < kBuildWaves ? wtot[lane] : 0;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const long long y = __shfl_up(t, off, 64);
            if (lane >= off) t += y;
        }
        if (lane < kBuildWaves) wtot[kBuildWaves + lane] = t;
    }
    __syncthreads();
    const long long before = w ? wtot[kBuildWaves + w - 1] : 0;
    *tot = wtot[2 * kBuildWaves - 1];
    __syncthreads();
    return before + x - v;
}

// Segments + chunk/hot work lists from a table's sorted (row, position) arrays; one
// 1024-thread workgroup per table.  K/V may live in LDS or global memory.
__device__ void build_segments(const IndexerDev& ix, int t, const uint32_t* K, const int32_t* V, int N,
                               uint32_t sentinel, SortLds& sl) {
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
        const int ex = block_scan_excl(head ? 1 : 0, sl.wtot, &tot);
        if (head) {
            seg_start[U + ex] = i;
            seg_row[U + ex] = k;
        }
        U += tot;
    }
    __syncthreads();
    const int nvalid = sl.nvalid;
    if (tid == 0) seg_start[U] = nvalid;
    __syncthreads();
    int4* chunks = ix.chunks + off;
    uint32_t* hot_row = ix.hot_row + off;
    int32_t* hot_slot0 = ix.hot_slot0 + off;
    int32_t* hot_n = ix.hot_n + off;
    long long C = 0, H = 0, HC = 0;
    constexpr long long M21 = (1ll << 21) - 1;
    for (int tile = 0; tile < U; tile += kBuildThreads) {
        const int s = tile + tid;
        int beg = 0, end = 0;
        if (s < U) { beg = seg_start[s]; end = seg_start[s + 1]; }
        const int nch = (end - beg + kChunk - 1) / kChunk;
        const bool hot = nch > 1;
        // one scan of three packed counters: chunks | hot segments | hot chunks (each < 2^21 per tile)
        const long long packed = (long long)nch | ((long long)(hot ? 1 : 0) << 21) | ((long long)(hot ? nch : 0) << 42);
        long long tot;
        const long long ex = block_scan_excl64(packed, sl.wtot64, &tot);
        const long long c0 = ex & M21, h0 = (ex >> 21) & M21, hc0 = (ex >> 42) & M21;
        if (s < U) {
            const uint32_t row = seg_row[s];
            for (int k = 0; k < nch; ++k) {
                const int cid = (int)(C + c0 + k);
                const int b0 = beg + k * kChunk;
                chunks[cid] = make_int4(b0, b0 + kChunk < end ? b0 + kChunk : end, hot ? (int)(H + h0) : (int)row,
                                        hot ? (int)(HC + hc0 + k) : -1);
            }
            if (hot) {
                hot_row[H + h0] = row;
                hot_slot0[H + h0] = (int)(HC + hc0);
                hot_n[H + h0] = nch;
                ix.hot_cnt[off + H + h0] = 0;  // arrival counter, reset every build
            }
        }
        C += tot & M21; H += (tot >> 21) & M21; HC += (tot >> 42) & M21;
    }
    if (tid == 0) {
        int32_t* cnt = ix.counts + (int64_t)t * 8;
        cnt[CNT_U] = U; cnt[CNT_C] = (int)C; cnt[CNT_H] = (int)H; cnt[CNT_HC] = (int)HC; cnt[CNT_NV] = nvalid;
    }
}

// One stable counting-sort pass of (key, val) by digit(key); digit 256 = invalid index.
// Tiles of 1024 positions in order; per wave the lanes sharing a digit are found with
// 9 ballots (multi-split), the cross-wave offsets go through LDS.
template <typename GetKV>
__device__ void radix_pass(int N, int shift, bool first_pass, uint32_t sentinel, GetKV get, uint32_t* kout,
                           int32_t* vout, SortLds& sl) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const unsigned long long lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int d = tid; d < kDigits; d += kBuildThreads) sl.hist[d] = 0;
    __syncthreads();
    for (int i = tid; i < N; i += kBuildThreads) {
        uint32_t key;
        int32_t val;
        get(i, key, val);
        atomicAdd(&sl.hist[key == sentinel ? 256 : (key >> shift) & 255u], 1);
    }
    __syncthreads();
    {
        const int v = tid < kDigits ? sl.hist[tid] : 0;
        int tot;
        const int ex = block_scan_excl(v, sl.wtot, &tot);
        if (tid < kDigits) {
            sl.digit_off[tid] = ex;
            if (first_pass) sl.bucket_start[tid] = ex;
        }
        if (first_pass && tid == 0) sl.bucket_start[kDigits] = N;
        if (first_pass) {
            // largest valid-row bucket (decides rank sort vs more radix passes)
            int m = tid < 256 ? v : 0;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
            if (tid == 0) sl.maxbucket = 0;
            __syncthreads();
            if (lane == 0 && m > 0) atomicMax(&sl.maxbucket, m);
        }
        __syncthreads();
    }
    for (int tile = 0; tile < N; tile += kBuildThreads) {
        const int i = tile + tid;
        const bool valid = i < N;
        uint32_t key = 0;
        int32_t val = 0;
        if (valid) get(i, key, val);
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
    }
}

template <bool IN_LDS>
__global__ __launch_bounds__(kBuildThreads) void indexer_build_kernel(
    IndexerDev ix, const TableDesc* __restrict__ tabs, const void* __restrict__ idx, int itype,
    int64_t tstride, int base, int B, int L, unsigned* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    __shared__ SortLds sl;
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
    // pass 0 straight from the index array (validated here)
    auto get0 = [&](int i, uint32_t& key, int32_t& val) {
        const int64_t r = load_index(idx, itype, t * tstride + i) - base;
        key = (r >= 0 && r < (int64_t)nrows) ? (uint32_t)r : sentinel;
        val = i;
    };
    for (int i = tid; i < N; i += kBuildThreads) {  // report invalid indices once
        uint32_t k;
        int32_t v;
        get0(i, k, v);
        if (k == sentinel) raise_index_error(err);
    }
    radix_pass(N, 0, true, sentinel, get0, kbuf[1], vbuf[1], sl);
    int cur = 1;
    if (nbits > 8) {
        if (sl.maxbucket <= kRankBucketMax) {
            // every low-byte bucket is small: order each bucket by (row, position) directly.
            // Stable pass 0 left each bucket in position order, so j < i <=> pos_j < pos_i.
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
            cur = 0;
        } else {
            // skewed rows: remaining LSD passes (invalid indices keep digit 256 -> stay last)
            for (int shift = 8; shift < nbits; shift += 8) {
                const uint32_t* kin = kbuf[cur];
                const int32_t* vin = vbuf[cur];
                auto get = [&](int i, uint32_t& key, int32_t& val) { key = kin[i]; val = vin[i]; };
                radix_pass(N, shift, false, sentinel, get, kbuf[cur ^ 1], vbuf[cur ^ 1], sl);
                cur ^= 1;
            }
        }
    }
    build_segments(ix, t, kbuf[cur], vbuf[cur], N, sentinel, sl);
}

// Row read-modify-write of NE consecutive elements at element offset c0: row -= lr * acc,
// one fma per element, 16-B (or 8-B) vector accesses.
template <typename TT, int NE>
__device__ __forceinline__ void rmw_row(TT* row, int c0, const float* acc, float lr) {
    constexpr int BYTES = (int)sizeof(TT) * NE;
    if constexpr (BYTES % 16 == 0) {
        typedef Vec<TT> V;
        constexpr int NV = BYTES / 16;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            typename V::type* p = (typename V::type*)(row + c0) + k;
            float f[V::N];
            V::to_f32(*p, f);
#pragma unroll
            for (int e = 0; e < V::N; ++e) f[e] = __builtin_fmaf(-lr, acc[k * V::N + e], f[e]);
            *p = V::from_f32(f);
        }
    } else {
#pragma unroll
        for (int e = 0; e < NE; ++e) row[c0 + e] = from_f32<TT>(__builtin_fmaf(-lr, acc[e], to_f32(row[c0 + e])));
    }
}

// ------------------------------------------------------------------------------ apply
template <typename TT, typename GT, int VPR>
struct ApplyGeom {
    typedef Vec<GT> GV;
    static constexpr int LPR = VPR <= 64 ? VPR : 64;
    static constexpr int VPL = VPR <= 64 ? 1 : VPR / 64;
    static constexpr int RPW = 64 / LPR;
};

// grad rows are fp32 or bf16; D elements = VPR vectors of 16 B of the GRAD dtype.
// One lane group per chunk, no loop over chunks: the grid covers the worst case (one chunk per
// lookup) and groups past the table's chunk count exit at once.  The dependency chain is
// descriptor -> {positions -> grad rows, table row} -> write, with up to 8 grad rows in flight.
template <typename TT, int NE>
__device__ __forceinline__ void load_row(const TT* row, int c0, float* f) {
    constexpr int BYTES = (int)sizeof(TT) * NE;
    if constexpr (BYTES % 16 == 0) {
        typedef Vec<TT> V;
#pragma unroll
        for (int k = 0; k < BYTES / 16; ++k) V::to_f32(*((const typename V::type*)(row + c0) + k), f + k * V::N);
    } else {
#pragma unroll
        for (int e = 0; e < NE; ++e) f[e] = to_f32(row[c0 + e]);
    }
}

template <typename TT, int NE>
__device__ __forceinline__ void store_row(TT* row, int c0, const float* f) {
    constexpr int BYTES = (int)sizeof(TT) * NE;
    if constexpr (BYTES % 16 == 0) {
        typedef Vec<TT> V;
#pragma unroll
        for (int k = 0; k < BYTES / 16; ++k) *((typename V::type*)(row + c0) + k) = V::from_f32(f + k * V::N);
    } else {
#pragma unroll
        for (int e = 0; e < NE; ++e) row[c0 + e] = from_f32<TT>(f[e]);
    }
}

template <typename TT, typename GT, int VPR>
__global__ __launch_bounds__(256) void sgd_chunks_kernel(IndexerDev ix, TableDesc* __restrict__ tabs, int L,
                                                         const GT* __restrict__ grad, int64_t grad_ld,
                                                         int64_t grad_offset, float lr, float* __restrict__ partial) {
    typedef ApplyGeom<TT, GT, VPR> G;
    typedef typename G::GV GV;
    constexpr int NE = GV::N;
    constexpr int D = VPR * NE;
    constexpr int U = 8;
    const int t = blockIdx.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int g = lane / G::LPR, v = lane % G::LPR;
    if (g >= G::RPW) return;
    const int cid = (blockIdx.x * (blockDim.x >> 6) + w) * G::RPW + g;
    const int nchunks = ix.counts[(int64_t)t * 8 + CNT_C];
    if (cid >= nchunks) return;
    const int64_t off = (int64_t)t * ix.cap;
    const int4 cd = ix.chunks[off + cid];
    const int beg = cd.x, end = cd.y, slot = cd.w;
    TT* row = (TT*)tabs[t].data + (slot < 0 ? (int64_t)(uint32_t)cd.z * D : 0);
    // table row early: its latency overlaps the position -> gradient chain
    float tv[G::VPL][NE];
    if (slot < 0) {
#pragma unroll
        for (int j = 0; j < G::VPL; ++j) load_row<TT, NE>(row, (v + j * 64) * NE, tv[j]);
    }
    const int32_t* perm = ix.perm + off;
    const GT* gbase = grad + grad_offset + (int64_t)t * D;
    float acc[G::VPL][NE];
#pragma unroll
    for (int j = 0; j < G::VPL; ++j)
#pragma unroll
        for (int e = 0; e < NE; ++e) acc[j][e] = 0.0f;
    for (int i = beg; i < end; i += U) {
        int32_t p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = (i + u < end) ? perm[i + u] : -1;
        typename GV::type gv[U][G::VPL];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (p[u] >= 0) {
                const GT* gr = gbase + (int64_t)(p[u] / L) * grad_ld;
#pragma unroll
                for (int j = 0; j < G::VPL; ++j) gv[u][j] = *((const typename GV::type*)gr + v + j * 64);
            }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (p[u] >= 0) {
#pragma unroll
                for (int j = 0; j < G::VPL; ++j) {
                    float f[NE];
                    GV::to_f32(gv[u][j], f);
#pragma unroll
                    for (int e = 0; e < NE; ++e) acc[j][e] += f[e];  // ascending position order
                }
            }
    }
    if (slot < 0) {
#pragma unroll
        for (int j = 0; j < G::VPL; ++j) {
#pragma unroll
            for (int e = 0; e < NE; ++e) tv[j][e] = __builtin_fmaf(-lr, acc[j][e], tv[j][e]);
            store_row<TT, NE>(row, (v + j * 64) * NE, tv[j]);
        }
    } else {
        float* pr = partial + ((int64_t)t * ix.hot_cap + slot) * D;
#pragma unroll
        for (int j = 0; j < G::VPL; ++j)
#pragma unroll
            for (int e = 0; e < NE; e += 4)
                *(f32x4*)(pr + (v + j * 64) * NE + e) = f32x4{acc[j][e], acc[j][e + 1], acc[j][e + 2], acc[j][e + 3]};
    }
    // Hot rows: every chunk published its partial; the LAST chunk to arrive adds all partials
    // of the segment in chunk order (deterministic whatever the arrival order) and writes the
    // row once.  Hand-off = cdna_hip_programming.md Guideline 16: stores drained, agent-scope
    // release, relaxed agent atomic ticket; the last arriver takes an agent-scope acquire
    // before reading the other chunks' partials.  Placement-independent.
    const bool hot = slot >= 0;
    if (!__any(hot)) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the fence's own wait may be dropped (G16 P12)
    const int h = cd.z;
    int old = -1;
    if (hot && v == 0) old = __hip_atomic_fetch_add(ix.hot_cnt + off + h, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __shfl(old, g * G::LPR, 64);
    const int n = hot ? ix.hot_n[off + h] : 0;
    const bool last = hot && old == n - 1;
    if (!__any(last)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!last) return;
    const int s0 = ix.hot_slot0[off + h];
    TT* hrow = (TT*)tabs[t].data + (int64_t)ix.hot_row[off + h] * D;
    const float* p0 = partial + ((int64_t)t * ix.hot_cap + s0) * D;
#pragma unroll
    for (int j = 0; j < G::VPL; ++j) {
        const int c0 = (v + j * 64) * NE;
        float hv[NE], sum[NE];
        load_row<TT, NE>(hrow, c0, hv);
#pragma unroll
        for (int e = 0; e < NE; ++e) sum[e] = 0.0f;
        for (int k = 0; k < n; k += 4) {
            f32x4 pv[4][NE / 4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (k + u < n)
#pragma unroll
                    for (int e = 0; e < NE; e += 4) pv[u][e / 4] = *(const f32x4*)(p0 + (int64_t)(k + u) * D + c0 + e);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (k + u < n)
#pragma unroll
                    for (int e = 0; e < NE; ++e) sum[e] += pv[u][e / 4][e % 4];
        }
#pragma unroll
        for (int e = 0; e < NE; ++e) hv[e] = __builtin_fmaf(-lr, sum[e], hv[e]);
        store_row<TT, NE>(hrow, c0, hv);
    }
    if (v == 0) __hip_atomic_store(ix.hot_cnt + off + h, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Generic (any D) versions: one thread per element column, loops over the chunk.
template <typename TT, typename GT>
__global__ __launch_bounds__(256) void sgd_chunks_scalar(IndexerDev ix, TableDesc* __restrict__ tabs, int D, int L,
                                                         const GT* __restrict__ grad, int64_t grad_ld,
                                                         int64_t grad_offset, float lr, float* __restrict__ partial) {
    const int t = blockIdx.y;
    const int nchunks = ix.counts[(int64_t)t * 8 + CNT_C];
    const int64_t off = (int64_t)t * ix.cap;
    const int64_t total = (int64_t)nchunks * D;
    TT* table = (TT*)tabs[t].data;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int cid = (int)(e / D), c = (int)(e % D);
        const int4 cd = ix.chunks[off + cid];
        const int beg = cd.x, end = cd.y;
        float acc = 0.0f;
        for (int i = beg; i < end; ++i) {
            const int64_t b = ix.perm[off + i] / L;
            acc += to_f32(grad[b * grad_ld + grad_offset + (int64_t)t * D + c]);
        }
        const int slot = cd.w;
        if (slot < 0) {
            TT* row = table + (int64_t)(uint32_t)cd.z * D;
            row[c] = from_f32<TT>(__builtin_fmaf(-lr, acc, to_f32(row[c])));
        } else {
            partial[((int64_t)t * ix.hot_cap + slot) * D + c] = acc;
        }
    }
}

template <typename TT>
__global__ __launch_bounds__(256) void sgd_hot_scalar(IndexerDev ix, TableDesc* __restrict__ tabs, int D, float lr,
                                                      const float* __restrict__ partial) {
    const int t = blockIdx.y;
    const int nhot = ix.counts[(int64_t)t * 8 + CNT_H];
    const int64_t off = (int64_t)t * ix.cap;
    const int64_t total = (int64_t)nhot * D;
    TT* table = (TT*)tabs[t].data;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int h = (int)(e / D), c = (int)(e % D);
        const int s0 = ix.hot_slot0[off + h], n = ix.hot_n[off + h];
        float acc = 0.0f;
        for (int k = 0; k < n; ++k) acc += partial[((int64_t)t * ix.hot_cap + s0 + k) * D + c];
        TT* row = table + (int64_t)ix.hot_row[off + h] * D;
        row[c] = from_f32<TT>(__builtin_fmaf(-lr, acc, to_f32(row[c])));
    }
}

// Non-deterministic: every lookup adds -lr * grad straight into its row (fp32 tables).
template <typename GT>
__global__ __launch_bounds__(256) void sgd_atomic_kernel(TableDesc* __restrict__ tabs, int ntab, int D,
                                                         const void* __restrict__ idx, int itype, int64_t tstride,
                                                         int base, int B, int L, const GT* __restrict__ grad,
                                                         int64_t grad_ld, int64_t grad_offset, float lr,
                                                         unsigned* __restrict__ err) {
    const int64_t N = (int64_t)B * L;
    const int64_t total = (int64_t)ntab * N * D;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(e % D);
        const int64_t item = e / D;
        const int t = (int)(item / N);
        const int64_t p = item - (int64_t)t * N;
        const int64_t r = load_index(idx, itype, t * tstride + p) - base;
        if (r < 0 || r >= tabs[t].nrows) {
            if (c == 0) raise_index_error(err);
            continue;
        }
        const float gval = to_f32(grad[(p / L) * grad_ld + grad_offset + (int64_t)t * D + c]);
        unsafeAtomicAdd((float*)tabs[t].data + r * D + c, -lr * gval);
    }
}

// ------------------------------------------------------------------------ launchers
size_t indexer_lds_bytes() { return sizeof(uint32_t) * 2 * kLdsSortMax + sizeof(int32_t) * 2 * kLdsSortMax; }
int indexer_chunk() { return kChunk; }

int launch_indexer_build(dlrm_ctx* ctx, const IndexerDev& ix, const TableDesc* tabs, int T_, const void* idx,
                         int itype, int64_t tstride, int base, int B, int L) {
    if (T_ == 0) return DLRM_OK;
    hipStream_t s = ctx_stream(ctx);
    const int64_t N = (int64_t)B * L;
    if (N <= kLdsSortMax)
        hipLaunchKernelGGL(indexer_build_kernel<true>, dim3(T_), dim3(kBuildThreads), indexer_lds_bytes(), s, ix, tabs,
                           idx, itype, tstride, base, B, L, ctx_error_word(ctx));
    else
        hipLaunchKernelGGL(indexer_build_kernel<false>, dim3(T_), dim3(kBuildThreads), 0, s, ix, tabs, idx, itype,
                           tstride, base, B, L, ctx_error_word(ctx));
    return ctx_hip(ctx, hipGetLastError(), "indexer_build launch");
}

template <typename TT, typename GT, int VPR>
static void launch_apply_vec(hipStream_t s, const IndexerDev& ix, TableDesc* tabs, int T_, int L, const void* grad,
                             int64_t grad_ld, int64_t grad_offset, float lr, float* partial, int64_t N) {
    typedef ApplyGeom<TT, GT, VPR> G;
    const int per_block = 4 * G::RPW;  // 4 waves x RPW lane groups, one chunk each
    const int64_t gx = (N + per_block - 1) / per_block;
    hipLaunchKernelGGL((sgd_chunks_kernel<TT, GT, VPR>), dim3((unsigned)(gx < 1 ? 1 : gx), T_), dim3(256), 0, s, ix,
                       tabs, L, (const GT*)grad, grad_ld, grad_offset, lr, partial);
}

template <typename TT, typename GT>
static bool dispatch_apply(int vpr, hipStream_t s, const IndexerDev& ix, TableDesc* tabs, int T_, int L,
                           const void* grad, int64_t grad_ld, int64_t grad_offset, float lr, float* partial, int64_t N) {
#define DLRM_CASE(V) \
    case V: launch_apply_vec<TT, GT, V>(s, ix, tabs, T_, L, grad, grad_ld, grad_offset, lr, partial, N); return true;
    switch (vpr) {
        DLRM_CASE(1) DLRM_CASE(2) DLRM_CASE(4) DLRM_CASE(8) DLRM_CASE(16) DLRM_CASE(32) DLRM_CASE(64) DLRM_CASE(128)
        default: return false;
    }
#undef DLRM_CASE
}

int launch_sgd_apply(dlrm_ctx* ctx, const IndexerDev& ix, TableDesc* tabs, bool tabs_aligned16, int T_, int D,
                     int tdtype, int L, int64_t N, const void* grad, int gdtype, int64_t grad_ld, int64_t grad_offset,
                     float lr, float* partial) {
    if (T_ == 0 || N == 0) return DLRM_OK;
    hipStream_t s = ctx_stream(ctx);
    const int gesz = gdtype == DLRM_F32 ? 4 : 2;
    const bool aligned = tabs_aligned16 && (uintptr_t)grad % 16 == 0 && (grad_ld * gesz) % 16 == 0 &&
                         (grad_offset * gesz) % 16 == 0 && (D * gesz) % 16 == 0;
    bool done = false;
    if (aligned) {
        const int vpr = D * gesz / 16;
        if (tdtype == DLRM_F32 && gdtype == DLRM_F32)
            done = dispatch_apply<float, float>(vpr, s, ix, tabs, T_, L, grad, grad_ld, grad_offset, lr, partial, N);
        else if (tdtype == DLRM_BF16 && gdtype == DLRM_F32)
            done = dispatch_apply<uint16_t, float>(vpr, s, ix, tabs, T_, L, grad, grad_ld, grad_offset, lr, partial, N);
        else if (tdtype == DLRM_F32 && gdtype == DLRM_BF16)
            done = dispatch_apply<float, uint16_t>(vpr, s, ix, tabs, T_, L, grad, grad_ld, grad_offset, lr, partial, N);
        else
            done = dispatch_apply<uint16_t, uint16_t>(vpr, s, ix, tabs, T_, L, grad, grad_ld, grad_offset, lr, partial, N);
    }
    if (!done) {
        const int64_t gx0 = (N * D + 255) / 256;
        const unsigned gx = (unsigned)(gx0 < 1 ? 1 : (gx0 > 4096 ? 4096 : gx0));
        const int64_t hx0 = (ix.hot_cap * D + 255) / 256;
        const unsigned hx = (unsigned)(hx0 < 1 ? 1 : (hx0 > 1024 ? 1024 : hx0));
#define DLRM_SCALAR(TT, GT)                                                                                        \
    hipLaunchKernelGGL((sgd_chunks_scalar<TT, GT>), dim3(gx, T_), dim3(256), 0, s, ix, tabs, D, L, (const GT*)grad, \
                       grad_ld, grad_offset, lr, partial);                                                          \
    hipLaunchKernelGGL((sgd_hot_scalar<TT>), dim3(hx, T_), dim3(256), 0, s, ix, tabs, D, lr, partial);
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
    const int64_t total = (int64_t)T_ * B * L * D;
    int64_t g = (total + 255) / 256;
    const int64_t cap = (int64_t)ctx_num_cus(ctx) * 16;
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
