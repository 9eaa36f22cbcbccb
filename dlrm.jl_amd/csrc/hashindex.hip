// hashindex.hip — SparseIndexer build for large per-table position counts (B*L > kFastMaxN).
//
// Reference: SparseIndexer() + update! (src/train/train.jl:276-290): per table, the lookup
// positions grouped by row (duplicates accumulated before the SGD step, validation.jl:125-146).
// The in-LDS build (indexer.hpp) keeps one table's positions in one workgroup, which caps it
// at 4096 positions and leaves most CUs idle when a table has many more (B = 8192, pooled bags,
// the sharded path's global batch).  This build spreads every table over the whole chip and
// never sorts the rows: the contract is "segments grouped by row, positions ascending within a
// segment, segment order unspecified" (the same arrays the apply reads).
//
//   1. insert (tiles of kHixTile positions per workgroup): rows are first merged in an LDS
//      hash (one entry per distinct row of the tile, with its count), then each distinct row
//      claims a slot of the table's global open-addressing hash (load <= 1/2, linear probing;
//      64-bit slots row << 32 | count: one CAS for a new row, + one add for a present one).
//   2. alloc (one thread per slot): occupied slots get a segment {first perm entry, length}
//      from one 64-bit atomic per workgroup (segment count and position cursor move together,
//      so seg_start stays monotone); chunk (<= kChunk) / hot (> kChunk) descriptors the same
//      way; the slot is reset for the next build.
//   3. place (same tiles): one-position segments are written directly (most rows of a large
//      table); the others are merged per slot in LDS and take one cursor add per slot per tile.
//   4. order: positions within each multi-position segment sorted ascending (the apply sums a
//      row's gradients in position order -> bitwise reproducible): a chunk per 32-lane half
//      wave (rank by shuffles), a hot segment per workgroup (LDS rank sort up to 256
//      positions, an N-bit position bitmap beyond).
// Four short launches, all tables at once; no host synchronisation (graph capturable).
#include "indexer.hpp"

namespace dlrm {

constexpr uint32_t kHixEmpty = 0xffffffffu;  // LDS hash: empty key
constexpr int kHixRankMax = 256;   // hot segments up to this length: LDS rank sort

__device__ __forceinline__ uint32_t hix_hash(uint32_t r, int hbits) { return (r * 0x9E3779B1u) >> (32 - hbits); }

// Adds c positions of row r to its slot (claimed when absent); returns the slot, or -1 only if
// the table were full (load <= 1/2: never).  A slot is one 64-bit word, row << 32 | count, so
// a row's first claim is a single CAS that also stores its count; a present row takes one
// more (no-return) add.  The CAS is the probe (it returns the slot's word): no plain load that
// another XCD's L2 could serve stale.  Random-address atomics leave L2 one 64-B request each
// (~20 G/s chip-wide), so their number per row is what this kernel's time is made of.
constexpr unsigned long long kHixEmpty64 = ~0ull;

__device__ __forceinline__ int hix_insert(unsigned long long* hent, uint32_t r, uint32_t c, int hbits) {
    const uint32_t mask = (hbits >= 32 ? 0xffffffffu : (1u << hbits) - 1u);
    uint32_t h = hix_hash(r, hbits);
    const unsigned long long mine = ((unsigned long long)r << 32) | c;
    for (uint32_t i = 0; i <= mask; ++i) {
        const unsigned long long old = atomicCAS(hent + h, kHixEmpty64, mine);
        if (old == kHixEmpty64) return (int)h;
        if ((uint32_t)(old >> 32) == r) {
            atomicAdd(hent + h, (unsigned long long)c);
            return (int)h;
        }
        h = (h + 1u) & mask;
    }
    return -1;
}

// Workgroup tile: one position per thread.  Rows repeated inside the tile (small tables, hot
// rows) are merged in an LDS hash first; the thread whose CAS created an LDS entry then owns
// that row's global work (one CAS chain + one count add per distinct row per tile), so no
// thread serialises several global round trips and hot rows see no same-address storms.
constexpr int kHixTile = 256;
constexpr int kHixLdsSlots = 2 * kHixTile;

struct HixLds {
    uint32_t key[kHixLdsSlots];
    uint32_t cnt[kHixLdsSlots];
    int32_t val[kHixLdsSlots];
};

// LDS slot of k; *created = this thread claimed it.
__device__ __forceinline__ int hix_lds_insert(HixLds& sl, uint32_t k, bool* created) {
    static_assert(kHixLdsSlots == 512, "LDS hash bits");
    uint32_t h = (k * 0x9E3779B1u) >> (32 - 9);
    for (int i = 0; i < kHixLdsSlots; ++i) {
        const uint32_t old = atomicCAS(&sl.key[h], kHixEmpty, k);
        if (old == kHixEmpty || old == k) {
            *created = old == kHixEmpty;
            return (int)h;
        }
        h = (h + 1u) & (kHixLdsSlots - 1);
    }
    *created = false;
    return -1;
}

__device__ __forceinline__ void hix_lds_clear(HixLds& sl) {
#pragma unroll
    for (int k = 0; k < kHixLdsSlots / 256; ++k) {
        sl.key[threadIdx.x + 256 * k] = kHixEmpty;
        sl.cnt[threadIdx.x + 256 * k] = 0u;
    }
}

// ---------------------------------------------------------------------------- 1. insert
// grid = (ceil(N / kHixTile), T)
__global__ __launch_bounds__(256) void hix_insert_kernel(IndexerDev ix, const TableDesc* __restrict__ tabs,
                                                         const void* __restrict__ idx, int itype, int64_t tstride,
                                                         int base, int N, unsigned* __restrict__ err) {
    __shared__ HixLds sl;
    const int t = blockIdx.y;
    const int tid = threadIdx.x;
    const int p = blockIdx.x * kHixTile + tid;
    if (blockIdx.x == 0 && tid < 8) {
        ix.counts[(int64_t)t * 8 + tid] = 0;
        if (tid < 4) ix.hstate[(int64_t)t * 4 + tid] = 0ull;
    }
    hix_lds_clear(sl);
    const int64_t nrows = load_table(tabs, t).nrows;
    const int64_t r = load_index_if(p < N, idx, itype, t * tstride + p) - base;
    const bool ok = p < N && r >= 0 && r < nrows;
    if (p < N && !ok) raise_index_error(err);
    __syncthreads();
    int ls = -1;
    bool own = false;
    if (ok) {
        ls = hix_lds_insert(sl, (uint32_t)r, &own);
        atomicAdd(&sl.cnt[ls], 1u);
    }
    __syncthreads();
    if (own) sl.val[ls] = hix_insert(ix.hent + (int64_t)t * ix.hsize, (uint32_t)r, sl.cnt[ls], ix.hbits);
    __syncthreads();
    if (p < N) ix.pslot[(int64_t)t * ix.cap + p] = ls >= 0 ? sl.val[ls] : -1;
}

// ----------------------------------------------------------------------------- 2. alloc
// grid = (hsize / (256 * kHixSPT), T), kHixSPT consecutive slots per thread.  SPLIT: one-position
// segments get no chunk (the step backward updates those rows itself, single[] flag written
// by the place pass).
constexpr int kHixSPT = 4;

__global__ __launch_bounds__(256) void hix_alloc_kernel(IndexerDev ix, int split) {
    __shared__ long long wtot64[8];
    __shared__ unsigned long long sbase[4];
    constexpr long long M21 = (1ll << 21) - 1;
    const int t = blockIdx.y;
    const int64_t s0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * kHixSPT;
    const int64_t ho = (int64_t)t * ix.hsize;
    uint32_t c[kHixSPT], row[kHixSPT];
    {
        const ulonglong2 e01 = *(const ulonglong2*)(ix.hent + ho + s0);
        const ulonglong2 e23 = *(const ulonglong2*)(ix.hent + ho + s0 + 2);
        const unsigned long long e[kHixSPT] = {e01.x, e01.y, e23.x, e23.y};
        static_assert(kHixSPT == 4, "two 16-B loads");
#pragma unroll
        for (int q = 0; q < kHixSPT; ++q) {
            c[q] = e[q] == kHixEmpty64 ? 0u : (uint32_t)e[q];
            row[q] = (uint32_t)(e[q] >> 32);
        }
        if (c[0] | c[1] | c[2] | c[3]) {
            const ulonglong2 ones = make_ulonglong2(kHixEmpty64, kHixEmpty64);
            *(ulonglong2*)(ix.hent + ho + s0) = ones;
            *(ulonglong2*)(ix.hent + ho + s0 + 2) = ones;
        }
    }
    long long av = 0, bv = 0;
#pragma unroll
    for (int q = 0; q < kHixSPT; ++q) {
        const bool chunk = c[q] > 0 && c[q] <= (uint32_t)kChunk && !(split && c[q] == 1);
        const bool hot = c[q] > (uint32_t)kChunk;
        const int ns = hot ? (int)((c[q] + kHotSlice - 1) / kHotSlice) : 0;
        av += ((long long)(c[q] ? 1 : 0) << 32) | c[q];
        bv += (chunk ? 1ll : 0ll) | ((hot ? 1ll : 0ll) << 21) | ((long long)ns << 42);
    }
    // (segments << 32 | positions) and (chunks | hot << 21 | slices << 42), block-wide
    long long atot, btot;
    long long aex = block_scan_nw<4, long long>(av, wtot64, &atot);
    long long bex = block_scan_nw<4, long long>(bv, wtot64, &btot);
    if (threadIdx.x < 4) {  // four independent atomics, one per lane (one round trip)
        int32_t* cnt = ix.counts + (int64_t)t * 8;
        const int q = threadIdx.x;
        if (q == 0) {
            sbase[0] = atot ? atomicAdd(ix.hstate + (int64_t)t * 4, (unsigned long long)atot) : 0ull;
        } else {
            const int v = (int)((btot >> (21 * (q - 1))) & M21);
            const int which = q == 1 ? CNT_C : (q == 2 ? CNT_H : CNT_S);
            sbase[q] = v ? (unsigned)atomicAdd(cnt + which, v) : 0u;
        }
    }
    __syncthreads();
    if (!(av | bv)) return;
    const int64_t off = (int64_t)t * ix.cap;
#pragma unroll
    for (int q = 0; q < kHixSPT; ++q) {
        if (!c[q]) continue;
        const bool chunk = c[q] <= (uint32_t)kChunk && !(split && c[q] == 1);
        const bool hot = c[q] > (uint32_t)kChunk;
        const int ns = hot ? (int)((c[q] + kHotSlice - 1) / kHotSlice) : 0;
        const unsigned long long a = sbase[0] + (unsigned long long)aex;
        const int seg = (int)(a >> 32), beg = (int)(a & 0xffffffffu);
        const int end = beg + (int)c[q];
        ix.hseg[ho + s0 + q] = make_int2(beg, (int)c[q]);
        ix.hfill[ho + s0 + q] = 0;
        ix.seg_start[(int64_t)t * (ix.cap + 1) + seg] = beg;
        ix.seg_row[off + seg] = row[q];
        // (a chunk's inline positions are written by the order pass, once they are sorted)
        if (chunk) write_chunk(ix.chunks + 2 * off, (int)sbase[1] + (int)(bex & M21), beg, end, (int)row[q], nullptr);
        if (hot) {
            const int h = (int)sbase[2] + (int)((bex >> 21) & M21);
            const int sl0 = (int)sbase[3] + (int)((bex >> 42) & M21);
            ix.hot[off + h] = make_int4(beg, end, (int)row[q], sl0);
            write_slices(ix.hot_slice + off, sl0, beg, end, (int)row[q], h);
        }
        aex += (1ll << 32) | c[q];
        bex += (chunk ? 1ll : 0ll) | ((hot ? 1ll : 0ll) << 21) | ((long long)ns << 42);
    }
}

// ----------------------------------------------------------------------------- 3. place
// grid = (ceil(N / kHixTile), T).  One-position segments are written directly; the others are
// merged per slot in LDS and take one cursor add per slot per tile (by the entry's owner).
__global__ __launch_bounds__(256) void hix_place_kernel(IndexerDev ix, int N, int split) {
    __shared__ HixLds sl;
    const int t = blockIdx.y;
    const int tid = threadIdx.x;
    const int p = blockIdx.x * kHixTile + tid;
    const int64_t off = (int64_t)t * ix.cap, ho = (int64_t)t * ix.hsize;
    if (blockIdx.x == 0 && tid == 0) {
        const unsigned long long st = ix.hstate[(int64_t)t * 4];
        const int U = (int)(st >> 32), n = (int)(st & 0xffffffffu);
        ix.counts[(int64_t)t * 8 + CNT_U] = U;
        ix.counts[(int64_t)t * 8 + CNT_NV] = n;
        ix.seg_start[(int64_t)t * (ix.cap + 1) + U] = n;
    }
    hix_lds_clear(sl);
    const int s = p < N ? ix.pslot[off + p] : -1;
    const int2 sg = s >= 0 ? ix.hseg[ho + s] : make_int2(0, 0);
    int32_t* perm = ix.perm + off;
    if (split && p < N) ix.single[off + p] = (s >= 0 && sg.y == 1) ? 1 : 0;
    if (s >= 0 && sg.y == 1) perm[sg.x] = p;
    __syncthreads();
    int ls = -1, rk = 0;
    bool own = false;
    if (s >= 0 && sg.y > 1) {
        ls = hix_lds_insert(sl, (uint32_t)s, &own);
        rk = (int)atomicAdd(&sl.cnt[ls], 1u);
    }
    __syncthreads();
    if (own) sl.val[ls] = (int)atomicAdd(ix.hfill + ho + s, sl.cnt[ls]);
    __syncthreads();
    if (ls >= 0) perm[sg.x + sl.val[ls] + rk] = p;
}

// ----------------------------------------------------------------------------- 4. order
// Persistent: items [0, H) = hot segments (one workgroup each), then ceil(C / 16) items of 16
// chunks (two per 32-lane half wave).  Dynamic LDS: max(ceil(N/32), kHixRankMax) words.
__global__ __launch_bounds__(256) void hix_order_kernel(IndexerDev ix, int T_, int N) {
    extern __shared__ uint32_t hix_lds[];
    __shared__ int wtot[8];
    const TableScan sH = scan_counts(ix, T_, CNT_H);
    const TableScan sC = scan_counts(ix, T_, CNT_C);
    const int items = sH.total + (sC.total + 15) / 16;
    const int nw = (N + 31) / 32;
    const int tid = threadIdx.x;
    for (int item = blockIdx.x; item < items; item += gridDim.x) {
        if (item >= sH.total) {
            // two chunks per 32-lane half wave, loads of both issued before either sort
            const int half = tid >> 5, hl = tid & 31;
            int tc[2], cl[2];
            locate(ix, T_, CNT_C, sC, (item - sH.total) * 16 + half, tc[0], cl[0]);
            locate(ix, T_, CNT_C, sC, (item - sH.total) * 16 + 8 + half, tc[1], cl[1]);
            int4 cd[2];
#pragma unroll
            for (int u = 0; u < 2; ++u)
                cd[u] = tc[u] >= 0 ? ix.chunks[2 * ((int64_t)tc[u] * ix.cap + cl[u])] : make_int4(0, 0, 0, 0);
            int v[2];
#pragma unroll
            for (int u = 0; u < 2; ++u)
                v[u] = hl < cd[u].y - cd[u].x ? ix.perm[(int64_t)tc[u] * ix.cap + cd[u].x + hl] : 0x7fffffff;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int len = cd[u].y - cd[u].x;
                int rank = 0;
                for (int i = 0; i < len; ++i) rank += __shfl(v[u], i, 32) < v[u] ? 1 : 0;
                if (hl < len) {
                    const int64_t off = (int64_t)tc[u] * ix.cap;
                    ix.perm[off + cd[u].x + rank] = v[u];
                    if (rank < kChunkInline) ((int*)(ix.chunks + 2 * (off + cl[u])))[3 + rank] = v[u];
                }
            }
            continue;
        }
        int th, hi;
        locate(ix, T_, CNT_H, sH, item, th, hi);
        const int64_t off = (int64_t)th * ix.cap;
        const int4 hd = ix.hot[off + hi];
        int32_t* perm = ix.perm + off;
        const int len = hd.y - hd.x;
        if (len <= kHixRankMax) {
            int* stage = (int*)hix_lds;
            const int v = tid < len ? perm[hd.x + tid] : 0x7fffffff;
            if (tid < len) stage[tid] = v;
            __syncthreads();
            int rank = 0;
            for (int i = 0; i < len; ++i) rank += stage[i] < v ? 1 : 0;
            if (tid < len) perm[hd.x + rank] = v;
            __syncthreads();
            continue;
        }
        for (int k = tid; k < nw; k += 256) hix_lds[k] = 0u;
        __syncthreads();
        for (int i = hd.x + tid; i < hd.y; i += 256) {
            const int q = perm[i];
            atomicOr(hix_lds + (q >> 5), 1u << (q & 31));
        }
        __syncthreads();
        const int W = (nw + 255) / 256;
        int cnt = 0;
        for (int j = 0; j < W; ++j) {
            const int wi = tid * W + j;
            if (wi < nw) cnt += __popc(hix_lds[wi]);
        }
        int tot;
        int o = hd.x + block_scan_nw<4, int>(cnt, wtot, &tot);
        for (int j = 0; j < W; ++j) {
            const int wi = tid * W + j;
            if (wi >= nw) break;
            uint32_t b = hix_lds[wi];
            while (b) {
                perm[o++] = wi * 32 + __builtin_ctz(b);
                b &= b - 1u;
            }
        }
        __syncthreads();  // the bitmap is reused by this workgroup's next item
    }
}

// ------------------------------------------------------------------------------ launch
int64_t hix_table_slots(int64_t cap) {
    int64_t h = 256 * kHixSPT;
    while (h < 2 * cap) h <<= 1;
    return h;
}

int launch_hix_build(dlrm_ctx* ctx, const IndexerDev& ix, const TableDesc* tabs, int T_, const void* idx, int itype,
                     int64_t tstride, int base, int N, bool split, hipStream_t stream) {
    hipStream_t s = stream ? stream : ctx_stream(ctx);
    if (T_ == 0 || N == 0) {
        // empty batch: every table reports zero segments
        if (T_) return ctx_hip(ctx, hipMemsetAsync(ix.counts, 0, sizeof(int32_t) * 8 * T_, s), "memset");
        return DLRM_OK;
    }
    if (!ix.hsize || N > kHixMaxN || (int64_t)N > ix.cap)
        return ctx_fail(ctx, DLRM_E_UNSUPPORTED, "hash indexer: N=%d (cap %lld, hash slots %lld)", N,
                        (long long)ix.cap, (long long)ix.hsize);
    const dim3 gp((N + kHixTile - 1) / kHixTile, T_), gs((unsigned)(ix.hsize / (256 * kHixSPT)), T_);
    hipLaunchKernelGGL(hix_insert_kernel, gp, dim3(256), 0, s, ix, tabs, idx, itype, tstride, base, N,
                       ctx_error_word(ctx));
    hipLaunchKernelGGL(hix_alloc_kernel, gs, dim3(256), 0, s, ix, split ? 1 : 0);
    hipLaunchKernelGGL(hix_place_kernel, gp, dim3(256), 0, s, ix, N, split ? 1 : 0);
    const size_t nw = (size_t)(N + 31) / 32;
    const size_t lds = 4 * (nw > (size_t)kHixRankMax ? nw : (size_t)kHixRankMax);
    static const hipError_t attr = hipFuncSetAttribute((const void*)hix_order_kernel,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 4 * (kHixMaxN / 32));
    (void)attr;
    hipLaunchKernelGGL(hix_order_kernel, dim3(8 * ctx_num_cus(ctx)), dim3(256), lds, s, ix, T_, N);
    return ctx_hip(ctx, hipGetLastError(), "hash indexer launch");
}

}  // namespace dlrm
