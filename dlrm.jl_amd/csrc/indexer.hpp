// indexer.hpp — the in-LDS SparseIndexer build (one workgroup per table, N <= 4096 positions),
// shared by the standalone indexer launch (update.hip) and the backward launch that builds the
// indexer in the same grid (interact.hip).  See update.hip for the apply that consumes it.
#pragma once
#include "common.hpp"

#ifndef PHASE
#define PHASE(k) do {} while (0)
#endif
#ifndef WPH
#define WPH(k) do {} while (0)
#endif

#include "bitonic.hpp"

namespace dlrm {

#ifndef DLRM_CHUNK
#define DLRM_CHUNK 32
#endif
constexpr int kChunk = DLRM_CHUNK;  // max positions of a segment handled by one lane group
// The wave build's chunk limit is chosen per indexer at run time (IndexerDev::chunk_max: 16 or 32,
// dlrm_indexer_set_chunk; round 6): at 16, segments of 17..32 positions become one-slice hot
// items, run by a whole workgroup in one round of grad loads instead of two rounds by one lane
// group.  kMinChunk bounds the slice counts the allocations are sized for.
constexpr int kMinChunk = 16;
constexpr int kRankBucketMax = 64;  // within-bucket rank sort when every bucket is this small
enum { CNT_U = 0, CNT_C = 1, CNT_H = 2, CNT_S = 3, CNT_NV = 4, CNT_OFF = kCntOff };
// Hot segments are cut into slices of kHotSlice positions, one work item (one 256-thread apply
// workgroup: 8 lane groups x 16 rows in flight at D = 128, two rounds) each, so a hot row's grad rows are read
// by several CUs at once; a segment of several slices is combined by its last-arriving slice (sc1
// partial rows + a counter; apply.hpp).
// 256 (round 3; was 128): fewer multi-slice segments to combine across workgroups.  A/B on one box
// (tools/r6v_check.sh): bf16 B=8192 apply 22.4 -> 20.4 us (78.6 -> 80.2 M samples/s), D=16 +0.6 %,
// pooled +0.4 %, the metric unchanged; 64 was slower everywhere.
#ifndef DLRM_HOT_SLICE
#define DLRM_HOT_SLICE 256
#endif
constexpr int kHotSlice = DLRM_HOT_SLICE;
// A chunk's descriptor is two int4: {beg, end, row, pos0}, {pos1, pos2, pos3, pos4}: its first
// kChunkInline positions (ascending; -1 past the end) travel with it, so the apply reads perm
// only for longer chunks.  A hot slice's descriptor is one int4 {p0, p1, row, hot segment}.
constexpr int kChunkInline = 5;

__device__ __forceinline__ void write_chunk(int4* chunks, int64_t c, int beg, int end, int row,
                                            const int32_t* sorted_pos /* [beg, end) or NULL */) {
    int q[kChunkInline];
#pragma unroll
    for (int k = 0; k < kChunkInline; ++k) q[k] = (sorted_pos && beg + k < end) ? sorted_pos[beg + k] : -1;
    chunks[2 * c] = make_int4(beg, end, row, q[0]);
    chunks[2 * c + 1] = make_int4(q[1], q[2], q[3], q[4]);
}

// write_chunk with the descriptor's perm entries given apart from where its positions are read
// (pos: the chunk's sorted positions, pos[0] its first)
__device__ __forceinline__ void write_chunk_rec(int4* chunks, int64_t c, int beg, int end, int row, const int32_t* pos) {
    int q[kChunkInline];
#pragma unroll
    for (int k = 0; k < kChunkInline; ++k) q[k] = beg + k < end ? pos[k] : -1;
    chunks[2 * c] = make_int4(beg, end, row, q[0]);
    chunks[2 * c + 1] = make_int4(q[1], q[2], q[3], q[4]);
}

__device__ __forceinline__ void write_slices(int4* hot_slice, int s0, int beg, int end, int row, int h) {
    for (int k = 0, p0 = beg; p0 < end; ++k, p0 += kHotSlice)
        hot_slice[s0 + k] = make_int4(p0, min(p0 + kHotSlice, end), row, h);
}

// Exclusive scan over the NW waves' 64*NW threads; returns this thread's prefix, total in *tot.
template <int NW, typename V>
__device__ __forceinline__ V block_scan_nw(V v, V* wtot, V* tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    V x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const V y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) wtot[w] = x;
    __syncthreads();
    if (w == 0) {
        V t = lane < NW ? wtot[lane] : V(0);
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const V y = __shfl_up(t, off, 64);
            if (lane >= off) t += y;
        }
        if (lane < NW) wtot[NW + lane] = t;  // inclusive wave totals
    }
    __syncthreads();
    const V before = w ? wtot[NW + w - 1] : V(0);
    *tot = wtot[2 * NW - 1];
    __syncthreads();  // wtot reusable after return
    return before + x - v;
}

// ------------------------------------------------------------------- fast indexer (N <= 4096)
// One 1024-thread workgroup per table; everything stays in LDS.
//  * Stable counting pass on an 8-bit digit: wave w walks positions [w*S, (w+1)*S) (S = 64*EPL)
//    in tiles of 64, so "earlier position" = earlier wave, earlier tile or lower lane.  Lanes
//    sharing a digit are found with 8 ballots; each wave keeps its running count of every
//    digit in its own column of cnt[digit][wave] (only that wave touches it, in program
//    order), which gives each key its rank among the wave's earlier equal digits.  One block
//    scan over cnt in (digit, wave) order turns the counts into output offsets: no serial
//    cross-wave loop.  Invalid indices are dropped (they raised the bounds flag).
//  * Rows of <= 8 bits are then grouped.  Larger rows: when every bucket is small (uniform
//    rows: N/256 keys per bucket) each bucket is ordered by a direct rank on (row, position);
//    skewed rows take the remaining LSD passes.
//  * Segments and the chunk / hot lists: one head-flag scan and one packed 64-bit scan.
// Output format = indexer_build_kernel's (the apply kernel and dlrm_indexer_read unchanged).

// NT threads (1024 standalone; 256 inside the backward launch), EPL positions per thread.
// Digit width: 8 bits with 16 waves, 11 bits with 4 (about one key per bucket at N = 2048, so
// the within-bucket rank is short where one wave per SIMD hides no latency).
template <int NT, int EPL, int DB_ = (NT >= 1024 ? 8 : 11)>
struct FastLds {
    static constexpr int NW = NT / 64;
    static constexpr int DB = DB_;                  // digit bits
    static constexpr int ND = 1 << DB;              // digits
    static constexpr int CPT = ND * NW / NT;        // (digit, wave) counters per thread: 4 or 32
    static_assert(CPT == 4 || CPT % 8 == 0, "counters per thread: 4, or whole uint4s");
    uint16_t cnt[ND][NW];       // digit-major: per-wave counts, then output offsets
    uint16_t bstart[ND + 8];    // first-pass bucket starts
    uint32_t K[2][NT * EPL];
    int32_t V[2][NT * EPL];
    int wtot[2 * NW];
    long long wtot64[2 * NW];
    int maxbucket;
};

// One stable counting pass.  FROM_REGS: the first pass's keys come from registers (tile j
// of wave w = position w*S + 64j + lane, S = 64*EPL); otherwise from kin/vin[0, n) in LDS,
// wave w taking [w*S, (w+1)*S) for the caller's S (a multiple of 64, S*NW >= n).  Returns the
// number of keys written to kout/vout.
template <int NT, int EPL, bool FROM_REGS, int DB>
__device__ int fast_pass(int n, int shift, const uint32_t (&rkey)[EPL], const bool (&rok)[EPL],
                         const uint32_t* kin, const int32_t* vin, uint32_t* kout, int32_t* vout,
                         FastLds<NT, EPL, DB>& sl, bool first, int S = 64 * EPL) {
    typedef FastLds<NT, EPL, DB> FL;
    constexpr int CPT = FL::CPT, NW = FL::NW;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    if (CPT == 4) {
        ((uint2*)&sl.cnt[0][0])[tid] = make_uint2(0, 0);
    } else {
#pragma unroll
        for (int k = 0; k < CPT / 8; ++k) ((uint4*)&sl.cnt[0][0])[tid * (CPT / 8) + k] = make_uint4(0, 0, 0, 0);
    }
    uint32_t key[EPL];
    int32_t val[EPL];
    bool ok[EPL];
    int lr[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        const int i = w * S + j * 64 + lane;
        if (FROM_REGS) {
            key[j] = rkey[j];
            ok[j] = rok[j];
            val[j] = i;
        } else {
            ok[j] = j * 64 < S && i < n;
            key[j] = ok[j] ? kin[i] : 0u;
            val[j] = ok[j] ? vin[i] : 0;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        if (j * 64 >= S) break;  // uniform
        const uint32_t d = (key[j] >> shift) & (FL::ND - 1);
        unsigned long long peers = __ballot(ok[j]);
#pragma unroll
        for (int bit = 0; bit < FL::DB; ++bit) {
            const unsigned long long bb = __ballot(ok[j] && ((d >> bit) & 1u));
            peers &= ((d >> bit) & 1u) ? bb : ~bb;
        }
        int base = 0;
        if (ok[j] && j > 0) base = sl.cnt[d][w];
        lr[j] = base + __popcll(peers & lt);
        if (ok[j] && (peers & lt) == 0) sl.cnt[d][w] = (uint16_t)(base + __popcll(peers));
    }
    __syncthreads();
    if (first) PHASE(2);
    // (digit, wave) offsets: thread tid owns the CPT counters [CPT tid, CPT tid + CPT) of cnt
    // in (digit, wave) order; one block scan over the per-thread sums
    uint32_t cw[CPT / 2];  // CPT uint16 counters, two per word
    if (CPT == 4) {
        const uint2 r = ((const uint2*)&sl.cnt[0][0])[tid];
        cw[0] = r.x;
        cw[1] = r.y;
    } else {
#pragma unroll
        for (int k = 0; k < CPT / 8; ++k) {
            const uint4 r = ((const uint4*)&sl.cnt[0][0])[tid * (CPT / 8) + k];
            cw[4 * k] = r.x; cw[4 * k + 1] = r.y; cw[4 * k + 2] = r.z; cw[4 * k + 3] = r.w;
        }
    }
    int sum = 0;
#pragma unroll
    for (int k = 0; k < CPT / 2; ++k) sum += (int)(cw[k] & 0xffffu) + (int)(cw[k] >> 16);
    int total;
    const int ex = block_scan_nw<NW, int>(sum, sl.wtot, &total);
    {
        int run = ex;
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
            const int e = CPT * tid + k;  // counter e = (digit e / NW, wave e % NW)
            const int c = (int)((cw[k >> 1] >> (16 * (k & 1))) & 0xffffu);
            if (first && e % NW == 0) sl.bstart[e / NW] = (uint16_t)run;
            if (k & 1) cw[k >> 1] = (cw[k >> 1] & 0xffffu) | ((uint32_t)run << 16);
            else cw[k >> 1] = (cw[k >> 1] & 0xffff0000u) | (uint32_t)run;
            run += c;
        }
    }
    if (CPT == 4) {
        ((uint2*)&sl.cnt[0][0])[tid] = make_uint2(cw[0], cw[1]);
    } else {
#pragma unroll
        for (int k = 0; k < CPT / 8; ++k)
            ((uint4*)&sl.cnt[0][0])[tid * (CPT / 8) + k] = make_uint4(cw[4 * k], cw[4 * k + 1], cw[4 * k + 2], cw[4 * k + 3]);
    }
    if (first && tid == 0) {
        sl.bstart[FL::ND] = (uint16_t)total;
        sl.maxbucket = 0;
    }
    __syncthreads();
    if (first) PHASE(3);
    if (first) {
        // largest bucket (decides rank sort vs more passes)
        int m = 0;
        for (int dd = tid; dd < FL::ND; dd += NT) m = max(m, (int)sl.bstart[dd + 1] - (int)sl.bstart[dd]);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
        if (lane == 0 && m > 0) atomicMax(&sl.maxbucket, m);
        PHASE(4);
    }
#pragma unroll
    for (int j = 0; j < EPL; ++j)
        if (ok[j]) {
            const uint32_t d = (key[j] >> shift) & (FL::ND - 1);
            const int dst = sl.cnt[d][w] + lr[j];
            kout[dst] = key[j];
            vout[dst] = val[j];
        }
    __syncthreads();
    return total;
}

// SPLIT (the training step's build, run before a backward that updates once-hit rows itself):
// segments of one position get no chunk, and single[p] = 1 marks each such position p.
// vs = 0: every position of table t, results under index v = t.  vs = 1 / 2: only the
// positions whose row has low bits == v mod 2^vs (virtual table v = (t << vs) + part,
// IndexerDev::vshift = vs): they are compacted in position order, sorted on row >> vs, and
// the rows written back whole.  2^vs workgroups then share a table's positions.
template <int NT, int EPL, bool SPLIT = false, int DB>
__device__ void fast_index_table(const IndexerDev& ix, int v, int t, int vs, uint32_t nrows,
                                 const void* __restrict__ idx, int itype, int64_t tstride, int base, int N,
                                 unsigned* __restrict__ err, FastLds<NT, EPL, DB>& sl) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int S = 64 * EPL;
    PHASE(0);
    const uint32_t part = (uint32_t)v & ((1u << vs) - 1u);
    const uint32_t kmax = nrows > 0 ? (nrows - 1) >> vs : 0u;
    const int nbits = 32 - __clz(kmax);
    // the indices, read once (coalesced 64-lane runs, all loads in flight) and validated
    uint32_t key[EPL];
    bool ok[EPL];
    int64_t raw[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        const int i = w * S + j * 64 + lane;
        raw[j] = load_index(idx, itype, t * tstride + min(i, N - 1));
    }
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        const int i = w * S + j * 64 + lane;
        const int64_t r = raw[j] - base;
        ok[j] = i < N && r >= 0 && r < (int64_t)nrows;
        key[j] = ok[j] ? (uint32_t)r : 0u;
        if (i < N && !ok[j] && part == 0) raise_index_error(err);
    }
    PHASE(1);
    int n, SW = S;  // keys; positions per wave in the counting passes
    if (vs == 0) {
        n = fast_pass<NT, EPL, true>(N, 0, key, ok, nullptr, nullptr, sl.K[1], sl.V[1], sl, true);
    } else {
        // stable compaction of this half's positions (position order = wave, tile, lane order)
        const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
        int run = 0, lr[EPL];
        bool keep[EPL];
#pragma unroll
        for (int j = 0; j < EPL; ++j) {
            keep[j] = ok[j] && (key[j] & ((1u << vs) - 1u)) == part;
            const unsigned long long b = __ballot(keep[j]);
            lr[j] = run + __popcll(b & lt);
            run += __popcll(b);
        }
        if (lane == 0) sl.wtot[w] = run;
        __syncthreads();
        int wb = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < NT / 64; ++k) {
            const int c = sl.wtot[k];
            wb += k < w ? c : 0;
            tot += c;
        }
#pragma unroll
        for (int j = 0; j < EPL; ++j)
            if (keep[j]) {
                sl.K[0][wb + lr[j]] = key[j] >> vs;
                sl.V[0][wb + lr[j]] = w * S + j * 64 + lane;
            }
        __syncthreads();
        SW = 64 * ((tot + NT - 1) / NT);
        n = fast_pass<NT, EPL, false>(tot, 0, key, ok, sl.K[0], sl.V[0], sl.K[1], sl.V[1], sl, true, SW);
    }
    PHASE(5);
    int cur = 1;
    typedef FastLds<NT, EPL, DB> FL;
    if (nbits > FL::DB) {
        if (sl.maxbucket <= kRankBucketMax) {
            // order each bucket by (row, position); the stable pass kept positions ascending
            if (FL::DB >= 11) {
                // ~1 key per bucket: issue every key's loads together (EPL in flight) rather
                // than one dependent chain per key
                uint32_t ki[EPL];
                int bs[EPL], len[EPL], rank[EPL];
                int maxlen = 0;
#pragma unroll
                for (int q = 0; q < EPL; ++q) {
                    const int i = tid + q * NT;
                    ki[q] = (q * NT < n && i < n) ? sl.K[1][i] : 0u;
                }
#pragma unroll
                for (int q = 0; q < EPL; ++q) {
                    const int i = tid + q * NT;
                    const int d = ki[q] & (FL::ND - 1);
                    bs[q] = i < n ? (int)sl.bstart[d] : 0;
                    len[q] = i < n ? (int)sl.bstart[d + 1] - bs[q] : 0;
                    rank[q] = 0;
                    maxlen = max(maxlen, len[q]);
                }
                for (int j = 0; j < maxlen; ++j) {
#pragma unroll
                    for (int q = 0; q < EPL; ++q)
                        if (q * NT < n && j < len[q]) {
                            const uint32_t kj = sl.K[1][bs[q] + j];
                            rank[q] += (kj < ki[q] || (kj == ki[q] && bs[q] + j < (int)(tid + q * NT))) ? 1 : 0;
                        }
                }
#pragma unroll
                for (int q = 0; q < EPL; ++q) {
                    const int i = tid + q * NT;
                    if (i < n) {
                        sl.K[0][bs[q] + rank[q]] = ki[q];
                        sl.V[0][bs[q] + rank[q]] = sl.V[1][i];
                    }
                }
            } else {
#pragma unroll
                for (int q = 0; q < EPL; ++q) {
                    const int i = tid + q * NT;
                    if (i >= n) continue;
                    const uint32_t ki = sl.K[1][i];
                    const int d = ki & (FL::ND - 1);
                    const int bs = sl.bstart[d], be = sl.bstart[d + 1];
                    int rank = 0;
                    int j = bs;
                    for (; j + 4 <= be; j += 4) {
                        const uint32_t k0 = sl.K[1][j], k1 = sl.K[1][j + 1], k2 = sl.K[1][j + 2], k3 = sl.K[1][j + 3];
                        rank += (k0 < ki || (k0 == ki && j < i)) + (k1 < ki || (k1 == ki && j + 1 < i)) +
                                (k2 < ki || (k2 == ki && j + 2 < i)) + (k3 < ki || (k3 == ki && j + 3 < i));
                    }
                    for (; j < be; ++j) {
                        const uint32_t kj = sl.K[1][j];
                        rank += (kj < ki || (kj == ki && j < i)) ? 1 : 0;
                    }
                    sl.K[0][bs + rank] = ki;
                    sl.V[0][bs + rank] = sl.V[1][i];
                }
            }
            __syncthreads();
            cur = 0;
        } else {
            for (int shift = FL::DB; shift < nbits; shift += FL::DB) {
                fast_pass<NT, EPL, false>(n, shift, key, ok, sl.K[cur], sl.V[cur], sl.K[cur ^ 1], sl.V[cur ^ 1], sl,
                                          false, SW);
                cur ^= 1;
            }
        }
    }
    PHASE(10);
    // ---- segments: thread tid owns sorted entries [E*tid, E*tid + E)
    const int E = (n + NT - 1) / NT;  // <= EPL
    const uint32_t* K = sl.K[cur];
    const int32_t* Vs = sl.V[cur];
    int32_t* sseg = sl.V[cur ^ 1];
    uint32_t* srow = sl.K[cur ^ 1];
    const int64_t off = (int64_t)v * ix.cap;
    int32_t* perm = ix.perm + off;
    int32_t* seg_start = ix.seg_start + (int64_t)v * (ix.cap + 1);
    uint32_t* seg_row = ix.seg_row + off;
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const int i = tid + q * NT;
        if (i < n) perm[i] = Vs[i];
    }
    int h = 0;
    bool head[EPL];
    uint32_t kq[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const int i = E * tid + q;
        const bool in = q < E && i < n;
        kq[q] = in ? K[i] : 0u;
        const uint32_t kp = (in && i > 0) ? K[i - 1] : ~kq[q];
        head[q] = in && kp != kq[q];
        h += head[q] ? 1 : 0;
    }
    int U;
    int s = block_scan_nw<NT / 64, int>(h, sl.wtot, &U);
#pragma unroll
    for (int q = 0; q < EPL; ++q)
        if (head[q]) {
            const int i = E * tid + q;
            const uint32_t row = (kq[q] << vs) | part;
            sseg[s] = i;
            srow[s] = row;
            seg_start[s] = i;
            seg_row[s] = row;
            ++s;
        }
    if (tid == 0) seg_start[U] = n;
    if (SPLIT) {  // once-hit positions: head of a segment whose next entry starts another
        uint8_t* single = ix.single + (int64_t)t * ix.cap;
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const int i = E * tid + q;
            if (q < E && i < n) single[Vs[i]] = (head[q] && (i + 1 == n || K[i + 1] != kq[q])) ? 1 : 0;
        }
    }
    __syncthreads();
    PHASE(20);
    // packed counts (N <= 4096 < 2^21): chunks bits 0-20, hot segments 21-41, hot slices 42-62
    constexpr long long M21 = (1ll << 21) - 1;
    long long cw = 0;
    int beg[EPL], end[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const int sidx = E * tid + q;
        beg[q] = end[q] = 0;
        if (q < E && sidx < U) {
            beg[q] = sseg[sidx];
            end[q] = sidx + 1 < U ? sseg[sidx + 1] : n;
            const int len = end[q] - beg[q];
            if (!(SPLIT && len == 1))
                cw += len <= kChunk ? 1ll : ((1ll << 21) | ((long long)((len + kHotSlice - 1) / kHotSlice) << 42));
        }
    }
    long long tot64;
    const long long ex = block_scan_nw<NT / 64, long long>(cw, sl.wtot64, &tot64);
    int c = (int)(ex & M21), hh = (int)((ex >> 21) & M21), ss = (int)((ex >> 42) & M21);
    int4* chunks = ix.chunks + 2 * off;
    int4* hot = ix.hot + off;
    int4* hot_slice = ix.hot_slice + off;
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const int sidx = E * tid + q;
        if (q < E && sidx < U) {
            const int len = end[q] - beg[q];
            if (SPLIT && len == 1) {
                // updated by the backward (single[] flag)
            } else if (len <= kChunk) {
                write_chunk(chunks, c++, beg[q], end[q], (int)srow[sidx], Vs);
            } else {
                const int ns = (len + kHotSlice - 1) / kHotSlice;
                hot[hh] = make_int4(beg[q], end[q], (int)srow[sidx], ss);
                write_slices(hot_slice, ss, beg[q], end[q], (int)srow[sidx], hh);
                ++hh;
                ss += ns;
            }
        }
    }
    if (tid == 0) {
        int32_t* cnt = ix.counts + (int64_t)v * 8;
        cnt[CNT_U] = U; cnt[CNT_C] = (int)(tot64 & M21); cnt[CNT_H] = (int)((tot64 >> 21) & M21);
        cnt[CNT_S] = (int)((tot64 >> 42) & M21); cnt[CNT_NV] = n;
    }
    PHASE(22);
}

// The training step's split build, as extra 256-thread workgroups of another launch (the step
// forward's, interact.hip; or the previous step's apply, update.hip): one per virtual table.
constexpr int kStepIndexEPL = kStepIndexMaxN / 256;  // positions per thread
#ifndef DLRM_STEP_DB
#define DLRM_STEP_DB 8
#endif
// 8-bit digits: a table part holds about N >> vshift positions, and the digit scan (NW << DB
// counters) is a fixed cost of every counting pass
typedef FastLds<256, kStepIndexEPL, DLRM_STEP_DB> StepLds;

// ------------------------------------------------- flat (table, item) lookup over counts
// Inclusive scan over the 64 lanes by DPP: Hillis-Steele inside each 16-lane row (row_shr 1, 2,
// 4, 8), then the row totals (row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3).
// Six VALU ops with no LDS permute (a __shfl_up chain is six dependent ds_bpermute round trips).
__device__ __forceinline__ int wave_incl_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// The same scan with max (values >= 0): lane 63 holds the wave's maximum.
__device__ __forceinline__ int wave_incl_max(int x) {
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false));
    return x;
}

__device__ __forceinline__ int lane63(int x) { return __builtin_amdgcn_readlane(x, 63); }

// Flat id -> (table, offset) over per-table counts, T tables in tiles of 64 lanes.  Every lane
// may carry its own id; shuffles run in uniform control flow.  table = -1 when id >= total.
__device__ __forceinline__ void locate_in_tile(int incl, int tile_total, int tb, int key, int& table, int& local) {
    // count of lanes with incl <= key (binary lifting over the non-decreasing prefix)
    int pos = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1) {
        const int vv = __shfl(incl, pos + step - 1, 64);
        if (vv <= key) pos += step;
    }
    const int before = __shfl(incl, pos > 0 ? pos - 1 : 0, 64);
    if (table < 0 && key >= 0 && key < tile_total) {
        table = tb + pos;
        local = key - (pos > 0 ? before : 0);
    }
}

// Per-wave prefix of one count over the tables.  T <= 64 * kScanTiles: lane l holds the counts
// of the G = ceil(T / 64) consecutive tables [l*G, l*G + G) and the inclusive prefix of their
// sums, so a lookup is one binary lifting over the lanes plus G independent shuffles.  More
// tables are re-scanned tile by tile on every lookup.
constexpr int kScanTiles = 2;  // (T <= 128 virtual tables; the wave build's 16-part tables use the item map)
struct TableScan {
    int cnt[kScanTiles];  // counts of this lane's tables
    int incl;             // inclusive prefix over the lanes' groups
    int total;            // over all tables
    int G;                // tables per lane (0: T > 64 * kScanTiles)
};

__device__ __forceinline__ TableScan scan_counts(const IndexerDev& ix, int T_, int which) {
    const int lane = threadIdx.x & 63;
    TableScan r{};
    if (T_ <= 64 * kScanTiles) {
        r.G = (T_ + 63) / 64;
        int sum = 0;
#pragma unroll
        for (int q = 0; q < kScanTiles; ++q) {  // every load in flight
            const int v = lane * r.G + q;
            r.cnt[q] = (q < r.G && v < T_) ? ix.counts[(int64_t)v * 8 + which] : 0;
            sum += r.cnt[q];
        }
        r.incl = wave_incl_scan(sum);
        r.total = lane63(r.incl);
        return r;
    }
    for (int tb = 0; tb < T_; tb += 64) {
        const int tt = tb + lane;
        const int c = tt < T_ ? ix.counts[(int64_t)tt * 8 + which] : 0;
        r.total += __shfl(wave_incl_scan(c), 63, 64);
    }
    return r;
}

__device__ __forceinline__ void locate(const IndexerDev& ix, int T_, int which, const TableScan& sc, int id,
                                       int& table, int& local) {
    table = -1;
    local = 0;
    if (sc.G == 1) {
        locate_in_tile(sc.incl, sc.total, 0, id, table, local);
        return;
    }
    if (sc.G > 1) {
        int grp = -1, loc = 0;
        locate_in_tile(sc.incl, sc.total, 0, id, grp, loc);
        const int src = grp < 0 ? 0 : grp;
        int run = 0;
#pragma unroll
        for (int q = 0; q < kScanTiles; ++q) {
            const int c = __shfl(sc.cnt[q], src, 64);
            if (grp >= 0 && table < 0 && q < sc.G && loc < run + c) {
                table = src * sc.G + q;
                local = loc - run;
            }
            run += c;
        }
        return;
    }
    const int lane = threadIdx.x & 63;
    int run = 0;
    for (int tb = 0; tb < T_; tb += 64) {
        const int tt = tb + lane;
        const int c = tt < T_ ? ix.counts[(int64_t)tt * 8 + which] : 0;
        const int incl = wave_incl_scan(c);
        const int tot = __shfl(incl, 63, 64);
        locate_in_tile(incl, tot, tb, id - run, table, local);
        run += tot;
    }
}


// ------------------------------------------------------------- wave build (round 4)
// The training step's split build of the NEXT batch, one WAVE per virtual table (t, part).  The
// 256-thread block build (fast_index_table) took ~12 us per part inside the apply launch: ~15
// dependent barrier + LDS phases with one wave per SIMD, the same alone, beside the apply, or
// run twice on a warm instruction cache (tools/phase_step.py).  Here a workgroup of 4 waves
// splits one table's positions among 4 parts together (each wave reads a quarter of them once),
// then each wave sorts its part (~N/16 keys at 16 parts per table) with wave-level steps: DPP
// scans, ballots, one LDS atomic per digit group, and no workgroup barrier.
// Output format = fast_index_table's (split): the apply, dlrm_indexer_read and the step backward
// read it unchanged.  Within a part, segments come in ascending row order, positions ascending.
constexpr int kWaveParts = 4;       // waves per build workgroup = parts of one table per workgroup
#ifndef DLRM_WAVE_RANK_MAX
#define DLRM_WAVE_RANK_MAX 16
#endif
// within-bucket rank when every low-digit bucket is this small (256: Terabyte Zipf rows 17.3 ->
// 33.4 us apply, each hot-bucket lane walks the whole bucket)
constexpr int kWaveRankMax = DLRM_WAVE_RANK_MAX;
constexpr int kWideDigit = 9;       // wide keys' first digit: 512 buckets for ~150 keys of a part
struct WaveBuildLds {
    // (each part's region starts 16-B aligned: up to 3 entries of padding after each of 4 parts)
    uint32_t K[2][kStepIndexMaxN + 16];  // keys (row >> vshift), sort ping-pong; the 4 parts' regions
    int32_t V[2][kStepIndexMaxN + 16];   // positions
    int32_t R[kStepIndexMaxN + 16];      // per-key rank in its digit, then segment starts
    uint32_t cnt[kWaveParts][1 << kWideDigit];  // per-wave digit counters, then digit offsets
    // [round][wave][part]: positions of the workgroup's part q that wave w read in round r (a round
    // = 2048 positions, 512 per wave)
    int tot[kWaveMaxN / kStepIndexMaxN][kWaveParts][kWaveParts];
    // per wave: the table's positions it read that fall in parts below the workgroup's (q < q0),
    // whose sum places the workgroup's parts in the table's compact region (common.hpp kSegPad)
    int below[16];
};
// the scan build's per-wave counts of its four parts (<= 16 waves), in the rounds form's tot array
__device__ __forceinline__ int4* scan_wave_totals(WaveBuildLds& sl) { return (int4*)&sl.tot[0][0][0]; }
static_assert(sizeof(WaveBuildLds::tot) >= 16 * sizeof(int4), "tot holds the scan build's wave totals");

// The flat item lists come in kResLists sub-lists: build workgroup g reserves in sub-list g mod 8
// (its XCD's), so each reservation word takes an eighth of the build's atomics (one word took ~2.7
// us to return with all 416 waves on it).  Word j (build_arrive, 64 bits, one per 256 B): chunks in
// bits 0..23, hot slices in 24..43, arrived waves in 44..63 (the wave build: <= 31 x 2048
// positions).  Sub-list j's records start at j * res_stride (a workgroup's positions, <= cap, give
// at most cap / 2 chunks and as many slices); item_tot[j] / [kResLists + j] = its slices / chunks.
constexpr int kResSliceShift = 24, kResArriveShift = 44;
constexpr int kResLists = 8, kResWordStride = 32;  // (u64 words: 256 B apart)
// (a sub-list's records also number at most half its positions: <= T0 cap / 2, T0 = the real
// tables, which bounds it once the parts outnumber 32 per table)
__host__ __device__ __forceinline__ int res_stride(int groups, int64_t cap, int vs) {
    const int64_t per_group = ((groups + kResLists - 1) / kResLists) * (cap / 2 + 8);
    const int64_t per_table = (int64_t)((groups * kWaveParts) >> vs) * (cap / 2 + 8);
    return (int)(per_group < per_table ? per_group : per_table);
}
// flat record index of item k of the sub-lists with counts cnt[0..kResLists), or -1 past the end
__device__ __forceinline__ int res_locate(const int* cnt, int k, int stride) {
    int run = 0, at = -1;
#pragma unroll
    for (int j = 0; j < kResLists; ++j) {
        if (at < 0 && k < run + cnt[j]) at = j * stride + (k - run);
        run += cnt[j];
    }
    return at;
}

__device__ __forceinline__ unsigned long long lanes_below() {
    const int lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Lanes (among `ok` ones) whose `bits`-bit digit (bits <= 8, uniform) equals this lane's.
__device__ __forceinline__ unsigned long long match_digit(uint32_t d, bool ok, int bits) {
    unsigned long long peers = __ballot(ok);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
        if (bit >= bits) break;  // uniform
        const unsigned long long bb = __ballot(ok && ((d >> bit) & 1u));
        peers &= ((d >> bit) & 1u) ? bb : ~bb;
    }
    return peers;
}

// The sort's in-wave barrier: LDS parts (the pool) need the wave's LDS operations ordered; a part
// sorted in HBM (G: the wave build's overflow path) needs its global stores visible to the other
// lanes of the wave before they read them (workgroup-scope release / acquire).
template <bool G>
__device__ __forceinline__ void part_sync() {
    if constexpr (G) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else {
        wave_lds_sync();
    }
}

// One stable counting pass of one wave over keys [0, n) of (Kin, Vin), on the `bits`-bit digit
// at `shift`, into (Kout, Vout).  Tiles of 64 keys in order; in a tile, the lanes sharing a digit
// are found by ballots and the group's first lane adds the group's size to the digit's counter
// with one LDS atomic, whose old value is the group's base (a wave's LDS operations complete in
// order, so the bases follow the tiles).  Leaves cnt[d] = the start of digit d's bucket; returns
// the largest bucket.
template <bool G>
__device__ int wave_count_pass(int n, int shift, int bits, const uint32_t* Kin, const int32_t* Vin, uint32_t* Kout,
                               int32_t* Vout, int32_t* R, uint32_t* cnt) {
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = lanes_below();
    const uint32_t dm = (1u << bits) - 1u;
    *(uint4*)&cnt[4 * lane] = make_uint4(0u, 0u, 0u, 0u);
    wave_lds_sync();  // (cnt: LDS)
    for (int j0 = 0; j0 < n; j0 += 64) {
        const int i = j0 + lane;
        const bool ok = i < n;
        const uint32_t d = ok ? (Kin[i] >> shift) & dm : 0u;
        const unsigned long long peers = match_digit(d, ok, bits);
        const int rank = __popcll(peers & lt);
        uint32_t old = 0;
        if (ok && rank == 0) old = atomicAdd(&cnt[d], (uint32_t)__popcll(peers));
        const int leader = ok ? __ffsll((long long)peers) - 1 : lane;
        const uint32_t b = (uint32_t)__shfl((int)old, leader, 64);
        if (ok) R[i] = (int)b + rank;
    }
    part_sync<G>();
    const uint4 c = *(const uint4*)&cnt[4 * lane];  // lane l: digits 4l .. 4l+3
    const int sum = (int)(c.x + c.y + c.z + c.w);
    int o = wave_incl_scan(sum) - sum;
    uint4 st;
    st.x = o; o += c.x;
    st.y = o; o += c.y;
    st.z = o; o += c.z;
    st.w = o;
    *(uint4*)&cnt[4 * lane] = st;
    const int m = lane63(wave_incl_max((int)max(max(c.x, c.y), max(c.z, c.w))));
    wave_lds_sync();  // (cnt: LDS)
    for (int j0 = 0; j0 < n; j0 += 64) {
        const int i = j0 + lane;
        if (i < n) {
            const uint32_t k = Kin[i];
            const int dst = (int)cnt[(k >> shift) & dm] + R[i];
            Kout[dst] = k;
            Vout[dst] = Vin[i];
        }
    }
    part_sync<G>();
    return m;
}

// The first pass of a wide-key part, unstable: one LDS atomic per key on the counter of its low
// kWideDigit bits (a bucket's keys land in any order; wave_rank_buckets orders them by (key,
// position)).  Leaves cnt[d] = the start of digit d's bucket; returns the largest bucket (and places
// nothing when it exceeds kWaveRankMax).
template <bool G>
__device__ int wave_count_pass_unstable(int n, const uint32_t* Kin, const int32_t* Vin, uint32_t* Kout,
                                        int32_t* Vout, int32_t* R, uint32_t* cnt) {
    constexpr uint32_t dm = (1u << kWideDigit) - 1u;
    constexpr int PL = (1 << kWideDigit) / 64;  // counters per lane
    static_assert(PL % 4 == 0, "whole uint4 per lane");
    const int lane = threadIdx.x & 63;
    uint4* c4 = (uint4*)&cnt[PL * lane];
#pragma unroll
    for (int q = 0; q < PL / 4; ++q) c4[q] = make_uint4(0u, 0u, 0u, 0u);
    wave_lds_sync();
    for (int i = lane; i < n; i += 64) R[i] = (int)atomicAdd(&cnt[Kin[i] & dm], 1u);
    part_sync<G>();
    uint32_t c[PL];
#pragma unroll
    for (int q = 0; q < PL / 4; ++q) {
        const uint4 x = c4[q];
        c[4 * q] = x.x; c[4 * q + 1] = x.y; c[4 * q + 2] = x.z; c[4 * q + 3] = x.w;
    }
    int sum = 0, mx = 0;
#pragma unroll
    for (int q = 0; q < PL; ++q) {
        sum += (int)c[q];
        mx = max(mx, (int)c[q]);
    }
    int o = wave_incl_scan(sum) - sum;
#pragma unroll
    for (int q = 0; q < PL / 4; ++q) {
        uint4 st;
        st.x = o; o += c[4 * q];
        st.y = o; o += c[4 * q + 1];
        st.z = o; o += c[4 * q + 2];
        st.w = o; o += c[4 * q + 3];
        c4[q] = st;
    }
    const int m = lane63(wave_incl_max(mx));
    wave_lds_sync();
    if (m > kWaveRankMax) return m;  // (skewed: the caller re-sorts (Kin, Vin) by stable passes)
    for (int i = lane; i < n; i += 64) {
        const uint32_t k = Kin[i];
        const int dst = (int)cnt[k & dm] + R[i];
        Kout[dst] = k;
        Vout[dst] = Vin[i];
    }
    part_sync<G>();
    return m;
}

// Every low-digit bucket small (uniform rows): each key's place in its bucket by a direct rank on
// (key, position) (positions are distinct, so the order is total and the sort stable).
template <bool G>
__device__ void wave_rank_buckets(int n, const uint32_t* K1, const int32_t* V1, uint32_t* K0, int32_t* V0,
                                  const uint32_t* start) {
    constexpr int dm = (1 << kWideDigit) - 1;
    for (int i = threadIdx.x & 63; i < n; i += 64) {
        const uint32_t ki = K1[i];
        const int d = (int)(ki & (uint32_t)dm);
        const int bs = (int)start[d], be = d < dm ? (int)start[d + 1] : n;
        const int32_t vi = V1[i];
        // four bucket entries per 16-B read pair (the part's region is 16-B aligned), so a skewed
        // bucket (a hot row: ~100+ keys) costs a quarter of the read latencies
        int rank = 0;
        for (int j0 = bs & ~3; j0 < be; j0 += 4) {
            const uint4 kq = *(const uint4*)(K1 + j0);
            const int4 vq = *(const int4*)(V1 + j0);
            const uint32_t kj[4] = {kq.x, kq.y, kq.z, kq.w};
            const int32_t vj[4] = {vq.x, vq.y, vq.z, vq.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int j = j0 + e;
                rank += (j >= bs && j < be && (kj[e] < ki || (kj[e] == ki && vj[e] < vi))) ? 1 : 0;
            }
        }
        K0[bs + rank] = ki;
        V0[bs + rank] = vi;
    }
    part_sync<G>();
}

// One lane's segment of a tile of the sorted part, as its flat record: kind 1 = a chunk (a =
// {first perm entry, end (global), row, pos0}, b = {pos1 .. pos4}; idx = the wave's chunk
// number), 2 = a hot segment (a = {beg, end (local), row}; idx = the wave's first slice, ns slices).
struct SegRec {
    int4 a, b;
    int kind, idx, ns;
};

struct SegPass {
    const IndexerDev& ix;
    int v, vs;
    uint32_t part;
    int n, U;
    const uint32_t* Ks;
    const int32_t* Vs;
    const int32_t* R;
    int64_t off;   // the part's per-part entries (compact: t * cap + its offset in the table)
    int64_t soff;  // its segment starts
    int kb = 0;          // > 0: segment 0 is a hot-row prefix of kb positions (key hkey, not in Ks / Vs,
    uint32_t hkey = 0;   // which hold the part's entries from kb on: entry i at Ks[i - kb])

    // segments [s0, s0 + 64): the per-part lists (seg_start, seg_row, chunks, hot, hot_slice) when
    // `lists`, and this lane's flat record; c / h / sl0 run over the tiles
    __device__ __forceinline__ SegRec tile(int s0, int& c, int& h, int& sl0, bool lists) const {
        const int lane = threadIdx.x & 63;
        const unsigned long long lt = lanes_below();
        const int s = s0 + lane;
        const bool ok = s < U;
        const int beg = ok ? R[s] : 0;
        const int end = ok ? (s + 1 < U ? R[s + 1] : n) : 0;
        const int len = end - beg;
        const bool isc = ok && len >= 2 && len <= ix.chunk_max;
        const bool ish = ok && len > ix.chunk_max;
        const int ns = ish ? (len + kHotSlice - 1) / kHotSlice : 0;
        const unsigned long long cb = __ballot(isc), hb = __ballot(ish);
        const int sincl = wave_incl_scan(ns);
        const int row = ok ? (int)(((kb > 0 && s == 0 ? hkey : Ks[beg - kb]) << vs) | part) : 0;
        SegRec r{};
        r.kind = isc ? 1 : (ish ? 2 : 0);
        r.ns = ns;
        if (isc) {
            int q[kChunkInline];
#pragma unroll
            for (int k = 0; k < kChunkInline; ++k) q[k] = beg + k < end ? Vs[beg + k - kb] : -1;
            r.idx = c + __popcll(cb & lt);
            r.a = make_int4((int)off + beg, (int)off + end, row, q[0]);
            r.b = make_int4(q[1], q[2], q[3], q[4]);
        } else if (ish) {
            r.idx = sl0 + sincl - ns;
            r.a = make_int4(beg, end, row, 0);
        }
        if (lists) {
            if (ok) {
                ix.seg_start[soff + s] = beg;
                ix.seg_row[off + s] = (uint32_t)row;
            }
            if (isc) {
                int4* chunks = ix.chunks + 2 * off;
                chunks[2 * r.idx] = make_int4(beg, end, row, r.a.w);
                chunks[2 * r.idx + 1] = r.b;
            }
            if (ish) {
                const int hi = h + __popcll(hb & lt);
                ix.hot[off + hi] = make_int4(beg, end, row, r.idx);
                for (int k = 0, p0 = beg; p0 < end; ++k, p0 += kHotSlice)
                    ix.hot_slice[off + r.idx + k] = make_int4(p0, min(p0 + kHotSlice, end), row, hi);
            }
        }
        c += __popcll(cb);
        h += __popcll(hb);
        sl0 += lane63(sincl);
        return r;
    }

    __device__ __forceinline__ void flat(const SegRec& r, int cbase, int sbase) const {
        if (r.kind == 1) {
            ix.chunk_rec[2 * (int64_t)(cbase + r.idx)] = r.a;
            ix.chunk_rec[2 * (int64_t)(cbase + r.idx) + 1] = r.b;
        } else if (r.kind == 2) {
            const int first = sbase + r.idx;
            for (int k = 0, p0 = r.a.x; p0 < r.a.y; ++k, p0 += kHotSlice) {
                ix.slice_rec[2 * (int64_t)(first + k)] =
                    make_int4((int)off + p0, (int)off + min(p0 + kHotSlice, r.a.y), r.a.z, v);
                ix.slice_rec[2 * (int64_t)(first + k) + 1] = make_int4(r.ns, first, 0, 0);
            }
        }
    }
};

// ---- the part's sort in registers (round 6): n <= 256 keys (row >> vs, < 2^nbits) with their
// index in the part's position-ordered list packed below them (IB = log2(64 R) bits), one
// bitonic network (bitonic.hpp) over R = 1, 2 or 4 registers, then each sorted key written with
// its position, read back through that index.  The same steps for any key distribution: skewed
// rows cost what uniform ones do.  32-bit keys while nbits + IB <= 32, else 64-bit (the 292M-row
// Terabyte table; its parts of more than 128 keys take the counting passes).
template <int R, typename V>
__device__ __forceinline__ void wave_sort_regs_r(int n, const uint32_t* K0, const int32_t* V0, uint32_t* K1,
                                                 int32_t* V1) {
    constexpr int IB = R == 1 ? 6 : (R == 2 ? 7 : (R == 4 ? 8 : 9));  // (n <= 64 R = 2^IB)
    const int lane = threadIdx.x & 63;
    V a[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = r * 64 + lane;
        // (padding: all ones, above every real key -- a real key of all ones would need i = 2^IB - 1,
        // i.e. n = 64 R, and then there is no padding)
        a[r] = i < n ? (((V)K0[i] << IB) | (V)i) : ~(V)0;
    }
    wave_bitonic_sort<R>(a);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = r * 64 + lane;
        if (i < n) {
            K1[i] = (uint32_t)(a[r] >> IB);
            V1[i] = V0[(int)(a[r] & (V)((1 << IB) - 1))];
        }
    }
    wave_lds_sync();
}

constexpr int kRegSortMax = 256;  // largest part sorted in registers (else the counting passes)

// Whether wave_sort_regs takes a part of n keys of nbits bits (uniform).
__device__ __forceinline__ bool regsort_takes(int n, int nbits) {
    return n > 1 && nbits > 0 && (n <= 128 || (n <= kRegSortMax && nbits + 8 <= 32));
}

// Sorts (K0, V0)[0, n) (LDS) into (K1, V1) by (key, position), where regsort_takes(n, nbits).
__device__ __forceinline__ void wave_sort_regs(int n, int nbits, const uint32_t* K0, const int32_t* V0, uint32_t* K1,
                                               int32_t* V1) {
    if (n <= 64 && nbits + 6 <= 32) wave_sort_regs_r<1, uint32_t>(n, K0, V0, K1, V1);
    else if (n <= 128 && nbits + 7 <= 32) wave_sort_regs_r<2, uint32_t>(n, K0, V0, K1, V1);
    else if (n <= 128) wave_sort_regs_r<2, uint64_t>(n, K0, V0, K1, V1);
    else wave_sort_regs_r<4, uint32_t>(n, K0, V0, K1, V1);
}

// A part of n > 256 keys dominated by one hot row (Zipf rows: a pooled table's hottest row takes
// ~18 % of its 20480 positions, all in one part): the wave picks the most frequent key of a
// 64-key sample, counts it (nh), and when the other n - nh keys fit the register sort, partitions
// the part stably -- the hot row's positions to the front of (K0, V0) in place (they come in
// position order: a segment as it is), the others to (K1, V1)[nh, n) -- and sorts those in
// registers back into (K0, V0)[nh, n).  Returns false (nothing written) otherwise: the caller
// sorts the part the general way.  The same cost whatever the hot row's share, instead of the
// counting passes' serial walk over every key of the hot bucket.
template <bool G>
__device__ __forceinline__ bool bag_hot_sort(int n, int nbits, uint32_t* K0, int32_t* V0, uint32_t* K1, int32_t* V1) {
    const int lane = threadIdx.x & 63;
    const uint32_t mine = K0[(int64_t)lane * n / 64];
    int c = 0;
    for (int j = 0; j < 64; ++j) c += __shfl(mine, j, 64) == mine ? 1 : 0;
    int best = (c << 6) | lane;  // the most frequent sample key (ties: highest lane)
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) best = max(best, __shfl_xor(best, off, 64));
    const uint32_t hkey = __shfl(mine, best & 63, 64);
    int nh = 0;
    for (int i0 = 0; i0 < n; i0 += 256) {  // (four tiles' loads in flight)
        uint32_t k[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) k[u] = i0 + 64 * u + lane < n ? K0[i0 + 64 * u + lane] : ~hkey;
#pragma unroll
        for (int u = 0; u < 4; ++u) nh += __popcll(__ballot(k[u] == hkey));
    }
    if (!regsort_takes(n - nh, nbits) && n - nh > 1) return false;
    const unsigned long long below = lanes_below();
    int hrun = 0, rrun = nh;
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        const bool ok = i < n;
        const uint32_t k = ok ? K0[i] : 0u;
        const int32_t p = ok ? V0[i] : 0;
        const bool hot = ok && k == hkey;
        const unsigned long long hb = __ballot(hot), rb = __ballot(ok && !hot);
        if (hot) {  // (in place: i >= hrun + rank, and every lane has read its entry)
            K0[hrun + __popcll(hb & below)] = hkey;
            V0[hrun + __popcll(hb & below)] = p;
        } else if (ok) {
            K1[rrun + __popcll(rb & below)] = k;
            V1[rrun + __popcll(rb & below)] = p;
        }
        hrun += __popcll(hb);
        rrun += __popcll(rb);
    }
    part_sync<G>();
    if (n - nh > 1) {
        wave_sort_regs(n - nh, nbits, K1 + nh, V1 + nh, K0 + nh, V0 + nh);
        part_sync<G>();
    } else if (n - nh == 1 && lane == 0) {
        K0[nh] = K1[nh];
        V0[nh] = V1[nh];
    }
    part_sync<G>();
    return true;
}

// The part the calling wave sorts and writes out: virtual table v = (t << vs) + part, its n keys
// (row >> vs) and positions in position order at K0 / V0 (K1, V1, R: the same span of the pool's
// other arrays, scratch).  Sorts them in LDS: keys wider than 8 bits by one unstable counting pass
// on the low byte and a within-bucket rank on (key, position); narrow keys, or buckets too big to
// rank (skewed rows), by stable LSD counting passes.  Then classifies the segments (LDS only), reserves the wave's ranges of the flat item lists and arrives in one packed atomic
// add, stores the per-table outputs while it is in flight, then the flat records at its return.
// DIRECT: a part of one row (its table has <= 2^vs rows): the caller already wrote perm (positions in
// order) and the once-hit flags; K0 / V0 hold the part's first (up to 8) keys / positions and R room
// for one segment start -- the part is one segment, nothing is sorted.
// PRESORTED: (K0, V0) already hold the part grouped by row (bag_hot_sort); only the pass below runs.
// nh0 > 0 (PRESORTED only): the part's first nh0 entries are one hot row's (key hkey) whose perm
// entries and once-hit flags the caller has written; (K0, V0) hold the other n - nh0, grouped.
template <bool G, bool DIRECT = false, bool PRESORTED = false>
__device__ __forceinline__ void wave_sort_part(const IndexerDev& ix, int v, int t, int vs, uint32_t nrows, int n,
                                               int toff, uint32_t* K0, int32_t* V0, uint32_t* K1, int32_t* V1,
                                               int32_t* R, uint32_t* cnt, int g, int groups, int nh0 = 0,
                                               uint32_t hkey = 0) {
    const int lane = threadIdx.x & 63;
    const uint32_t part = (uint32_t)v & ((1u << vs) - 1u);
    const uint32_t kmax = nrows > 0 ? (nrows - 1) >> vs : 0u;
    const int nbits = 32 - __clz(kmax);
    WPH(2);
    const uint32_t* Ks = K0;
    const int32_t* Vs = V0;
    const int nr = n - nh0;  // (the entries in K0 / V0: all but a hot prefix)
    if (DIRECT || PRESORTED) {
    } else if (!G && regsort_takes(nr, nbits)) {  // (uniform: n, nbits)
        WPH(3);
        wave_sort_regs(nr, nbits, K0, V0, K1, V1);
        Ks = K1;
        Vs = V1;
    } else if (nr > 1 && nbits > 8 && wave_count_pass_unstable<G>(nr, K0, V0, K1, V1, R, cnt) <= kWaveRankMax) {
        WPH(3);
        wave_rank_buckets<G>(nr, K1, V1, K0, V0, cnt);
    } else if (nr > 1 && nbits > 0) {  // narrow keys, or skewed rows: stable LSD passes from (K0, V0)
        wave_count_pass<G>(nr, 0, nbits < 8 ? nbits : 8, K0, V0, K1, V1, R, cnt);
        WPH(3);
        Ks = K1;
        Vs = V1;
        for (int shift = 8; shift < nbits; shift += 8) {
            const bool from1 = Ks == K1;
            wave_count_pass<G>(nr, shift, nbits - shift < 8 ? nbits - shift : 8, from1 ? K1 : K0, from1 ? V1 : V0,
                            from1 ? K0 : K1, from1 ? V0 : V1, R, cnt);
            Ks = from1 ? K0 : K1;
            Vs = from1 ? V0 : V1;
        }
    }
    WPH(4);
    // One pass over the sorted keys, four consecutive keys per lane (16-B LDS reads: the part's
    // region starts 16-B aligned): perm and the once-hit flags stored, segment starts R[s], and the
    // counts that size the wave's share of the flat lists -- chunks (a head that is not a tail and
    // whose key differs cm places on: 2 .. cm positions) and hot segments (longer), whose
    // slices are counted from R after.  (Its stores precede the reservation atomic below; they
    // complete before it returns anyway.)
    const int cm = ix.chunk_max;  // this build's chunk limit (16 or 32)
    const int64_t off = (int64_t)t * ix.cap + toff;  // (the compact layout, common.hpp)
    const int64_t soff = (int64_t)t * (ix.cap + kSegPad) + toff + (int)part;
    int32_t* perm = ix.perm + off + nh0;
    uint8_t* single = ix.single + (int64_t)t * ix.cap;
    const bool pvec = ((off + nh0) & 3) == 0;  // perm + i 16-B aligned
    int U = 0, C = 0, H = 0;
    if (DIRECT || nh0 > 0) {  // (one segment already written: the whole part, or the hot prefix)
        const int n1 = DIRECT ? n : nh0;
        U = n1 > 0 ? 1 : 0;
        C = n1 >= 2 && n1 <= cm ? 1 : 0;
        H = n1 > cm ? 1 : 0;
        if (lane == 0) R[0] = 0;
    }
    for (int j0 = 0; j0 < (DIRECT ? 0 : nr); j0 += 256) {
        const int i = j0 + 4 * lane;
        const uint4 k4 = *(const uint4*)(Ks + i);  // (past n: garbage, masked below)
        const int4 v4 = *(const int4*)(Vs + i);
        const uint4 kf = *(const uint4*)(Ks + i + cm);  // (cm % 4 == 0: 16-B aligned)
        const uint32_t kp = Ks[i > 0 ? i - 1 : 0], kn = Ks[i + 4];
        const uint32_t kk[6] = {kp, k4.x, k4.y, k4.z, k4.w, kn};
        const uint32_t kfa[4] = {kf.x, kf.y, kf.z, kf.w};
        const int vv[4] = {v4.x, v4.y, v4.z, v4.w};
        int nh = 0, nc = 0, nhot = 0;
        bool hd[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int ie = i + e;
            const bool ok = ie < nr;
            const bool head = ok && (ie == 0 || kk[e] != kk[e + 1]);
            const bool tail = ok && (ie + 1 == nr || kk[e + 2] != kk[e + 1]);
            const bool longer = ok && ie + cm < nr && kfa[e] == kk[e + 1];
            hd[e] = head;
            nh += head ? 1 : 0;
            nc += (head && !tail && !longer) ? 1 : 0;
            nhot += (head && longer) ? 1 : 0;
            if (ok) single[vv[e]] = (head && tail) ? 1 : 0;
        }
        if (pvec && i + 3 < nr)
            *(int4*)(perm + i) = v4;
        else
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (i + e < nr) perm[i + e] = vv[e];
        // (three 10-bit fields: <= 256 per tile)
        const int packed = nh | (nc << 10) | (nhot << 20);
        const int incl = wave_incl_scan(packed), tot = lane63(incl);
        int at = U + ((incl - packed) & 1023);
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (hd[e]) R[at++] = nh0 + i + e;
        U += tot & 1023;
        C += (tot >> 10) & 1023;
        H += tot >> 20;
    }
    part_sync<G>();
    int S = 0;
    if (H)  // (rows hit more than cm times in this part: small tables)
        for (int s0 = 0; s0 < U; s0 += 64) {
            const int s = s0 + lane;
            const int len = s < U ? (s + 1 < U ? R[s + 1] : n) - R[s] : 0;
            S += lane63(wave_incl_scan(len > cm ? (len + kHotSlice - 1) / kHotSlice : 0));
        }
    // The wave reserves its flat-list ranges and arrives in ONE atomic add (lane 0): the segment
    // stores below run while it is in flight, and only the flat records wait for it.
    unsigned long long res = 0ull;
    const int list = g & (kResLists - 1);
    unsigned long long* word = (unsigned long long*)ix.build_arrive + list * kResWordStride;
    if (lane == 0) {
        // (a zero the compiler cannot see through: a uniform address gets the wave-aggregating
        // atomic rewrite, whose readfirstlane would wait for the return right here)
        int zero;
        asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
        res = __hip_atomic_fetch_add(word + zero,
                                     (unsigned long long)C + ((unsigned long long)S << kResSliceShift) +
                                         (1ull << kResArriveShift),
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    WPH(5);
    WPH(9);
    // segments: the first two tiles keep their flat records in registers for after the reservation
    // returns; later tiles (U > 128) are recomputed then
    SegPass sp{ix, v, vs, part, n, U, Ks, Vs, R, off, soff, nh0, hkey};
    int c = 0, h = 0, sl0 = 0;
    const SegRec r0 = sp.tile(0, c, h, sl0, true);
    const SegRec r1 = U > 64 ? sp.tile(64, c, h, sl0, true) : SegRec{};
    const int c2 = c, s2 = sl0;
    for (int s0 = 128; s0 < U; s0 += 64) (void)sp.tile(s0, c, h, sl0, true);
    if (lane == 0) {
        ix.seg_start[soff + U] = n;
        int32_t* cn = ix.counts + (int64_t)v * 8;
        cn[CNT_U] = U; cn[CNT_C] = c; cn[CNT_H] = h; cn[CNT_S] = sl0; cn[CNT_NV] = n; cn[CNT_OFF] = toff;
    }
    // the reservation's return: the wave's bases in its sub-list; the sub-list's last wave to arrive
    // publishes its totals and clears the word for this indexer's next build (read in a later launch)
    res = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(res >> 32)) << 32) |
          (unsigned)__builtin_amdgcn_readfirstlane((unsigned)res);
    WPH(8);
    const int cloc = (int)(res & ((1u << kResSliceShift) - 1u));
    const int sloc = (int)((res >> kResSliceShift) & ((1u << (kResArriveShift - kResSliceShift)) - 1u));
    const int lwaves = ((groups - list + kResLists - 1) / kResLists) * kWaveParts;  // this sub-list's
    if (lane == 0 && (unsigned)(res >> kResArriveShift) == (unsigned)(lwaves - 1)) {
        ix.item_tot[list] = sloc + S;
        ix.item_tot[kResLists + list] = cloc + C;
        *word = 0ull;
    }
    const int lbase = list * res_stride(groups, ix.cap, vs);
    const int cbase = lbase + cloc, sbase = lbase + sloc;
    // the flat records (chunk_rec, slice_rec) at the reserved ranges
    sp.flat(r0, cbase, sbase);
    sp.flat(r1, cbase, sbase);
    c = c2;
    sl0 = s2;
    for (int s0 = 128; s0 < U; s0 += 64) sp.flat(sp.tile(s0, c, h, sl0, false), cbase, sbase);
    WPH(6);
}

// One round of a build wave's index loads: positions 2048 r + 512 w + 256 k + 4 lane + e (k < 2,
// e < 4) of table t.  wave_round_load issues them (a caller loads the next round before decoding this
// one, so one round's latency hides behind the other's work); wave_round_decode gives rv[j] =
// row >> vs, code (3 bits per element j = 4 k + e) = its part - q0 (0..3) or 4 (another workgroup's
// part, past N, or out of range), and per piece k and part q this lane's exclusive prefix over the
// wave (pre) and the wave's total (ptot), by DPP scans of two 16-bit fields per word.  bad: an
// out-of-range index among this lane's.
struct WaveRaw {
    int64_t rr[8];
    bool in[8];
};

struct WaveRound {
    uint32_t rv[8];
    uint32_t code;
    bool bad;
    int below;  // this lane's positions in parts below q0 (the compact layout's table offset)
    int pre[2][kWaveParts], ptot[2][kWaveParts];
};

__device__ __forceinline__ WaveRaw wave_round_load(int r, int w, int t, const void* __restrict__ idx, int itype,
                                                   int64_t tstride, int N) {
    constexpr int PK = 2;
    const int lane = threadIdx.x & 63;
    const int p0 = kStepIndexMaxN * r + (kStepIndexMaxN / kWaveParts) * w;
    const int32_t* i32 = (const int32_t*)idx + (int64_t)t * tstride;
    const int64_t* i64 = (const int64_t*)idx + (int64_t)t * tstride;
    const bool vec = N % 256 == 0 && (itype == DLRM_I32 ? (uintptr_t)i32 % 16 == 0 : (uintptr_t)i64 % 16 == 0);
    WaveRaw o;
    if (vec && itype == DLRM_I32) {
        int4 q[PK];
#pragma unroll
        for (int k = 0; k < PK; ++k)
            if (p0 + 256 * k < N) q[k] = ldg<int4>(i32 + p0 + 256 * k + 4 * lane);
#pragma unroll
        for (int k = 0; k < PK; ++k) {
            const bool kin = p0 + 256 * k < N;
            o.rr[4 * k] = q[k].x; o.rr[4 * k + 1] = q[k].y; o.rr[4 * k + 2] = q[k].z; o.rr[4 * k + 3] = q[k].w;
#pragma unroll
            for (int e = 0; e < 4; ++e) o.in[4 * k + e] = kin;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4 * PK; ++j) {
            const int pj = p0 + 256 * (j >> 2) + 4 * lane + (j & 3);
            o.in[j] = pj < N;
            o.rr[j] = load_index_if(o.in[j], idx, itype, (int64_t)t * tstride + pj);
        }
    }
    return o;
}

__device__ __forceinline__ void wave_round_decode(WaveRound& o, const WaveRaw& raw, int q0, int vs, uint32_t nrows,
                                                  int base) {
    constexpr int PK = 2;
    const uint32_t pmask = (1u << vs) - 1u;
    WPH(7);
    o.code = 0;
    o.bad = false;
    o.below = 0;
#pragma unroll
    for (int j = 0; j < 4 * PK; ++j) {
        const int64_t x = raw.rr[j] - base;
        const bool ok = raw.in[j] && (uint64_t)x < (uint64_t)nrows;  // (negative: a huge unsigned)
        o.bad |= raw.in[j] && !ok;
        o.below += ok && ((uint32_t)x & pmask) < (uint32_t)q0 ? 1 : 0;
        const uint32_t pq = ((uint32_t)x & pmask) - (uint32_t)q0;
        o.code |= (ok && pq < (uint32_t)kWaveParts ? pq : 4u) << (3 * j);
        o.rv[j] = (uint32_t)x >> vs;
    }
#pragma unroll
    for (int k = 0; k < PK; ++k) {
        int cq[kWaveParts] = {0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t cd = (o.code >> (3 * (4 * k + e))) & 7u;
#pragma unroll
            for (int q = 0; q < kWaveParts; ++q) cq[q] += cd == (uint32_t)q ? 1 : 0;
        }
        const int a = cq[0] | (cq[1] << 16), b = cq[2] | (cq[3] << 16);
        const int ia = wave_incl_scan(a), ib = wave_incl_scan(b);
        const int ta = lane63(ia), tb = lane63(ib);
        o.pre[k][0] = (ia - a) & 0xffff; o.pre[k][1] = (ia - a) >> 16;
        o.pre[k][2] = (ib - b) & 0xffff; o.pre[k][3] = (ib - b) >> 16;
        o.ptot[k][0] = ta & 0xffff; o.ptot[k][1] = ta >> 16; o.ptot[k][2] = tb & 0xffff; o.ptot[k][3] = tb >> 16;
    }
}

// One build workgroup (kWaveParts waves = 256 threads): parts q0 .. q0 + 3 (q0 = 4 (g mod P / 4))
// of table t = g / (P / 4), P = 2^vs >= 4 parts per table.  Every thread of the workgroup calls
// it.  The four waves first split the table's positions among the four parts together -- in rounds
// of 2048 positions, wave w reading positions [2048 r + 512 w, + 512), 16-B loads, and the parts'
// lists keep position order by (round, wave, piece, lane) offsets from DPP scans and one exchange
// of per-wave counts -- then wave q sorts part q0 + q alone (wave_sort_part).  Up to 2048
// positions (one round) the loads are kept in registers across the exchange; beyond, a second pass
// reloads them (from L2) to place them.  When the four parts overflow the LDS pool (their positions
// total more than 2048: a tiny table's few rows, or hot rows, at large N) the parts are placed and
// sorted in HBM scratch instead (ix.wscratch; the same sort, G = true).  The last of the T P / 4
// workgroups to arrive publishes the flat lists' totals (finish_item_lists).
// BIG = false: N <= 2048 (one round, the pool never overflows) -- the forward launch's build, whose
// registers the HBM path would crowd; BIG = true: any N <= kWaveMaxN.
template <bool BIG = true>
__device__ __forceinline__ void wave_build_group(const IndexerDev& ix, int g, int T, const TableDesc* __restrict__ tabs,
                                 const void* __restrict__ idx, int itype, int64_t tstride, int base, int N,
                                 unsigned* __restrict__ err, WaveBuildLds& sl) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int vs = ix.vshift, gpt = (1 << vs) / kWaveParts;  // workgroups per table
    const int t = g / gpt, q0 = (g - t * gpt) * kWaveParts;
    const uint32_t nrows = (uint32_t)load_table(tabs, t).nrows;
    const int R = BIG ? (N + kStepIndexMaxN - 1) / kStepIndexMaxN : 1;  // rounds (<= kWaveMaxN / 2048)
    WPH(0);
    WaveRound rd;
    bool bad = false;
    int blw = 0;  // positions of parts below q0 this lane read
    // BIG with 16-B int32 index loads: rounds in batches of RB, each batch's loads issued together
    // (one latency per batch, not per round); otherwise round by round
    constexpr int RB = BIG ? 2 : 1;
    const int32_t* i32 = (const int32_t*)idx + (int64_t)t * tstride;
    const bool vec32 = BIG && itype == DLRM_I32 && N % 256 == 0 && (uintptr_t)i32 % 16 == 0;
    int4 qa[RB][2];
    auto load_batch = [&](int r0) {  // (vec32) rounds r0 .. r0 + RB - 1
#pragma unroll
        for (int j = 0; j < RB; ++j)
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int p = kStepIndexMaxN * (r0 + j) + (kStepIndexMaxN / kWaveParts) * w + 256 * k;
                if (r0 + j < R && p < N) qa[j][k] = ldg<int4>(i32 + p + 4 * lane);
            }
    };
    auto raw_of = [&](int r, int j) {  // (vec32) round r = r0 + j's raw indices from registers
        WaveRaw o;
        const int p0 = kStepIndexMaxN * r + (kStepIndexMaxN / kWaveParts) * w;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const bool kin = p0 + 256 * k < N;
            o.rr[4 * k] = qa[j][k].x; o.rr[4 * k + 1] = qa[j][k].y; o.rr[4 * k + 2] = qa[j][k].z;
            o.rr[4 * k + 3] = qa[j][k].w;
#pragma unroll
            for (int e = 0; e < 4; ++e) o.in[4 * k + e] = kin;
        }
        return o;
    };
    auto count_round = [&](int r) {  // pass 1's bookkeeping of round r (rd decoded)
        bad |= rd.bad;
        blw += rd.below;
        if (lane < kWaveParts) {
            int tw = 0;
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int q = 0; q < kWaveParts; ++q) tw += lane == q ? rd.ptot[k][q] : 0;
            sl.tot[r][w][lane] = tw;
        }
    };
    if (vec32) {  // pass 1: count
        for (int r0 = 0; r0 < R; r0 += RB) {
            load_batch(r0);
#pragma unroll
            for (int j = 0; j < RB; ++j)
                if (r0 + j < R) {
                    wave_round_decode(rd, raw_of(r0 + j, j), q0, vs, nrows, base);
                    count_round(r0 + j);
                }
        }
    } else {
        for (int r = 0; r < R; ++r) {
            wave_round_decode(rd, wave_round_load(r, w, t, idx, itype, tstride, N), q0, vs, nrows, base);
            count_round(r);
        }
    }
    // out of range raises BoundsError; the workgroup of parts 0..3 reports it
    if (q0 == 0 && __ballot(bad) && lane == 0) raise_index_error(err);
    blw = lane63(wave_incl_scan(blw));
    if (lane == 0) sl.below[w] = blw;
    __syncthreads();
    // part q's size, its region (pool: 16-B aligned, in part order; HBM: its compact region), the
    // offset of each round's share of wave w in it, and its offset in the table's compact region
    int n_of[kWaveParts], pbase[kWaveParts], toff[kWaveParts], total = 0;
    int tq = 0;
#pragma unroll
    for (int ww = 0; ww < kWaveParts; ++ww) tq += sl.below[ww];
#pragma unroll
    for (int q = 0; q < kWaveParts; ++q) {
        int nq = 0;
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int ww = 0; ww < kWaveParts; ++ww) nq += sl.tot[r][ww][q];
        n_of[q] = nq;
        pbase[q] = total;
        toff[q] = tq;
        tq += nq;
        total += (nq + 3) & ~3;  // (16-B aligned regions: wave_sort_part's vector reads)
    }
    // a table of <= 2^vs rows: every part is one row (DIRECT: positions go straight to perm in order,
    // nothing is sorted); else a workgroup whose parts overflow the pool sorts them in HBM (G)
    const bool direct = BIG && nrows > 0 && ((nrows - 1) >> vs) == 0;
    const bool G = BIG && !direct && total > kStepIndexMaxN;  // (uniform over the workgroup)
    WPH(1);
    int run[kWaveParts];  // part q's positions in the rounds before this one
#pragma unroll
    for (int q = 0; q < kWaveParts; ++q) run[q] = 0;
    auto place_round = [&](int r) {  // pass 2: round r (rd decoded) into the parts' regions
        int at0[kWaveParts];
#pragma unroll
        for (int q = 0; q < kWaveParts; ++q) {
            int before = run[q], all = 0;  // earlier rounds, then this round's earlier waves
#pragma unroll
            for (int ww = 0; ww < kWaveParts; ++ww) {
                const int c = sl.tot[r][ww][q];
                before += ww < w ? c : 0;
                all += c;
            }
            at0[q] = (G || direct ? 0 : pbase[q]) + before;
            run[q] += all;
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            int at[kWaveParts];
#pragma unroll
            for (int q = 0; q < kWaveParts; ++q) at[q] = at0[q] + (k ? rd.ptot[0][q] : 0) + rd.pre[k][q];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t cd = (rd.code >> (3 * (4 * k + e))) & 7u;
                if (cd < (uint32_t)kWaveParts) {
                    int dst = 0;
#pragma unroll
                    for (int q = 0; q < kWaveParts; ++q)
                        if (cd == (uint32_t)q) dst = at[q]++;
                    const int32_t pos = kStepIndexMaxN * r + (kStepIndexMaxN / kWaveParts) * w + 256 * k + 4 * lane + e;
                    if (direct) {  // the part's perm entry and the position's once-hit flag, now
                        int nq = 0, to = 0;
#pragma unroll
                        for (int q = 0; q < kWaveParts; ++q) {
                            nq = cd == (uint32_t)q ? n_of[q] : nq;
                            to = cd == (uint32_t)q ? toff[q] : to;
                        }
                        ix.perm[(int64_t)t * ix.cap + to + dst] = pos;
                        ix.single[(int64_t)t * ix.cap + pos] = nq == 1 ? 1 : 0;
                        if (dst < 8) {  // (the part's first positions: its chunk record carries 5 inline)
                            sl.K[0][8 * (int)cd + dst] = rd.rv[4 * k + e];
                            sl.V[0][8 * (int)cd + dst] = pos;
                        }
                    } else if (G) {
                        int to = 0;
#pragma unroll
                        for (int q = 0; q < kWaveParts; ++q) to = cd == (uint32_t)q ? toff[q] : to;
                        const int64_t vo = (int64_t)t * ix.cap + to + dst;
                        ix.wscratch[vo] = rd.rv[4 * k + e];
                        ((int32_t*)ix.wscratch)[ix.wstride + vo] = pos;
                    } else {
                        sl.K[0][dst] = rd.rv[4 * k + e];
                        sl.V[0][dst] = pos;
                    }
                }
            }
        }
    };
    if (!BIG) {
        place_round(0);  // (one round: rd still holds it)
    } else if (vec32) {
        for (int r0 = 0; r0 < R; r0 += RB) {
            load_batch(r0);
#pragma unroll
            for (int j = 0; j < RB; ++j)
                if (r0 + j < R) {
                    wave_round_decode(rd, raw_of(r0 + j, j), q0, vs, nrows, base);
                    place_round(r0 + j);
                }
        }
    } else {
        for (int r = 0; r < R; ++r) {
            wave_round_decode(rd, wave_round_load(r, w, t, idx, itype, tstride, N), q0, vs, nrows, base);
            place_round(r);
        }
    }
    if (G) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (G) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // wave w sorts part q0 + w
    const int n = n_of[w];
    const int v = (t << vs) + q0 + w;
    const int groups = (T << vs) / kWaveParts;
    if (BIG && direct) {
        wave_sort_part<false, true>(ix, v, t, vs, nrows, n, toff[w], sl.K[0] + 8 * w, sl.V[0] + 8 * w,
                                    sl.K[1] + 8 * w, sl.V[1] + 8 * w, sl.R + 8 * w, sl.cnt[w], g, groups);
    } else if (BIG && G) {
        uint32_t* K0 = ix.wscratch + (int64_t)t * ix.cap + toff[w];
        const int64_t S = ix.wstride;
        wave_sort_part<true>(ix, v, t, vs, nrows, n, toff[w], K0, (int32_t*)(K0 + S), K0 + 2 * S,
                             (int32_t*)(K0 + 3 * S), (int32_t*)(K0 + 4 * S), sl.cnt[w], g, groups);
    } else {
        const int pb = pbase[w];
        wave_sort_part<false>(ix, v, t, vs, nrows, n, toff[w], sl.K[0] + pb, sl.V[0] + pb, sl.K[1] + pb,
                              sl.V[1] + pb, sl.R + pb, sl.cnt[w], g, groups);
    }
}

// The large-N builds' last step (after the workgroup barrier that follows the placement): wave w
// sorts part q0 + w of table t -- n positions placed at pool offset pb, in HBM scratch (G), or
// already in perm (direct).
__device__ __forceinline__ void wave_build_sort(const IndexerDev& ix, int g, int T, int t, int q0, int vs,
                                                uint32_t nrows, int n, int toff, int pb, bool direct, bool G,
                                                WaveBuildLds& sl) {
    const int w = threadIdx.x >> 6;
    const int v = (t << vs) + q0 + w;
    const int groups = (T << vs) / kWaveParts;
    if (direct) {
        wave_sort_part<false, true>(ix, v, t, vs, nrows, n, toff, sl.K[0] + 8 * w, sl.V[0] + 8 * w,
                                    sl.K[1] + 8 * w, sl.V[1] + 8 * w, sl.R + 8 * w, sl.cnt[w], g, groups);
    } else if (G) {
        uint32_t* K0 = ix.wscratch + (int64_t)t * ix.cap + toff;
        const int64_t S = ix.wstride;
        wave_sort_part<true>(ix, v, t, vs, nrows, n, toff, K0, (int32_t*)(K0 + S), K0 + 2 * S,
                             (int32_t*)(K0 + 3 * S), (int32_t*)(K0 + 4 * S), sl.cnt[w], g, groups);
    } else {
        wave_sort_part<false>(ix, v, t, vs, nrows, n, toff, sl.K[0] + pb, sl.V[0] + pb, sl.K[1] + pb,
                              sl.V[1] + pb, sl.R + pb, sl.cnt[w], g, groups);
    }
}

// ---------------------------------------------------------------- scan wave build (N > 2048)
// The one-launch build above 2048 positions per table without rounds: wave w of the workgroup's NW
// (parts q0 .. q0 + 3 of table t) takes a contiguous 1 / NW of the table's positions, so the
// parts' lists keep position order by (wave, piece, lane) offsets and the waves exchange nothing
// but one count per part.  The quarter's indices are loaded once, all at once (pieces of 256
// positions, one 16-B load per lane; <= 16 pieces = 64 registers at 16384 positions), and stay in
// registers for two lean passes:
//   1. count: per lane, this workgroup's positions per part in four 8-bit fields (<= 64 per lane),
//      and a bit per position that is this workgroup's ("mine"); one wave reduction at the end;
//   2. place: through a staging list when the four parts fit the LDS pool -- the wave's mine
//      positions (~N / 32 at 128 parts) are appended in position order to its range of the pool's
//      second array (part code in the top bits; one DPP scan per two pieces, of the lanes' mine
//      counts), then split by part into their regions (two scans per 64 staged entries), so the
//      per-part placement runs once per staged entry instead of once per piece; else (HBM scratch,
//      or perm straight away for a table of <= P rows) by per-piece prefixes per part.
// Every workgroup of a table still reads all N of its indices (from L2: 64 KB at 16384).  The scan
// is a chain of dependent VALU / DPP steps, so more waves shorten it: the standalone build runs 16
// waves per workgroup (4 per SIMD; waves 4 .. 15 leave before the sort), the in-apply build 4.  Needs
// int32 indices, 16-B aligned per table, N % 4 == 0 (else the rounds form runs).
template <int NW, int MAXN = kWaveApplyMaxN>
__device__ __forceinline__ void wave_build_group_scan(const IndexerDev& ix, int g, int T, const TableDesc* __restrict__ tabs,
                                      const void* __restrict__ idx, int64_t tstride, int base, int N,
                                      unsigned* __restrict__ err, WaveBuildLds& sl) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int vs = ix.vshift, gpt = (1 << vs) / kWaveParts;  // workgroups per table
    const int t = g / gpt, q0 = (g - t * gpt) * kWaveParts;
    const uint32_t nrows = (uint32_t)load_table(tabs, t).nrows;
    const uint32_t pmask = (1u << vs) - 1u;
    const int32_t* i32 = (const int32_t*)idx + (int64_t)t * tstride;
    const int Q = ((N + NW * 256 - 1) / (NW * 256)) * 256;  // positions per wave (whole pieces)
    const int pw0 = w * Q;
    const int npc = pw0 < N ? (min(pw0 + Q, N) - pw0 + 255) / 256 : 0;  // this wave's pieces
    constexpr int MP = MAXN / NW / 256;  // pieces per wave (<= 16: mbits; 16384 / 16 waves: 4, / 4: 16)
    static_assert(MP >= 1 && MP <= 16 && MAXN <= kWaveMaxN, "scan build: <= 16 pieces per wave");
    WPH(0);
    int4 v[MP];
#pragma unroll
    for (int u = 0; u < MP; ++u) {
        const int p = pw0 + 256 * u + 4 * lane;
        if (u < npc && p < N) v[u] = ldg<int4>(i32 + p);
    }
    // pass 1: count
    uint32_t acc = 0;
    uint64_t mbits = 0;
    bool bad = false;
    int blw = 0;  // positions of parts below q0 (the compact layout's table offset)
#pragma unroll
    for (int u = 0; u < MP; ++u) {
        // (a guard, not a break: a loop with two exits is not unrolled, and v[] would go to scratch)
        const bool in = u < npc && pw0 + 256 * u + 4 * lane < N;
        const int xv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t x = (uint32_t)(xv[e] - base);
            const bool ok = in && x < nrows;
            bad |= in && !ok;
            const uint32_t pq = (x & pmask) - (uint32_t)q0;
            const bool m = ok && pq < (uint32_t)kWaveParts;
            blw += ok && (x & pmask) < (uint32_t)q0 ? 1 : 0;
            acc += m ? 1u << (8 * pq) : 0u;
            mbits |= m ? 1ull << (4 * u + e) : 0ull;
        }
    }
    if (q0 == 0 && __ballot(bad) && lane == 0) raise_index_error(err);
    {
        const int a = (int)((acc & 0xffu) | (((acc >> 8) & 0xffu) << 16));
        const int b = (int)(((acc >> 16) & 0xffu) | ((acc >> 24) << 16));
        const int ta = lane63(wave_incl_scan(a)), tb = lane63(wave_incl_scan(b));
        const int tbl = lane63(wave_incl_scan(blw));
        if (lane == 0) {
            scan_wave_totals(sl)[w] = make_int4(ta & 0xffff, ta >> 16, tb & 0xffff, tb >> 16);
            sl.below[w] = tbl;
        }
    }
    __syncthreads();
    int n_of[kWaveParts], pbase[kWaveParts], at0[kWaveParts], toff[kWaveParts], total = 0, sbase = 0;
    int4 nall = make_int4(0, 0, 0, 0), nbef = make_int4(0, 0, 0, 0);
    int tq = 0;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) {
        tq += sl.below[ww];
        const int4 c = scan_wave_totals(sl)[ww];
        nall = make_int4(nall.x + c.x, nall.y + c.y, nall.z + c.z, nall.w + c.w);
        if (ww < w) nbef = make_int4(nbef.x + c.x, nbef.y + c.y, nbef.z + c.z, nbef.w + c.w);
    }
#pragma unroll
    for (int q = 0; q < kWaveParts; ++q) {
        const int nq = q == 0 ? nall.x : (q == 1 ? nall.y : (q == 2 ? nall.z : nall.w));
        const int before = q == 0 ? nbef.x : (q == 1 ? nbef.y : (q == 2 ? nbef.z : nbef.w));
        n_of[q] = nq;
        pbase[q] = total;
        toff[q] = tq;
        tq += nq;
        at0[q] = before;
        sbase += before;
        total += (nq + 3) & ~3;  // (16-B aligned regions: wave_sort_part's vector reads)
    }
    const bool direct = nrows > 0 && ((nrows - 1) >> vs) == 0;
    const bool G = !direct && total > kStepIndexMaxN;  // (uniform over the workgroup)
    WPH(1);
    if (!G && !direct) {
#pragma unroll
        for (int q = 0; q < kWaveParts; ++q) at0[q] += pbase[q];
        uint32_t* SK = sl.K[1];
        int32_t* SV = sl.V[1];
        int run = sbase;
        auto stage = [&](const int4 vu, int u, int at) {  // (vu = v[u]: registers, u unrolled)
            const int p = pw0 + 256 * u + 4 * lane;
            const int xv[4] = {vu.x, vu.y, vu.z, vu.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if ((mbits >> (4 * u + e)) & 1ull) {
                    const uint32_t x = (uint32_t)(xv[e] - base);
                    SK[at] = x >> vs;
                    SV[at] = (p + e) | (int)(((x & pmask) - (uint32_t)q0) << 28);
                    ++at;
                }
        };
#pragma unroll
        for (int u = 0; u < MP; u += 2) {
            if (u >= npc) continue;  // (uniform)
            const int c0 = __popc((uint32_t)(mbits >> (4 * u)) & 15u);
            const int c1 = u + 1 < npc ? __popc((uint32_t)(mbits >> (4 * u + 4)) & 15u) : 0;
            const int pk = c0 | (c1 << 16);
            const int incl = wave_incl_scan(pk), tot = lane63(incl);
            const int ex = incl - pk;
            stage(v[u], u, run + (ex & 0xffff));
            if (u + 1 < npc) stage(v[u + 1], u + 1, run + (tot & 0xffff) + (ex >> 16));
            run += (tot & 0xffff) + (tot >> 16);
        }
        wave_lds_sync();
        for (int s0 = sbase; s0 < run; s0 += 64) {
            const int s = s0 + lane;
            const bool ok = s < run;
            const uint32_t key = ok ? SK[s] : 0u;
            const int32_t sv = ok ? SV[s] : 0;
            const int q = ok ? (int)((uint32_t)sv >> 28) : 4;
            const int a = (q == 0 ? 1 : 0) | (q == 1 ? 1 << 16 : 0), b = (q == 2 ? 1 : 0) | (q == 3 ? 1 << 16 : 0);
            const int ia = wave_incl_scan(a), ib = wave_incl_scan(b);
            const int ta = lane63(ia), tb = lane63(ib);
            const int pre[kWaveParts] = {(ia - a) & 0xffff, (ia - a) >> 16, (ib - b) & 0xffff, (ib - b) >> 16};
            int dst = 0;
#pragma unroll
            for (int qq = 0; qq < kWaveParts; ++qq) dst = q == qq ? at0[qq] + pre[qq] : dst;
            if (ok) {
                sl.K[0][dst] = key;
                sl.V[0][dst] = sv & 0x0fffffff;
            }
            at0[0] += ta & 0xffff;
            at0[1] += ta >> 16;
            at0[2] += tb & 0xffff;
            at0[3] += tb >> 16;
        }
    } else {
        // placed straight away (HBM scratch or perm: the staging list would not fit the pool; rare --
        // a tiny table or hot rows -- so piece by piece, the indices reloaded from L2, which keeps the
        // common path's registers free)
#pragma unroll 1
        for (int u = 0; u < npc; ++u) {
            const int p = pw0 + 256 * u + 4 * lane;
            int4 vu = make_int4(0, 0, 0, 0);
            if (p < N) vu = ldg<int4>(i32 + p);
            const int xv[4] = {vu.x, vu.y, vu.z, vu.w};
            uint32_t rv[4], cd[4];
            int cq[kWaveParts] = {0, 0, 0, 0};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t x = (uint32_t)(xv[e] - base);
                cd[e] = (mbits >> (4 * u + e)) & 1ull ? (x & pmask) - (uint32_t)q0 : 4u;
                rv[e] = x >> vs;
#pragma unroll
                for (int q = 0; q < kWaveParts; ++q) cq[q] += cd[e] == (uint32_t)q ? 1 : 0;
            }
            const int a = cq[0] | (cq[1] << 16), b = cq[2] | (cq[3] << 16);
            const int ia = wave_incl_scan(a), ib = wave_incl_scan(b);
            const int ta = lane63(ia), tb = lane63(ib);
            int at[kWaveParts] = {at0[0] + ((ia - a) & 0xffff), at0[1] + ((ia - a) >> 16),
                                  at0[2] + ((ib - b) & 0xffff), at0[3] + ((ib - b) >> 16)};
            at0[0] += ta & 0xffff;
            at0[1] += ta >> 16;
            at0[2] += tb & 0xffff;
            at0[3] += tb >> 16;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (cd[e] >= (uint32_t)kWaveParts) continue;
                const int q = (int)cd[e];
                int dst = 0, nq = 0, to = 0;
#pragma unroll
                for (int x = 0; x < kWaveParts; ++x)
                    if (q == x) {
                        dst = at[x]++;
                        nq = n_of[x];
                        to = toff[x];
                    }
                const int32_t pos = p + e;
                const int64_t vo = (int64_t)t * ix.cap + to + dst;
                if (direct) {  // the part's perm entry and the position's once-hit flag, now
                    ix.perm[vo] = pos;
                    ix.single[(int64_t)t * ix.cap + pos] = nq == 1 ? 1 : 0;
                    if (dst < 8) {  // (the part's first positions: its chunk record carries 5 inline)
                        sl.K[0][8 * q + dst] = rv[e];
                        sl.V[0][8 * q + dst] = pos;
                    }
                } else {
                    ix.wscratch[vo] = rv[e];
                    ((int32_t*)ix.wscratch)[ix.wstride + vo] = pos;
                }
            }
        }
    }
    if (G) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (G) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (w >= kWaveParts) return;  // (NW > 4: the extra waves only scanned; the sort has no barrier)
    WPH(7);
    wave_build_sort(ix, g, T, t, q0, vs, nrows, n_of[w], toff[w], pbase[w], direct, G, sl);
}

}  // namespace dlrm
