// indexer.hpp — the in-LDS SparseIndexer build (one workgroup per table, N <= 4096 positions),
// shared by the standalone indexer launch (update.hip) and the backward launch that builds the
// indexer in the same grid (interact.hip).  See update.hip for the apply that consumes it.
#pragma once
#include "common.hpp"

#ifndef PHASE
#define PHASE(k) do {} while (0)
#endif

namespace dlrm {

constexpr int kChunk = 32;          // max positions of a segment handled by one lane group
constexpr int kRankBucketMax = 64;  // within-bucket rank sort when every bucket is this small
enum { CNT_U = 0, CNT_C = 1, CNT_H = 2, CNT_S = 3, CNT_NV = 4 };
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
// Flat id -> (table, offset) over per-table counts, T tables in tiles of 64 lanes.  Every lane
// may carry its own id; shuffles run in uniform control flow.  table = -1 when id >= total.
__device__ __forceinline__ int wave_incl_scan(int x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    return x;
}

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
constexpr int kScanTiles = 4;
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
        r.total = __shfl(r.incl, 63, 64);
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


}  // namespace dlrm
