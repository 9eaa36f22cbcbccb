// common.hpp — shared device helpers for the gfx950 DLRM hot-path kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dlrm_hip.h"

namespace dlrm {

constexpr int kWave = 64;  // CDNA wavefront

// Device-side descriptor of one embedding table (SimpleEmbedding{Static{D}}.data).
struct __attribute__((aligned(16))) TableDesc {
    void* data;     // [nrows][dim] row-major, f32 or bf16
    int64_t nrows;
};

// Up to kArgTables table pointers travel by value in a forward kernel's arguments (TabPtrs).
constexpr int kArgTables = 32;

// Device-side error word: bit 0 = an out-of-range index was skipped.
constexpr unsigned kErrIndex = 1u;

// The ctx's error word is 16 bytes: [0] the flag, [2..3] the device address of a host-memory copy
// of it (dlrm_ctx_create).  One thread of a step backward (the launch after the forward that raises
// the flag) stores the flag there, so the host reads it without a GPU call (dlrm_error_peek).
__device__ __forceinline__ void snapshot_error(const unsigned* err, unsigned v) {
    unsigned* h = *reinterpret_cast<unsigned* const*>(err + 2);
    if (h) __hip_atomic_store(h, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void raise_index_error(unsigned* err) {
    __hip_atomic_fetch_or(err, kErrIndex, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Orders one wave's LDS writes before its later LDS reads by other lanes.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// Round-to-nearest-even; NaN stays NaN (MI355X_MICROARCH.md, correctness boundaries).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (uint16_t)((u >> 16) | 0x40);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// Global-address-space accesses.  Pointers that come out of memory (TableDesc::data, kernel
// argument structs) are generic to the compiler, which then emits flat_* instructions: those
// count against both vmcnt and lgkmcnt, so every wait for one of them also drains LDS traffic.
// Casting to address space 1 gives global_* instructions.
#define DLRM_GLOBAL __attribute__((address_space(1)))
#if defined(__HIP_DEVICE_COMPILE__)
template <typename V> __device__ __forceinline__ V ldg(const void* p) { return *(const DLRM_GLOBAL V*)p; }
template <typename V> __device__ __forceinline__ void stg(void* p, const V& v) { *(DLRM_GLOBAL V*)p = v; }
// Non-temporal store (global_store ... nt): streamed toward memory instead of parked dirty in
// the XCD's L2, so it drains during the kernel rather than in the end-of-kernel L2 write-back
// (tools/bwd_probe.hip: the step backward's dt rows + once-hit rows, 14.5 -> 13.0 us).
template <typename V> __device__ __forceinline__ void stg_nt(void* p, const V& v) {
    __builtin_nontemporal_store(v, (DLRM_GLOBAL V*)p);
}
#else  // host pass of the device code: never executed
template <typename V> __device__ __forceinline__ V ldg(const void* p) { return *(const V*)p; }
template <typename V> __device__ __forceinline__ void stg(void* p, const V& v) { *(V*)p = v; }
template <typename V> __device__ __forceinline__ void stg_nt(void* p, const V& v) { *(V*)p = v; }
#endif

// n / d for 0 <= n < 2^31 and d >= 1 by a multiply-high, an add and a shift (the round-up magic:
// m = floor(2^32 (2^l - d) / d) + 1, l = ceil(log2 d); exact over that range), set up once per
// kernel: the apply's position -> bag (sample) for every grad row it reads, where the compiler's
// division by a run-time L costs ~15 VALU per row.
struct FastDiv {
    uint32_t m;
    int l;
    __device__ __forceinline__ explicit FastDiv(int d) {
        if (d <= 1) {  // (one-hot: no 64-bit division at the kernel's start)
            m = 1u;
            l = 0;
            return;
        }
        l = 32 - __clz(d - 1);
        m = (uint32_t)((((unsigned long long)1 << 32) * (((unsigned long long)1 << l) - (unsigned)d)) / (unsigned)d + 1);
    }
    __device__ __forceinline__ int operator()(int n) const {
        return (int)((__umulhi(m, (uint32_t)n) + (uint32_t)n) >> l);
    }
};

// Index i of an int32 / int64 index array, without a branch on the type: a branch per load
// makes the compiler wait for each load at the join, serialising a lane's index loads.
// (int32: the second word read is the first one again.)
__device__ __forceinline__ int64_t load_index(const void* idx, int itype, int64_t i) {
    const uint32_t* p = (const uint32_t*)idx + (i << itype);
    const uint32_t lo = ldg<uint32_t>(p), hi = ldg<uint32_t>(p + itype);
    return itype ? (int64_t)(((uint64_t)hi << 32) | lo) : (int64_t)(int32_t)lo;
}

// One 16-B load (the compiler would otherwise sink the nrows half into the branch that tests it).
__device__ __forceinline__ TableDesc load_table(const TableDesc* tabs, int t) {
    const uint4 v = ldg<uint4>(tabs + t);
    TableDesc d;
    d.data = (void*)(((uint64_t)v.y << 32) | v.x);
    d.nrows = (int64_t)(((uint64_t)v.w << 32) | v.z);
    return d;
}

// load_index where the position may be invalid: the load always executes (at position 0) and
// the result is masked, so no branch surrounds it.
__device__ __forceinline__ int64_t load_index_if(bool ok, const void* idx, int itype, int64_t i) {
    const int64_t v = load_index(idx, itype, ok ? i : 0);
    return ok ? v : 0;
}

// 16-byte vector types
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

// Element traits: storage type -> 16-byte vector of it, element count per vector.
template <typename T> struct Vec;
template <> struct Vec<float> {
    static constexpr int N = 4;
    typedef f32x4 type;
    __device__ static inline void to_f32(const type& v, float* o) { o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = v[3]; }
    __device__ static inline type from_f32(const float* o) { type v; v[0] = o[0]; v[1] = o[1]; v[2] = o[2]; v[3] = o[3]; return v; }
};
template <> struct Vec<uint16_t> {
    static constexpr int N = 8;
    typedef u16x8 type;
    __device__ static inline void to_f32(const type& v, float* o) {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = bf16_to_f32(v[i]);
    }
    __device__ static inline type from_f32(const float* o) {
        type v;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = f32_to_bf16(o[i]);
        return v;
    }
};

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(uint16_t v) { return bf16_to_f32(v); }
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ uint16_t from_f32<uint16_t>(float v) { return f32_to_bf16(v); }

// NE consecutive elements of a row as fp32 (16-B vector accesses where the size allows).
template <typename TT, int NE>
__device__ __forceinline__ void load_row(const TT* row, int c0, float* f) {
    constexpr int BYTES = (int)sizeof(TT) * NE;
    if constexpr (BYTES % 16 == 0) {
        typedef Vec<TT> V;
#pragma unroll
        for (int k = 0; k < BYTES / 16; ++k) V::to_f32(ldg<typename V::type>((const typename V::type*)(row + c0) + k), f + k * V::N);
    } else {
#pragma unroll
        for (int e = 0; e < NE; ++e) f[e] = to_f32(ldg<TT>(row + c0 + e));
    }
}

template <typename TT, int NE, bool NT = false>
__device__ __forceinline__ void store_row(TT* row, int c0, const float* f) {
    constexpr int BYTES = (int)sizeof(TT) * NE;
    if constexpr (BYTES % 16 == 0) {
        typedef Vec<TT> V;
#pragma unroll
        for (int k = 0; k < BYTES / 16; ++k) {
            if constexpr (NT) stg_nt<typename V::type>((typename V::type*)(row + c0) + k, V::from_f32(f + k * V::N));
            else stg<typename V::type>((typename V::type*)(row + c0) + k, V::from_f32(f + k * V::N));
        }
    } else if constexpr (NT && NE == 4 && sizeof(TT) == 2) {  // 4 bf16 = one 8-B store
        typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
        u32x2_t u;
        u[0] = (uint32_t)from_f32<TT>(f[0]) | ((uint32_t)from_f32<TT>(f[1]) << 16);
        u[1] = (uint32_t)from_f32<TT>(f[2]) | ((uint32_t)from_f32<TT>(f[3]) << 16);
        stg_nt<u32x2_t>(row + c0, u);
    } else {
#pragma unroll
        for (int e = 0; e < NE; ++e) stg<TT>(row + c0 + e, from_f32<TT>(f[e]));
    }
}

// The descriptors of up to kArgTables tables by value, as a kernel argument (the one-hot forward,
// the lookup): a lane's row address then waits on its index load alone, and the pointer is read
// with the kernel-argument base in SGPRs (tools/fwd_probe.hip bisect: 12.0 -> 10.9 us).
struct TabPtrs {
    const void* p[kArgTables];
    uint32_t n[kArgTables];  // rows (every table here has < 2^32)
};
inline bool fill_tab_ptrs(TabPtrs& tp, const TableDesc* host, int T) {
    if (!host || T <= 0 || T > kArgTables) return false;
    for (int t = 0; t < T; ++t) {
        if (host[t].nrows >= (int64_t)UINT32_MAX) return false;
        tp.p[t] = host[t].data;
        tp.n[t] = (uint32_t)host[t].nrows;
    }
    for (int t = T; t < kArgTables; ++t) { tp.p[t] = nullptr; tp.n[t] = 0; }
    return true;
}

// A zero row: the source of padding rows (16NB > F) and of rows whose index is out of range, so
// that every row load of the one-hot forward and of the lookup is an unconditional, unmasked load.
constexpr int kZeroElems = 1024;  // fp32 elements (4 KB); column offsets wrap modulo this
static __device__ __attribute__((aligned(16))) float g_zero_row[kZeroElems];

}  // namespace dlrm

namespace dlrm {
// Per-table indexer arrays (device), each [T][cap] (seg_start [T][cap+1]).
// Output row addressing of a lookup: row b of table t lands at
//   (b / brows) * bstride + (b % brows) * ld + off + t * tstride
// (plain [B][ld] rows: tstride = D, brows >= B; the sharded send layout [peer][table][b][D]:
// ld = D, tstride = B_local * D, brows = B_local, bstride = T_r * B_local * D).
struct OutMap {
    int64_t ld, off, tstride, brows, bstride;
    __device__ __forceinline__ int64_t row(int64_t b) const {
        const int64_t q = b / brows;
        return q * bstride + (b - q * brows) * ld + off;
    }
};

constexpr int kFastMaxN = 4096;     // in-LDS indexer (indexer.hpp): positions per table
constexpr int kHixMaxN = 1 << 20;   // hash indexer (hashindex.hip): positions per table
constexpr int kStepIndexMaxN = 2048;  // the forward-launch indexer (interact.hip): positions per table
constexpr int kStepMaxParts = 16;     // ... which sorts a table as up to 16 parts (by the row's low bits)
// the wave build (indexer.hpp wave_build_group) of the next batch (in the apply launch) or of a
// prepared batch (dlrm_indexer_prepare, and dlrm_indexer_build's pooled bags): up to kWaveMaxN
// positions per table, as 16 parts per 2048 positions (2^wave_vshift(N) parts per table; a part
// averages <= 128 positions).  The in-apply build (dlrm_step_bwd_prepare) takes up to
// kWaveApplyMaxN (its scan build keeps a quarter of the table's indices in registers).
constexpr int kWaveMaxN = 32768;
constexpr int kWaveApplyMaxN = 16384;
constexpr int kWaveMaxVshift = 8;
__host__ __device__ constexpr int wave_vshift(int64_t N) {
    return N <= 2048 ? 4 : (N <= 4096 ? 5 : (N <= 8192 ? 6 : (N <= 16384 ? 7 : 8)));
}
// The wave builds' per-part arrays are packed per table (round 6, "compact" layout): part q of
// table t (virtual table v = (t << vs) + q) keeps its entries at t * cap + off_q, off_q = the
// table's positions in parts < q (IndexerDev::counts[v][CNT_OFF]); its segment starts at
// t * (cap + kSegPad) + off_q + q (one sentinel per part).  So an indexer of cap positions per table
// holds any wave build in T * cap slots, whatever the parts (the old layout gave every part a whole
// cap: 128 x the table at 16384 positions).
constexpr int kSegPad = 1 << kWaveMaxVshift;
constexpr int kCntOff = 5;  // counts[v][kCntOff]: the part's offset in its table (wave builds)
// the next batch's split build in the apply launch (indexer.hpp wave_build_group): parts per
// table, one wave each, 4 per workgroup (>= 4)
#ifndef DLRM_WAVE_PARTS
#define DLRM_WAVE_PARTS 16
#endif
constexpr int kWaveBuildParts = DLRM_WAVE_PARTS;
// split builds of kFastMaxN < N <= kPartsMaxN positions per table: the in-LDS build (1024
// threads x 8 positions) over 2^kPartsLog2 parts per table (by the row's low bits), each part's
// workgroup sized for the worst case (all N positions in one part); larger N: the hash build
constexpr int kPartsMaxN = 8192;
#ifndef DLRM_BUILD_PARTS_LOG2
#define DLRM_BUILD_PARTS_LOG2 2
#endif
constexpr int kPartsLog2 = DLRM_BUILD_PARTS_LOG2;
#ifndef DLRM_STEP_PARTS_DEFAULT
#define DLRM_STEP_PARTS_DEFAULT 4
#endif
constexpr int kStepParts = DLRM_STEP_PARTS_DEFAULT;

struct IndexerDev {
    uint32_t* keys0;  uint32_t* keys1;   // global sort scratch (cap > kLdsSortMax)
    int32_t* vals0;   int32_t* vals1;
    int32_t* perm;         // positions grouped by row, ascending within a row
    int32_t* seg_start;    // [cap+1]
    uint32_t* seg_row;
    int4* chunks;          // [2 cap] per table: segments of <= kChunk positions (indexer.hpp write_chunk)
    int4* hot;             // longer segments: {beg, end, row, first slice}
    int4* hot_slice;       // their slices of kHotSlice positions: {p0, p1, row, hot segment}
    int32_t* hot_cnt;      // arrivals per hot segment (multi-slice combine; reset by the last)
    float* partial;        // [T][pcap][pdim] slice partial sums (multi-slice hot segments)
    int32_t* counts;       // [T][8]: U, chunks, hot, slices, nvalid
    uint8_t* single;       // [T][cap]: 1 = the position's row is hit once in the batch (split builds)
    // hash indexer (hashindex.hip; capacities above the in-LDS build's kFastMaxN)
    int32_t* pslot;        // [T][cap] hash slot of each position (-1: invalid index)
    unsigned long long* hent;  // [T][hsize] row << 32 | positions, all ones = empty (reset by the alloc pass)
    int2* hseg;            // [T][hsize] {first perm entry, length} of the slot's segment
    uint32_t* hfill;       // [T][hsize] placement cursor
    unsigned long long* hstate;  // [T][4] {segments << 32 | positions} allocation cursor, ...
    int64_t hsize;         // slots per table (power of two >= 2 cap), 0 = no hash arrays
    // > 0: the build split each table's positions by the row's low vshift bits into virtual
    // tables v = (t << vshift) + (row & mask) (the forward launch's indexer: 2^vshift workgroups
    // per table); the per-table arrays above (perm ... counts, not single / pslot / hash) are then
    // indexed by v, and the apply maps v -> t.
    int vshift;
    int hbits;
    // flat item lists of the wave build (apply.hpp reads them when has_map), in 8 sub-lists (by
    // build workgroup mod 8): every build wave reserves its hot slices and chunks and arrives with
    // ONE 64-bit atomic add on its sub-list's word of build_arrive (indexer.hpp kRes*) and writes
    // them whole; a sub-list's last wave to arrive copies its totals to item_tot[j] (slices) /
    // item_tot[8 + j] (chunks) and clears the word.
    //   slice_rec[2k, 2k+1]: {first perm entry, end (global: v * cap + local), row, v},
    //                        {slices of its segment, flat index of the segment's first slice, 0, 0}
    //   chunk_rec[2c, 2c+1]: the chunk descriptor (write_chunk) with global perm entries
    int4* slice_rec;
    int4* chunk_rec;
    // the wave build's global sort scratch (cap > kStepIndexMaxN): 5 arrays (K0, V0, K1, V1, R) of
    // wstride entries, part v's region at v * cap -- for a build workgroup whose four parts overflow
    // its LDS pool (tiny tables and hot rows at large N), which then sorts in HBM instead
    uint32_t* wscratch;
    int64_t wstride;
    int32_t* item_tot;
    uint32_t* build_arrive;  // the reservation words (64 bits, 256 B apart)
    // the bounds word of a standalone prepared build (dlrm_indexer_prepare), or null: the apply of
    // this indexer folds it into the ctx's flag (its lookups raise the same errors; this covers a
    // prebuilt update without one)
    const unsigned* build_err;
    int chunk_max;         // the wave build's chunk limit (16 or 32; indexer.hpp kMinChunk .. kChunk)
    int has_map;           // 1: a wave build (flat item map, compact per-part layout)
    int64_t cap;
    int64_t pcap;          // slices per table (upper bound)
    int pdim;              // partial row capacity (elements)

    // where virtual table v's per-part entries (perm, seg_row, hot, hot_slice; chunks at twice it)
    // and its segment starts begin: packed per table after a wave build (has_map), else v * cap
    __device__ __forceinline__ int64_t part_off(int v) const {
        return has_map ? (int64_t)(v >> vshift) * cap + counts[(int64_t)v * 8 + kCntOff] : (int64_t)v * cap;
    }
    __device__ __forceinline__ int64_t seg_off(int v) const {
        return has_map ? (int64_t)(v >> vshift) * (cap + kSegPad) + counts[(int64_t)v * 8 + kCntOff] +
                             (v & ((1 << vshift) - 1))
                       : (int64_t)v * (cap + 1);
    }
};
int64_t indexer_slice_cap(int64_t cap);
constexpr int kPartialDim = 256;  // partial rows allocated with the indexer (larger D: regrown on use)

}  // namespace dlrm

// Host-side launch helpers (defined in abi.cpp) and the per-kernel launchers.
struct dlrm_ctx;
namespace dlrm {
unsigned* ctx_error_word(dlrm_ctx* ctx);
hipStream_t ctx_stream(dlrm_ctx* ctx);
int ctx_fail(dlrm_ctx* ctx, int code, const char* fmt, ...);
int ctx_hip(dlrm_ctx* ctx, hipError_t e, const char* what);
int ctx_num_cus(dlrm_ctx* ctx);
int ctx_device(dlrm_ctx* ctx);

// Comparison knobs: every environment variable the library reads, read once (abi.cpp), in this
// one place.  0 = the default (the measured-best form); a non-zero value forces a variant for
// A/B runs.  None is needed for correctness.
struct Knobs {
    int step_parts;   // DLRM_STEP_PARTS  (1/2/4/8): table parts of the step's split indexer build
    int build_parts;  // DLRM_BUILD_PARTS (2/4/8): parts of a standalone split build, 4096 < N <= 8192
    int relu_1pass;   // DLRM_RELU_2PASS=0: the one-launch (last-arriver) relu seam instead of two launches
    int bwd_ys_body;  // DLRM_BWD_YS=0: the bwd_body kernel for a materialized ys with 33..96 features
    int bwd_nosplit;  // DLRM_BWD_SPLIT=0: the one-wave step backward instead of the split kernel
    int bwd_spb;      // DLRM_BWD_SPB (2/4/8): samples per block of the split step backward
    int bwd_cpl;      // DLRM_BWD_CPL (4/8): columns per lane of the bf16 split step backward
    int upd_sbu;      // DLRM_UPD_SBU (1/2): super-blocks in flight in the one-wave step backward
    int wave_rounds;  // DLRM_WAVE_ROUNDS=1: the wave build in rounds above 2048 positions per table
                      // instead of the scan build
    int bag_hash;     // DLRM_BAG_WAVE=0: dlrm_indexer_build of 8192 < N <= 32768 positions per table (pooled
                      // bags) by the hash build instead of the bag build
    int bag_vs;       // DLRM_BAG_VS (2..8): the bag build's log2 parts per table (default wave_vshift(N))
    int bag_split;    // DLRM_BAG_SPLIT=0: dlrm_indexer_build_split of 4096 < N <= 32768 by the in-LDS parts /
                      // hash builds instead of the bag build
};
const Knobs& knobs();

int launch_maplookup(dlrm_ctx* ctx, const TableDesc* d_tabs, bool tabs_aligned16, int T, int D, int dtype,
                     const void* idx, int itype, int64_t tstride, int base, int B, int L, void* out,
                     int64_t out_ld, int64_t out_off, const TableDesc* htabs = nullptr);
int launch_interact_fwd(dlrm_ctx* ctx, int dtype, int d, int F, int B, const void* x, int64_t x_ld, void* ys,
                        int64_t ys_ld, void* out, int64_t out_ld, int padding);
int launch_lookup_interact_fwd(dlrm_ctx* ctx, const TableDesc* tabs, bool tabs_aligned16, int T, int dtype,
                               const void* idx, int itype, int64_t tstride, int base, int L, int d, int B,
                               const void* x, int64_t x_ld, void* ys, int64_t ys_ld, void* out, int64_t out_ld,
                               int padding,
    const TableDesc* htabs = nullptr);
int launch_interact_bwd_gather(dlrm_ctx* ctx, const TableDesc* tabs, bool tabs_aligned16, int T, int dtype,
                               const void* idx, int itype, int64_t tstride, int base, int L, int d, int B,
                               const void* x, int64_t x_ld, const void* dout, int64_t dout_ld, float* dx,
                               int64_t dx_ld, float* dt, int64_t dt_ld, const IndexerDev* ix,
    const TableDesc* htabs = nullptr);
int launch_interact_bwd_blocked(dlrm_ctx* ctx, const TableDesc* tabs, bool tabs_aligned16, int T, int dtype,
                                const void* idx, int itype, int64_t tstride, int base, int L, int d, int B,
                                const void* x, int64_t x_ld, const void* dout, int64_t dout_ld, float* dx,
                                int64_t dx_ld, float* dst, const int64_t* dbase, const int64_t* dld,
    const TableDesc* htabs = nullptr);
int launch_step_fwd(dlrm_ctx* ctx, const TableDesc* tabs, bool tabs_aligned16, int T, int dtype, const void* idx,
                    int itype, int64_t tstride, int base, int d, int B, const void* x, int64_t x_ld, void* out,
                    int64_t out_ld, int padding, const IndexerDev& ix,
    const TableDesc* htabs = nullptr);
int launch_step_bwd(dlrm_ctx* ctx, const TableDesc* tabs, int T, int dtype, const void* idx, int itype,
                    int64_t tstride, int base, int d, int B, const void* x, int64_t x_ld, const void* dout,
                    int64_t dout_ld, float* dx, int64_t dx_ld, float* dt, int64_t dt_ld, const IndexerDev& ix,
                    float lr,
    const TableDesc* htabs = nullptr);
int launch_interact_bwd(dlrm_ctx* ctx, int dtype, int d, int F, int B, const void* dout, int64_t dout_ld,
                        const void* t, int64_t t_ld, float* dx, int64_t dx_ld, float* dt, int64_t dt_ld);
int64_t hix_table_slots(int64_t cap);
int launch_hix_build(dlrm_ctx* ctx, const IndexerDev& ix, const TableDesc* tabs, int T, const void* idx, int itype,
                     int64_t tstride, int base, int N, bool split, hipStream_t stream = nullptr);
bool step_split_supported(bool tabs_aligned16, int T, int dtype, int d, const void* x, int64_t x_ld);
int launch_maplookup_map(dlrm_ctx* ctx, const TableDesc* d_tabs, bool tabs_aligned16, int T, int D, int dtype,
                         const void* idx, int itype, int64_t tstride, int base, int B, int L, void* out,
                         const OutMap& om, const TableDesc* htabs = nullptr);
int launch_dac_decode(dlrm_ctx* ctx, const void* rec, int B, float* labels, float* dense, int64_t dense_ld,
                      void* sparse, int itype, int64_t tstride);
int launch_bce_head(dlrm_ctx* ctx, int B, const float* z, int64_t z_ld, const float* y, float* prob, float* dz,
                    float* loss, float* dbias);
int64_t relu_bwd_chunks(int B);
int64_t relu_bwd_groups(int N);
int launch_relu_bwd_bias(dlrm_ctx* ctx, int B, int N, const float* y, int64_t y_ld, float* g, int64_t g_ld, float* gb,
                         float* part, unsigned* counters);
int launch_scatter_rows(dlrm_ctx* ctx, int esize, int T, int B, int D, const void* src, int64_t src_ld,
                        int64_t src_off, void* dst, const int64_t* dbase, const int64_t* dld, bool vec_ok);
int launch_indexer_build(dlrm_ctx* ctx, const IndexerDev& ix, const TableDesc* tabs, int T, const void* idx,
                         int itype, int64_t tstride, int base, int B, int L, bool split = false,
                         hipStream_t stream = nullptr);
int launch_bag_build(dlrm_ctx* ctx, const IndexerDev& ix, const TableDesc* tabs, int T, const void* idx, int itype,
                     int64_t tstride, int base, int N, unsigned* err);
int launch_step_prepare(dlrm_ctx* ctx, const IndexerDev& ix, const TableDesc* tabs, int T, const void* idx, int itype,
                        int64_t tstride, int base, int N, unsigned* err);
struct SinglesArgs;
struct PrepArgs;
int launch_sgd_apply(dlrm_ctx* ctx, const IndexerDev& ix, TableDesc* tabs, bool tabs_aligned16, int T, int D,
                     int tdtype, int L, int64_t N, const void* grad, int gdtype, int64_t grad_ld, int64_t grad_offset,
                     float lr, const SinglesArgs& singles, const PrepArgs* prep = nullptr);
int launch_triangular_slice(dlrm_ctx* ctx, int dtype, int sz, int B, const void* z, int64_t z_bs, void* out,
                            int64_t out_ld);
int launch_triangular_slice_back(dlrm_ctx* ctx, int dtype, int sz, int B, const void* dy, int64_t dy_ld, void* a,
                                 int64_t a_bs, int sym);
int launch_self_batched_mul(dlrm_ctx* ctx, int dtype, int d, int F, int B, const void* t, int64_t t_ld, void* z,
                            int64_t z_bs);
int launch_self_batched_mul_back(dlrm_ctx* ctx, int dtype, int d, int F, int B, const void* t, int64_t t_ld,
                                 const void* dz, int64_t dz_bs, float* dt, int64_t dt_ld);
int launch_sgd_atomic(dlrm_ctx* ctx, TableDesc* tabs, int T, int D, const void* idx, int itype, int64_t tstride,
                      int base, int B, int L, const void* grad, int gdtype, int64_t grad_ld, int64_t grad_offset,
                      float lr);
}  // namespace dlrm
