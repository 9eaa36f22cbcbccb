// bitonic.hpp — one wave sorts up to 64·R keys held in its registers (gfx950).
//
// The wave build (indexer.hpp) groups a table part's ~128 positions by row.  Its LDS counting
// sort runs a chain of LDS atomics, scans and placements whose length depends on the keys: a
// part whose low-digit buckets are skewed (Zipf rows, hot rows) falls back to stable LSD passes,
// several times as long.  A bitonic network does the same compare-exchanges whatever the keys:
// log2(n)·(log2(n)+1)/2 steps, each one lane exchange and a min / max per register, with no LDS
// and no branch on the data.  Element i of the sequence lives in register i / 64 of lane i % 64.
// Lane exchanges (partner lane ^ j) by the cheapest gfx950 form for each distance:
//   j = 1, 2   DPP quad_perm                  (one VALU op)
//   j = 4      DPP row_shl:4 / row_shr:4      (two VALU ops + select)
//   j = 8      DPP row_ror:8                  (one VALU op)
//   j = 16     v_permlane16_swap              (one op, both halves of each row pair)
//   j = 32     v_permlane32_swap
//   j >= 64    another register of the same lane (no exchange)
// Keys are distinct (the caller packs the position into the low bits), so the result is the
// unique sorted order -- deterministic, and "stable" on the row part of the key.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dlrm {

// The value lane ^ J holds (J < 64, uniform), for every lane.
template <int J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t x) {
    static_assert(J == 1 || J == 2 || J == 4 || J == 8 || J == 16 || J == 32, "lane distance");
    const int lane = threadIdx.x & 63;
    if constexpr (J == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
    } else if constexpr (J == 2) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
    } else if constexpr (J == 4) {
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x104, 0xf, 0xf, false);  // row_shl:4
        const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
        return (lane & 4) ? dn : up;
    } else if constexpr (J == 8) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xf, 0xf, false);  // row_ror:8
    } else if constexpr (J == 16) {
        // (x, x) -> first: odd rows replaced by the even rows below them; second: even rows by the
        // odd rows above them
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (lane & 16) ? r[0] : r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (lane & 32) ? r[0] : r[1];
    }
}

template <int J>
__device__ __forceinline__ uint64_t xor_lane(uint64_t x) {
    return (uint64_t)xor_lane<J>((uint32_t)x) | ((uint64_t)xor_lane<J>((uint32_t)(x >> 32)) << 32);
}

// One step (K, J) of the network over R registers: element i = 64 r + lane pairs with i ^ J; the
// lower of the two keeps the min when its block of K elements ascends ((i & K) == 0).
template <int R, int K, int J, typename V>
__device__ __forceinline__ void bitonic_step(V (&a)[R]) {
    const int lane = threadIdx.x & 63;
    if constexpr (J >= 64) {
        constexpr int JR = J / 64;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if ((r & JR) != 0) continue;
            const bool up = ((r * 64) & K) == 0;  // (K >= 128 here: uniform per register)
            const V lo = a[r] < a[r | JR] ? a[r] : a[r | JR];
            const V hi = a[r] < a[r | JR] ? a[r | JR] : a[r];
            a[r] = up ? lo : hi;
            a[r | JR] = up ? hi : lo;
        }
    } else {
        const bool lower = (lane & J) == 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const V p = xor_lane<J>(a[r]);
            const bool up = ((r * 64 + lane) & K) == 0;
            const V mn = a[r] < p ? a[r] : p;
            const V mx = a[r] < p ? p : a[r];
            a[r] = (lower == up) ? mn : mx;
        }
    }
}

template <int R, int K, int J, typename V>
__device__ __forceinline__ void bitonic_merge(V (&a)[R]) {
    bitonic_step<R, K, J>(a);
    if constexpr (J > 1) bitonic_merge<R, K, J / 2>(a);
}

template <int R, int K, typename V>
__device__ __forceinline__ void bitonic_stages(V (&a)[R]) {
    bitonic_merge<R, K, K / 2>(a);
    if constexpr (K < 64 * R) bitonic_stages<R, 2 * K>(a);
}

// Sorts the 64·R keys of the wave ascending: afterwards register r of lane l holds the
// (64 r + l)-th smallest.  Fully unrolled (measured, 416 waves alone on the chip, 32-bit keys:
// 0.23 / 0.55 / 1.3 us for R = 1 / 2 / 4; a form with run-time stage loops, one copy of each step,
// took 4.2 us at R = 2).  The caller must inline it: an outlined call puts the whole launch on
// scratch (round 6: the apply launch with the build's sort outlined ran 2x longer).  Every lane
// of the wave must call it (uniform control flow).
template <int R, typename V>
__device__ __forceinline__ void wave_bitonic_sort(V (&a)[R]) {
    static_assert(R == 1 || R == 2 || R == 4 || R == 8, "64, 128, 256 or 512 keys");
    bitonic_stages<R, 2>(a);
}

}  // namespace dlrm
