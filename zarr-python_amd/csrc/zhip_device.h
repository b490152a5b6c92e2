// Device helpers shared by the decode and encode kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/zarrhip.h"
#include "zhip_gf2.h"
#include "zhip_internal.h"

namespace zhip {

__device__ __forceinline__ uint32_t bswap_item(uint32_t x, int item) {
    if (item == 2) return ((x & 0x00FF00FFu) << 8) | ((x >> 8) & 0x00FF00FFu);
    if (item == 4) return __builtin_bswap32(x);
    return x;
}

template <int ITEM, bool SWAP>
__device__ __forceinline__ uint4 swap_block(uint4 v) {
    if constexpr (!SWAP || ITEM == 1) {
        return v;
    } else if constexpr (ITEM == 8) {
        return make_uint4(__builtin_bswap32(v.y), __builtin_bswap32(v.x), __builtin_bswap32(v.w),
                          __builtin_bswap32(v.z));
    } else {
        return make_uint4(bswap_item(v.x, ITEM), bswap_item(v.y, ITEM), bswap_item(v.z, ITEM),
                          bswap_item(v.w, ITEM));
    }
}

// Load the 16 chunk bytes [o, o+16) (o a multiple of 16, chunk-relative), zero
// outside [0, n).  AL4: `cp` is 4-byte aligned -> one dwordx4 load; otherwise
// five aligned dwords are funnel-shifted.
__device__ __forceinline__ uint4 mask_tail(uint4 v, int32_t o, uint32_t n) {
    const uint32_t valid = n - (uint32_t)o;
    if (valid < 16u) {
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int32_t keep = (int32_t)valid - 4 * i;
            if (keep <= 0) w[i] = 0;
            else if (keep < 4) w[i] &= (1u << (8 * keep)) - 1u;
        }
        v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    return v;
}

template <bool AL4>
__device__ __forceinline__ uint4 load_block(const uint8_t* cp, int32_t o, uint32_t n) {
    if (o < 0 || (uint32_t)o >= n) return make_uint4(0, 0, 0, 0);
    uint4 v;
    if constexpr (AL4) {
        v = *reinterpret_cast<const uint4*>(cp + o);
    } else {
        const uintptr_t a = reinterpret_cast<uintptr_t>(cp + o);
        const uint32_t* b = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
        const uint32_t sh = (uint32_t)(a & 3u) * 8u;
        const uint4 lo = *reinterpret_cast<const uint4*>(b);
        const uint32_t hi = b[4];
        v.x = (uint32_t)((((uint64_t)lo.y << 32) | lo.x) >> sh);
        v.y = (uint32_t)((((uint64_t)lo.z << 32) | lo.y) >> sh);
        v.z = (uint32_t)((((uint64_t)lo.w << 32) | lo.z) >> sh);
        v.w = (uint32_t)((((uint64_t)hi << 32) | lo.w) >> sh);
    }
    return mask_tail(v, o, n);
}

typedef unsigned int zhip_v4u __attribute__((ext_vector_type(4)));

// Cache policy of the streaming 16-byte loads of every kernel.  Default
// policy: measured 9-13 % faster than nontemporal loads on the headline, up to
// 50 % on C1, 14-18 % on the encodes (profiles/r02/load_policy_ab.jsonl);
// nontemporal stays a build-time measurement switch (EXTRA=-DZHIP_NT_LOADS=1).
#ifndef ZHIP_NT_LOADS
#define ZHIP_NT_LOADS 0
#endif
constexpr bool kNtLoads = ZHIP_NT_LOADS != 0;

// Streaming 16-byte load / store: the decode touches every encoded and
// decoded byte exactly once (stores nontemporal; loads per kNtLoads).
__device__ __forceinline__ uint4 load_stream16(const uint8_t* p) {
    zhip_v4u w;
    if constexpr (kNtLoads) w = __builtin_nontemporal_load(reinterpret_cast<const zhip_v4u*>(p));
    else w = *reinterpret_cast<const zhip_v4u*>(p);
    return make_uint4(w.x, w.y, w.z, w.w);
}

__device__ __forceinline__ void store_nt16(uint8_t* p, uint4 v) {
    zhip_v4u w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<zhip_v4u*>(p));
}

template <bool AL4, bool NT>
__device__ __forceinline__ uint4 load_block_t(const uint8_t* cp, int32_t o, uint32_t n) {
    if constexpr (AL4 && NT) {
        if (o < 0 || (uint32_t)o >= n) return make_uint4(0, 0, 0, 0);
        return mask_tail(load_stream16(cp + o), o, n);
    } else {
        return load_block<AL4>(cp, o, n);
    }
}

// XOR of v over the wave's 64 lanes, returned wave-uniform.  Four DPP steps
// leave every lane holding its 16-lane row's total (quad_perm [1,0,3,2],
// quad_perm [2,3,0,1], row_half_mirror, row_mirror); the four row totals are
// then read into scalar registers.  No LDS round trips (a __shfl_xor ladder
// is six dependent ds_bpermute's).  Every lane of the wave must be active.
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, true);
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, true);
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, true);
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, true);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 16) ^
           (uint32_t)__builtin_amdgcn_readlane((int)v, 32) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

__device__ __forceinline__ uint32_t tab_apply(const uint32_t* tab, uint32_t w) {
    return tab[w & 255u] ^ tab[256 + ((w >> 8) & 255u)] ^ tab[512 + ((w >> 16) & 255u)] ^
           tab[768 + (w >> 24)];
}

__device__ __forceinline__ uint64_t load_u64_le_bytes(const uint8_t* p) {
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

// Output byte offset of selected stored-dims coordinates; `rem` is the
// (flattened, C-order) index over dims [0, last] where `last` = ndim-1 for an
// element index or ndim-2 for a row index.  Returns false if not selected.
__device__ __forceinline__ bool sel_offset(const Geom& g, const zhip_sel& s, uint32_t rem, int last,
                                           int64_t& dst) {
    bool ok = true;
#pragma unroll
    for (int d = ZHIP_MAX_DIMS - 1; d >= 0; --d) {
        if (d > last) continue;
        uint32_t q = d > 0 ? fdiv_apply(rem, g.dshape[d].m, g.dshape[d].s) : 0u;
        const int32_t sd = (int32_t)(rem - q * (uint32_t)g.shape[d]);
        if (d == 0) { /* rem < shape[0] for in-range indices */
            q = 0;
        }
        rem = q;
        const int32_t rel = sd - s.start[d];
        const uint32_t kq = fdiv_apply((uint32_t)max(rel, 0), s.div_step[d].m, s.div_step[d].s);
        ok = ok && rel >= 0 && (int32_t)(kq * (uint32_t)s.step[d]) == rel && (int32_t)kq < s.count[d];
        dst += (int64_t)kq * g.ostride[d];
    }
    return ok;
}

template <int ITEM, bool SWAP>
__device__ __forceinline__ void store_item(uint8_t* dst, uint32_t lo, uint32_t hi) {
    if constexpr (ITEM == 1) {
        *dst = (uint8_t)lo;
    } else if constexpr (ITEM == 2) {
        uint16_t v = (uint16_t)lo;
        if constexpr (SWAP) v = (uint16_t)((v >> 8) | (v << 8));
        *reinterpret_cast<uint16_t*>(dst) = v;
    } else if constexpr (ITEM == 4) {
        *reinterpret_cast<uint32_t*>(dst) = SWAP ? __builtin_bswap32(lo) : lo;
    } else {
        uint2 v = SWAP ? make_uint2(__builtin_bswap32(hi), __builtin_bswap32(lo)) : make_uint2(lo, hi);
        *reinterpret_cast<uint2*>(dst) = v;
    }
}

// Scatter one 16-byte block (chunk bytes [o, o+16), whole items) element by element.
template <int ITEM, bool SWAP>
__device__ __forceinline__ void scatter_block_generic(const Geom& g, uint8_t* out, const zhip_sel& s,
                                                      int64_t out_off, int32_t o, uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    constexpr int kItems = 16 / ITEM;
    const uint32_t e0 = (uint32_t)o / ITEM;
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        if ((uint32_t)o + (uint32_t)(j * ITEM) >= g.nbytes) break;
        int64_t dst = out_off;
        if (!sel_offset(g, s, e0 + j, g.ndim - 1, dst)) continue;
        uint32_t lo, hi = 0;
        if constexpr (ITEM == 8) {
            lo = w[2 * j];
            hi = w[2 * j + 1];
        } else {
            lo = (w[(j * ITEM) / 4] >> (8 * ((j * ITEM) % 4))) & (ITEM == 4 ? 0xFFFFFFFFu : ((1u << (8 * ITEM)) - 1u));
        }
        store_item<ITEM, SWAP>(out + dst, lo, hi);
    }
}

// Whole-row fast path: rows of the innermost stored dim are fully selected,
// contiguous in out and a multiple of 16 bytes, out rows 16-byte aligned.
template <int ITEM, bool SWAP, bool NT = false>
__device__ __forceinline__ void scatter_block_rows(const Geom& g, uint8_t* out, const zhip_sel& s,
                                                   int64_t out_off, int32_t o, uint4 v) {
    const uint32_t r = fdiv_apply((uint32_t)o, g.drow.m, g.drow.s);
    const uint32_t col = (uint32_t)o - r * g.row_bytes;
    int64_t dst = out_off + col;
    if (!sel_offset(g, s, r, g.ndim - 2, dst)) return;
    if constexpr (NT) store_nt16(out + dst, swap_block<ITEM, SWAP>(v));
    else *reinterpret_cast<uint4*>(out + dst) = swap_block<ITEM, SWAP>(v);
}


}  // namespace zhip
