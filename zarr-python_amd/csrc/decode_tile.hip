// k_decode_tile4: decode of transposed chunks (a stored dim other than the
// innermost is contiguous in out: TransposeCodec, src/zarr/codecs/transpose.py:
// 89-118), four 64-row x 256-byte LDS tiles per workgroup.
//
// Same structure as k_decode_pair (decode_rows.hip): non-persistent, every
// vector load of the workgroup issued first (4 tiles x 4 blocks per thread,
// one static count on every path), headers and trailer through the scalar
// cache, and one CRC run end per workgroup.  Per tile the data goes registers
// -> LDS (stored order) -> registers (out order) -> 16-byte stores, then the
// tile's Horner steps (while the stores drain).  The CRC state of
// a thread carries from tile to tile through one table multiply (the four
// tiles sit at a uniform base step), and the lane / tile / chunk-end shifts
// are one host-built per-lane constant (kq4) applied once.
//
// Eligible plans (zhip_plan.tile4): full tiles (shape[tq] % 64 == 0,
// row_bytes % 256 == 0), t_per_chunk % 4 == 0, groups of four consecutive
// tiles at one base step; the launch covers whole chunks with a full
// selection (planner _tile_ok).  Others take the persistent k_decode_tile.

#include <hip/hip_runtime.h>

#include "../../include/zarrhip.h"
#include "zhip_gf2.h"
#include "zhip_internal.h"
#include "zhip_device.h"
#include "zhip_decode_common.h"

namespace zhip {
namespace {

constexpr int kTiles = 4;                   // tiles per workgroup
constexpr int kPasses = kTileRows / 16;     // 16-byte blocks per thread per tile

__device__ uint4 g_tile_zero[1];            // dummy-load target (never written)
__device__ uint4 g_tile_sink[kThreads];     // dummy-store target

typedef unsigned int zhip_v4u_a1t __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) const zhip_v4u_a1t zhip_gv4u_a1t;

__device__ __forceinline__ uint4 load_stream16_a1(const uint8_t* a) {  // any alignment, one dwordx4 (kNtLoads)
    zhip_v4u_a1t w;
    if constexpr (kNtLoads) w = __builtin_nontemporal_load((zhip_gv4u_a1t*)(reinterpret_cast<uintptr_t>(a)));
    else w = *(zhip_gv4u_a1t*)(reinterpret_cast<uintptr_t>(a));
    return make_uint4(w.x, w.y, w.z, w.w);
}

typedef __attribute__((address_space(1))) zhip_v4u_a1t zhip_gv4u_a1tw;

__device__ __forceinline__ void store_nt16_a1(uint8_t* a, uint4 v) {  // any alignment, one dwordx4 nt
    zhip_v4u_a1t w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, (zhip_gv4u_a1tw*)(reinterpret_cast<uintptr_t>(a)));
}

// NDBuffer.all_equal against the fill (buffer/core.py:534-558): bitwise, except
// that any NaN equals a NaN fill; 16 native-order bytes.
template <int ITEM>
__device__ __forceinline__ bool block_eq_fill_e(uint4 v, const EncodeParams& p) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    bool all = true;
#pragma unroll
    for (int j = 0; j < 16 / ITEM; ++j) {
        if constexpr (ITEM == 8) {
            const uint64_t x = ((uint64_t)w[2 * j + 1] << 32) | w[2 * j];
            const bool e = w[2 * j] == p.fill[0] && w[2 * j + 1] == p.fill[1];
            all = all && (e || (p.fill_nan && (x & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull));
        } else {
            constexpr uint32_t m = ITEM == 4 ? 0xFFFFFFFFu : ((1u << (8 * ITEM)) - 1u);
            const uint32_t x = (w[(j * ITEM) / 4] >> (8 * ((j * ITEM) % 4))) & m;
            bool e = x == (p.fill[0] & m);
            if constexpr (ITEM == 4) e = e || (p.fill_nan && (x & 0x7FFFFFFFu) > 0x7F800000u);
            if constexpr (ITEM == 2) e = e || (p.fill_nan && (x & 0x7FFFu) > 0x7C00u);
            all = all && e;
        }
    }
    return all;
}

struct TileMap4 {
    TileEnt e[kTiles];
};

// The 64-row x 256-byte LDS tile image, XOR-swizzled instead of padded: dword
// d of row r sits at dword r*64 + (d ^ tile_swz(r)), tile_swz(r) = 2*(r / kPer)
// (kPer = 16 / ITEM rows per 16-byte out piece).  The column accesses (each
// lane kPer rows of one element column; a half wave covers 64/kPer pieces of
// two adjacent columns) then hit 32 distinct banks -- the 260-byte pitch left
// them 2-way conflicted -- and a thread's 16-byte row block stays one
// aligned 16-byte slot (one ds_write_b128 / ds_read_b128, its dword pairs
// swapped when bit 1 of the swizzle is set).
template <int ITEM>
__device__ __forceinline__ uint32_t tile_swz(uint32_t r) {
    return (2u * (r / (16u / ITEM))) & 63u;
}

template <int ITEM>
__device__ __forceinline__ uint32_t tile_byte(uint32_t r, uint32_t b) {  // byte b of row r
    return r * 256u + ((((b >> 2) ^ tile_swz<ITEM>(r)) << 2) | (b & 3u));
}

template <int ITEM>
__device__ __forceinline__ void tile_put16(uint8_t* s, uint32_t r, uint32_t b16, uint4 v) {
    const uint32_t sw = tile_swz<ITEM>(r);
    uint4* d = reinterpret_cast<uint4*>(s + r * 256u + (((b16 >> 2) ^ (sw & ~3u)) << 2));
    *d = (sw & 2u) ? make_uint4(v.z, v.w, v.x, v.y) : v;
}

template <int ITEM>
__device__ __forceinline__ uint4 tile_get16(const uint8_t* s, uint32_t r, uint32_t b16) {
    const uint32_t sw = tile_swz<ITEM>(r);
    const uint4 v = *reinterpret_cast<const uint4*>(s + r * 256u + (((b16 >> 2) ^ (sw & ~3u)) << 2));
    return (sw & 2u) ? make_uint4(v.z, v.w, v.x, v.y) : v;
}

}  // namespace

// PUB: 3 (production) = the returning publication with arrival bits, the
// chunk's word alone in its 128-byte line (p.ws + kPubLine c); 0 (arm
// ZHIP_TUNE_ARM = 1) = the same at p.ws + 4 c (round 3); 2 (arm 2) = deferred
// CRC verdicts (zarrhip.h: a non-returning xor per workgroup, the first
// workgroup of a chunk checks the previous launch's verdict).  Graph-timed on
// C3 (profiles/r04/b/arms_c3.jsonl): returning 29.30 us, deferred 29.85.
template <bool CRC, int ITEM, bool SWAP, int PUB = 3>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_decode_tile4(
    const DecodeParams p) {
    constexpr int kPer = 16 / ITEM;                // rows per 16-byte out piece
    constexpr int kPiecesPerCol = kTileRows / kPer;
    __shared__ uint32_t s_tab[CRC ? 16 * 256 : 1];
    __shared__ uint32_t s_tz[CRC ? 1024 : 1];
    __shared__ __attribute__((aligned(16))) uint8_t s_tile[kTileRows * 256];
    __shared__ uint32_t s_red[kThreads / 64];
    const int t = threadIdx.x;
    const uint32_t g = blockIdx.x;
    const uint32_t gpc = p.t_per_chunk / kTiles;  // workgroups per chunk (grid = n_chunks * gpc)
    const uint32_t c = g / gpc;
    const uint32_t grp = g - c * gpc;
    const uint32_t expected = p.g.nbytes + (CRC ? 4u : 0u);
    // 1. loads: tables and the lane constant first (L2 hits), then the chunk
    //    header (scalar), then the 16 data blocks
    uint4 tv0, tv1, tv2, tv3, tzv;
    uint32_t kq = 0;
    if constexpr (CRC) {
        const uint4* gt = reinterpret_cast<const uint4*>(p.horner);
        tv0 = gt[t];
        tv1 = gt[t + kThreads];
        tv2 = gt[t + 2 * kThreads];
        tv3 = gt[t + 3 * kThreads];
        tzv = reinterpret_cast<const uint4*>(p.tz)[t];
        kq = p.kq4[(size_t)grp * kThreads + t];
    }
    uint64_t dvprev = 0;
    if constexpr (CRC && PUB == 2) dvprev = dv_prev(p, c, grp == 0, g_tile_zero);
    const Unit U = resolve_unit(p, c * p.nseg, expected);
    const TileMap4 tm = load_uniform<TileMap4>(p.tmap + (size_t)grp * kTiles);
    const bool ok = U.mode == ZHIP_ST_OK;
    const uint32_t sq = p.sstride[p.tq];
    const uint32_t row0 = (uint32_t)t >> 4, col = 16u * (uint32_t)(t & 15);
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_tile_zero);
    uint4 blk[kTiles][kPasses];
#pragma unroll
    for (int j = 0; j < kTiles; ++j)
#pragma unroll
        for (int k = 0; k < kPasses; ++k)
            blk[j][k] = load_stream16_a1(ok ? U.cp + tm.e[j].tbase + (row0 + 16u * k) * sq + col : zero);
    uint32_t stored = 0;
    if (CRC && ok) stored = load_trailer_uniform(U.cp, p.g.nbytes);
    if constexpr (CRC) {
        uint4* st = reinterpret_cast<uint4*>(s_tab);
        st[t] = tv0;
        st[t + kThreads] = tv1;
        st[t + 2 * kThreads] = tv2;
        st[t + 3 * kThreads] = tv3;
        reinterpret_cast<uint4*>(s_tz)[t] = tzv;
    }
    // 2. per tile: LDS in stored order, out order back, 16-byte stores, then
    //    the tile's Horner steps
    const bool writes = ok || U.mode == ZHIP_ST_MISSING;
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
    const int32_t last = p.g.ndim - 1;
    const int64_t oq = p.g.ostride[p.tq];    // == ITEM
    const int64_t ocol = p.g.ostride[last];  // out stride of the innermost stored dim
    uint8_t* const obase = p.out + U.out_off;
    uint8_t* const sink = reinterpret_cast<uint8_t*>(g_tile_sink) + 16 * t;
    uint32_t S = 0;  // this thread's CRC state, referenced at the current tile
#pragma unroll
    for (int j = 0; j < kTiles; ++j) {
        if (j > 0) __syncthreads();  // the previous tile's LDS reads are done
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint4 v = swap_block<ITEM, SWAP>(blk[j][k]);
            tile_put16<ITEM>(s_tile, 16 * k + row0, col, v);
        }
        __syncthreads();  // tile j (and, first time, the tables) in LDS
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint32_t pc = (uint32_t)(k * kThreads + t);
            const uint32_t jc = pc / kPiecesPerCol;          // element of the stored row
            const uint32_t r0 = (pc % kPiecesPerCol) * kPer; // first of kPer tile rows
            uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int e = 0; e < kPer; ++e) {
                const uint8_t* src = s_tile + tile_byte<ITEM>(r0 + e, jc * ITEM);
                if constexpr (ITEM == 8) {
                    const uint2 v = *reinterpret_cast<const uint2*>(src);
                    w[2 * e] = v.x;
                    w[2 * e + 1] = v.y;
                } else if constexpr (ITEM == 4) {
                    w[e] = *reinterpret_cast<const uint32_t*>(src);
                } else if constexpr (ITEM == 2) {
                    w[e / 2] |= (uint32_t)(*reinterpret_cast<const uint16_t*>(src)) << (16 * (e & 1));
                } else {
                    w[e / 4] |= (uint32_t)(*src) << (8 * (e & 3));
                }
            }
            // every path stores (failed chunks to the sink): a static store count
            uint8_t* dst = writes ? obase + tm.e[j].orel + (int64_t)jc * ocol + (int64_t)r0 * oq : sink;
            store_nt16(dst, ok ? make_uint4(w[0], w[1], w[2], w[3]) : f);
        }
        // the tile's Horner steps after its stores are out (tables in LDS since
        // the first barrier); the state moves to this tile's reference
        if constexpr (CRC) {
            if (ok) {
                uint32_t acc = 0;
#pragma unroll
                for (int k = 0; k < kPasses; ++k) {
                    const uint4 v = blk[j][k];
                    acc = tab_apply(s_tab, acc ^ v.x) ^ tab_apply(s_tab + 1024, v.y) ^
                          tab_apply(s_tab + 2048, v.z) ^ tab_apply(s_tab + 3072, v.w);
                }
                S = (j == 0 ? 0u : tab_apply(s_tz, S)) ^ acc;
            }
        }
    }
    // 3. run end: shift (lane, last tile, chunk end in one constant), reduce,
    //    publish; the arrival completing the chunk compares with the trailer
    if (CRC && ok) {
        uint32_t v = wave_xor(gf_mul(S, kq));
        if ((t & 63) == 0) s_red[t >> 6] = v;
        __syncthreads();
        if (t < 64) {
            const uint32_t V = __builtin_amdgcn_readfirstlane(s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3]);
            uint32_t raw = 0, last_arrival = 0;
            if (PUB == 2) {
                if (t == 0) dv_publish(p, c, grp == 0, V, __builtin_amdgcn_readfirstlane(stored));
            } else if (t == 0) {
                if (gpc <= 32) {
                    const uint64_t full = gpc == 32 ? 0xFFFFFFFFull : ((1ull << gpc) - 1ull);
                    const uint64_t bits = 1ull << grp;
                    uint64_t* w = reinterpret_cast<uint64_t*>(p.ws + (PUB == 3 ? (uint64_t)kPubLine * c : 4ull * c));
                    const uint64_t prev = __hip_atomic_fetch_xor(w, (bits << 32) | V, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT);
                    if (((prev >> 32) ^ bits) == full) {
                        __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        raw = (uint32_t)prev ^ V;
                        last_arrival = 1;
                    }
                } else {  // more than 32 workgroups per chunk: xor, then count arrivals
                    uint32_t* accw = p.ws + 4ull * c;
                    const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
                    const uint32_t tk = __hip_atomic_fetch_add(accw + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (tk + 1u == gpc) {
                        raw = __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        last_arrival = 1;
                    }
                }
                if (last_arrival) {
                    const uint32_t computed = ~(raw ^ p.c3);  // kq4 carries t_c_inv
                    const uint32_t code = computed == stored ? ZHIP_ST_OK : ZHIP_ST_CRC_MISMATCH;
                    zhip_status st = {code, stored, computed, 0u};
                    p.status[c] = st;
                    if (code != ZHIP_ST_OK) atomicOr(p.errflag, 1u << code);
                }
            }
        }
    }
    // statuses not produced by the CRC finalize (deferred verdicts: a present
    // chunk is OK here, a mismatch is reported from its bank word)
    if (grp == 0 && t == 0) {
        if (ok) {
            if (!CRC || PUB == 2) {
                zhip_status st = {ZHIP_ST_OK, 0u, 0u, 0u};
                p.status[c] = st;
            }
        } else {
            zhip_status st = {U.mode, 0u, 0u, 0u};
            p.status[c] = st;
            if (U.mode != ZHIP_ST_MISSING) atomicOr(p.errflag, 1u << U.mode);
        }
        if constexpr (CRC && PUB == 2) dv_settle(p, c, dvprev);
    }
}

// k_decode_tile4f: k_decode_tile4 with one CRC chain per thread, for layouts
// whose four tiles per workgroup are the four 256-byte pieces of 1 KiB of every
// stored row (tile step 256 B; C3's transpose (2,1,0) of 64^3 chunks).  Thread
// t loads row t/4, blocks 16 (t%4) + 64 m of each tile, so its 16 blocks lie
// 64 B apart in the stored stream: one Horner chain through A_64 in the pair
// kernel's 11/11/10 layout (four word accumulators, 12 LDS lookups per block
// instead of 16, no tile-to-tile carry), one fold, one lane multiply by a
// host-built constant in the il kernel's frame (capi.cpp), one publication as
// in k_decode_tile4.  The LDS image and the out-order pass are k_decode_tile4's;
// 24 KiB of tables + the 16 KiB image (the reduction words reuse the image
// after the last pass): 40 KiB, four workgroups per CU.  A tuning arm
// (kTuneTile4F): exact on every tile4 test, but 0.3-0.4 us SLOWER than
// k_decode_tile4 on C3 (31.5-32.0 vs 31.2-31.6 us graph-timed,
// profiles/r03/tile4f/) -- its loads are 64-byte pieces of 16 rows per wave
// instruction instead of 256-byte rows, two requests per 128-byte line.
template <int ITEM, bool SWAP>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_decode_tile4f(
    const DecodeParams p) {
    constexpr int kPer = 16 / ITEM;
    constexpr int kPiecesPerCol = kTileRows / kPer;
    __shared__ __attribute__((aligned(16))) uint32_t s_mem[kPairTabWords + kTileRows * 64];
    uint32_t* const s_tab = s_mem;
    uint8_t* const s_tile = reinterpret_cast<uint8_t*>(s_mem + kPairTabWords);
    uint32_t* const s_red = s_mem + kPairTabWords;  // after the last out-order pass
    const int t = threadIdx.x;
    const uint32_t g = blockIdx.x;
    const uint32_t gpc = p.t_per_chunk / kTiles;
    const uint32_t c = g / gpc;
    const uint32_t grp = g - c * gpc;
    const uint32_t expected = p.g.nbytes + 4u;
    // 1. tables and the lane constant (L2 hits), the chunk header, 16 data blocks
    const uint4* gt = reinterpret_cast<const uint4*>(p.t4f_tab);
    const uint4 tv0 = gt[t], tv1 = gt[t + kThreads], tv2 = gt[t + 2 * kThreads], tv3 = gt[t + 3 * kThreads],
                tv4 = gt[t + 4 * kThreads], tv5 = gt[t + 5 * kThreads];
    const uint32_t kq = p.t4f_kq[(size_t)grp * kThreads + t];
    const Unit U = resolve_unit(p, c * p.nseg, expected);
    const TileMap4 tm = load_uniform<TileMap4>(p.tmap + (size_t)grp * kTiles);
    const bool ok = U.mode == ZHIP_ST_OK;
    const uint32_t sq = p.sstride[p.tq];
    const uint32_t row = (uint32_t)t >> 2, col0 = 16u * (uint32_t)(t & 3);
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_tile_zero);
    uint4 blk[kTiles][kPasses];
#pragma unroll
    for (int j = 0; j < kTiles; ++j)
#pragma unroll
        for (int k = 0; k < kPasses; ++k)
            blk[j][k] = load_stream16_a1(ok ? U.cp + tm.e[j].tbase + row * sq + col0 + 64u * k : zero);
    uint32_t stored = 0;
    if (ok) stored = load_trailer_uniform(U.cp, p.g.nbytes);
    {
        uint4* st = reinterpret_cast<uint4*>(s_tab);
        st[t] = tv0;
        st[t + kThreads] = tv1;
        st[t + 2 * kThreads] = tv2;
        st[t + 3 * kThreads] = tv3;
        st[t + 4 * kThreads] = tv4;
        st[t + 5 * kThreads] = tv5;
    }
    // 2. per tile: LDS in stored order, out order back, 16-byte stores, then
    //    the tile's four Horner steps (blocks 4 j .. 4 j + 3 of the chain)
    const bool writes = ok || U.mode == ZHIP_ST_MISSING;
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
    const int32_t last = p.g.ndim - 1;
    const int64_t oq = p.g.ostride[p.tq];
    const int64_t ocol = p.g.ostride[last];
    uint8_t* const obase = p.out + U.out_off;
    uint8_t* const sink = reinterpret_cast<uint8_t*>(g_tile_sink) + 16 * t;
    Acc4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < kTiles; ++j) {
        if (j > 0) __syncthreads();  // the previous tile's LDS reads are done
#pragma unroll
        for (int k = 0; k < kPasses; ++k) tile_put16<ITEM>(s_tile, row, col0 + 64u * k, swap_block<ITEM, SWAP>(blk[j][k]));
        __syncthreads();  // tile j (and, first time, the tables) in LDS
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint32_t pc = (uint32_t)(k * kThreads + t);
            const uint32_t jc = pc / kPiecesPerCol;
            const uint32_t r0 = (pc % kPiecesPerCol) * kPer;
            uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int e = 0; e < kPer; ++e) {
                const uint8_t* src = s_tile + tile_byte<ITEM>(r0 + e, jc * ITEM);
                if constexpr (ITEM == 8) {
                    const uint2 v = *reinterpret_cast<const uint2*>(src);
                    w[2 * e] = v.x;
                    w[2 * e + 1] = v.y;
                } else if constexpr (ITEM == 4) {
                    w[e] = *reinterpret_cast<const uint32_t*>(src);
                } else if constexpr (ITEM == 2) {
                    w[e / 2] |= (uint32_t)(*reinterpret_cast<const uint16_t*>(src)) << (16 * (e & 1));
                } else {
                    w[e / 4] |= (uint32_t)(*src) << (8 * (e & 3));
                }
            }
            uint8_t* dst = writes ? obase + tm.e[j].orel + (int64_t)jc * ocol + (int64_t)r0 * oq : sink;
            store_nt16(dst, ok ? make_uint4(w[0], w[1], w[2], w[3]) : f);
        }
        if (ok) {
#pragma unroll
            for (int k = 0; k < kPasses; ++k) crc_block4(s_tab, acc, blk[j][k]);
        }
    }
    // 3. run end: fold, lane multiply (lane, group and chunk end in one
    //    constant), reduce, publish; the arrival completing the chunk compares
    //    with the trailer
    if (ok) {
        const uint32_t v = wave_xor(lanemul_reg(kq, fold4(s_tab, acc)));
        __syncthreads();  // every out-order read of the last tile is done: s_red reuses the image
        if ((t & 63) == 0) s_red[t >> 6] = v;
        __syncthreads();
        if (t < 64) {
            const uint32_t V = __builtin_amdgcn_readfirstlane(s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3]);
            uint32_t raw = 0, last_arrival = 0;
            if (t == 0) {
                if (gpc <= 32) {
                    const uint64_t full = gpc == 32 ? 0xFFFFFFFFull : ((1ull << gpc) - 1ull);
                    const uint64_t bits = 1ull << grp;
                    uint64_t* w = reinterpret_cast<uint64_t*>(p.ws) + 2ull * c;
                    const uint64_t prev = __hip_atomic_fetch_xor(w, (bits << 32) | V, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT);
                    if (((prev >> 32) ^ bits) == full) {
                        __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        raw = (uint32_t)prev ^ V;
                        last_arrival = 1;
                    }
                } else {  // more than 32 workgroups per chunk: xor, then count arrivals
                    uint32_t* accw = p.ws + 4ull * c;
                    const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
                    const uint32_t tk = __hip_atomic_fetch_add(accw + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (tk + 1u == gpc) {
                        raw = __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        last_arrival = 1;
                    }
                }
                if (last_arrival) {
                    const uint32_t computed = ~(raw ^ p.c3);  // the lane constants carry c_inv
                    const uint32_t code = computed == stored ? ZHIP_ST_OK : ZHIP_ST_CRC_MISMATCH;
                    zhip_status st = {code, stored, computed, 0u};
                    p.status[c] = st;
                    if (code != ZHIP_ST_OK) atomicOr(p.errflag, 1u << code);
                }
            }
        }
    }
    // statuses not produced by the CRC finalize
    if (grp == 0 && t == 0 && !ok) {
        zhip_status st = {U.mode, 0u, 0u, 0u};
        p.status[c] = st;
        if (U.mode != ZHIP_ST_MISSING) atomicOr(p.errflag, 1u << U.mode);
    }
}

// k_decode_tile4w: k_decode_tile4 with one CRC chain per lane and one wave
// per tile.  Wave w of a workgroup loads tile w (of its four): lane l takes
// rows l/16 + 4 m (m < 16) at column block l % 16, so a wave instruction
// still loads four whole 256-byte rows (k_decode_tile4's width; k_decode_tile4f
// lost on its 64-byte pieces) and the lane's 16 blocks are 4 sq apart in the
// stored stream: ONE Horner chain through A_(4 sq) in the pair kernel's
// 11/11/10 layout (12 LDS lookups per block instead of 16, no tile-to-tile
// carry), one fold, one lane multiply by a host-built constant in the il
// frame (capi.cpp), one publication (a 128-byte line per chunk).  In tile
// iteration j wave j writes the whole 16 KiB image of tile j; every wave then
// reads it back in out order and stores, and takes four Horner steps of its
// own chain.  24 KiB of tables + the 16 KiB image: four workgroups per CU.
// Production for transposed layouts with a CRC since round 4: C3 28.9 vs
// 30.3-30.6 us graph-timed (profiles/r04/k/arms_c3.jsonl); ZHIP_TUNE_ARM 5
// (or 1 / 2, its publication arms) takes k_decode_tile4.
// (tileg_arrive: zhip_decode_common.h)

template <int N>
struct TileMapN {
    TileEnt e[N];
};

// NT: tiles per workgroup -- 4 (production) or 2 (arm 36: 2 048 workgroups of
// 32 KiB on C3, two residency rounds instead of one; two waves per tile, lane
// l of half h taking rows 32 h + l/16 + 4 m, m < 8: the same A_(4 sq) chain
// over 8 blocks)
// SPL (tuning arm 49): chunks of 17..32 workgroups publish through two
// subwords of 16 on lines of their own and a second level (tileg_arrive SPR)
// instead of 32 arrivals on the chunk's one word.
// BT (tuning arm 67): the chain through byte tables (crc_block4_t): 24 KiB of
// LDS per workgroup instead of 40, six resident per CU instead of four
template <int ITEM, bool SWAP, int NT = kTiles, bool SPL = false, bool BT = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_decode_tile4w(
    const DecodeParams p) {
    constexpr int kPer = 16 / ITEM;
    constexpr int kPiecesPerCol = kTileRows / kPer;
    constexpr int WPT = kTiles / NT;        // waves per tile
    constexpr int RPW = kTileRows / WPT;    // tile rows per wave
    constexpr int KB = RPW / 4;             // blocks per lane
    constexpr int HS = KB / NT;             // Horner steps per tile iteration
    constexpr int TW = BT ? kByteTabWords : kPairTabWords;  // table words
    __shared__ __attribute__((aligned(16))) uint32_t s_mem[TW + kTileRows * 64];
    uint32_t* const s_tab = s_mem;
    uint8_t* const s_tile = reinterpret_cast<uint8_t*>(s_mem + TW);
    uint32_t* const s_red = s_mem + TW;  // after the last out-order pass
    const int t = threadIdx.x;
    const uint32_t wv = __builtin_amdgcn_readfirstlane((uint32_t)t >> 6);
    const uint32_t tj = wv / WPT, hh = wv % WPT;  // this wave's tile and its row band
    const uint32_t ln = (uint32_t)t & 63u, rg = ln >> 4, cl = 16u * (ln & 15u);
    const uint32_t g = blockIdx.x;
    const uint32_t gpc = p.t_per_chunk / NT;
    const uint32_t c = g / gpc;
    const uint32_t grp = g - c * gpc;
    const uint32_t expected = p.g.nbytes + 4u;
    // 1. tables and the lane constant (L2 hits), the chunk header, the data blocks
    // (six uint4 table pieces per thread, two for the byte tables; named
    // registers -- an indexed array of them was placed in scratch)
    const uint4* gt = reinterpret_cast<const uint4*>(BT ? p.tbt_tab : p.t4w_tab);
    const uint4 tv0 = gt[t], tv1 = gt[t + kThreads];
    uint4 tv2, tv3, tv4, tv5;
    if constexpr (!BT) {
        tv2 = gt[t + 2 * kThreads];
        tv3 = gt[t + 3 * kThreads];
        tv4 = gt[t + 4 * kThreads];
        tv5 = gt[t + 5 * kThreads];
    }
    const uint32_t kq = p.t4w_kq[(size_t)grp * kThreads + t];
    const Unit U = resolve_unit(p, c * p.nseg, expected);
    const TileMapN<NT> tm = load_uniform<TileMapN<NT>>(p.tmap + (size_t)grp * NT);
    const TileEnt mine = load_uniform<TileEnt>(p.tmap + (size_t)grp * NT + tj);
    const bool ok = U.mode == ZHIP_ST_OK;
    const uint32_t sq = p.sstride[p.tq];
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_tile_zero);
    uint4 blk[KB];
#pragma unroll
    for (int m = 0; m < KB; ++m)
        blk[m] = load_stream16_a1(ok ? U.cp + mine.tbase + (hh * RPW + rg + 4u * (uint32_t)m) * sq + cl : zero);
    uint32_t stored = 0;
    if (ok) stored = load_trailer_uniform(U.cp, p.g.nbytes);
    {
        uint4* st = reinterpret_cast<uint4*>(s_tab);
        st[t] = tv0;
        st[t + kThreads] = tv1;
        if constexpr (!BT) {
            st[t + 2 * kThreads] = tv2;
            st[t + 3 * kThreads] = tv3;
            st[t + 4 * kThreads] = tv4;
            st[t + 5 * kThreads] = tv5;
        }
    }
    // 2. per tile: wave j writes tile j into LDS in stored order, every wave
    //    reads it back in out order and stores 16-byte pieces, then takes four
    //    Horner steps of its own chain
    const bool writes = ok || U.mode == ZHIP_ST_MISSING;
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
    const int32_t last = p.g.ndim - 1;
    const int64_t oq = p.g.ostride[p.tq];
    const int64_t ocol = p.g.ostride[last];
    uint8_t* const obase = p.out + U.out_off;
    uint8_t* const sink = reinterpret_cast<uint8_t*>(g_tile_sink) + 16 * t;
    Acc4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        if (j > 0) __syncthreads();  // the previous tile's LDS reads are done
        if (tj == (uint32_t)j) {
#pragma unroll
            for (int m = 0; m < KB; ++m)
                tile_put16<ITEM>(s_tile, hh * RPW + rg + 4u * (uint32_t)m, cl, swap_block<ITEM, SWAP>(blk[m]));
        }
        __syncthreads();  // tile j (and, first time, the tables) in LDS
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint32_t pc = (uint32_t)(k * kThreads + t);
            const uint32_t jc = pc / kPiecesPerCol;
            const uint32_t r0 = (pc % kPiecesPerCol) * kPer;
            uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int e = 0; e < kPer; ++e) {
                const uint8_t* src = s_tile + tile_byte<ITEM>(r0 + e, jc * ITEM);
                if constexpr (ITEM == 8) {
                    const uint2 v = *reinterpret_cast<const uint2*>(src);
                    w[2 * e] = v.x;
                    w[2 * e + 1] = v.y;
                } else if constexpr (ITEM == 4) {
                    w[e] = *reinterpret_cast<const uint32_t*>(src);
                } else if constexpr (ITEM == 2) {
                    w[e / 2] |= (uint32_t)(*reinterpret_cast<const uint16_t*>(src)) << (16 * (e & 1));
                } else {
                    w[e / 4] |= (uint32_t)(*src) << (8 * (e & 3));
                }
            }
            uint8_t* dst = writes ? obase + tm.e[j].orel + (int64_t)jc * ocol + (int64_t)r0 * oq : sink;
            store_nt16(dst, ok ? make_uint4(w[0], w[1], w[2], w[3]) : f);
        }
        if (ok) {
#pragma unroll
            for (int m = HS * j; m < HS * j + HS; ++m) crc_block4_t<BT>(s_tab, acc, blk[m]);
        }
    }
    // 3. run end: fold, lane multiply, reduce, publish (returning, the chunk's
    //    word alone in its 128-byte line); the arrival completing the chunk
    //    compares with the trailer
    if (ok) {
        const uint32_t v = wave_xor(lanemul_reg(kq, fold4_t<BT>(s_tab, acc)));
        __syncthreads();  // every out-order read of the last tile is done: s_red reuses the image
        if ((t & 63) == 0) s_red[t >> 6] = v;
        __syncthreads();
        if (t < 64) {
            const uint32_t V = __builtin_amdgcn_readfirstlane(s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3]);
            uint32_t raw = 0, last_arrival = 0;
            if (t == 0) {
                if (SPL && gpc > 16u && gpc <= 32u) {
                    bool any_ne;
                    last_arrival = tileg_arrive<true>(p.ws, p.n_chunks, c, grp, gpc, 2u, V, false, raw, any_ne) ? 1u : 0u;
                } else if (gpc <= 32) {
                    const uint64_t full = gpc == 32 ? 0xFFFFFFFFull : ((1ull << gpc) - 1ull);
                    const uint64_t bits = 1ull << grp;
                    uint64_t* w = reinterpret_cast<uint64_t*>(p.ws) + (uint64_t)(kPubLine / 2u) * c;
                    const uint64_t prev = __hip_atomic_fetch_xor(w, (bits << 32) | V, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT);
                    if (((prev >> 32) ^ bits) == full) {
                        __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        raw = (uint32_t)prev ^ V;
                        last_arrival = 1;
                    }
                } else if (gpc <= 256u) {  // subwords of 16 workgroups (tile pairs of large chunks;
                    // two tiles: on lines of their own, as k_decode_tilegw's two-tile form)
                    bool any_ne;
                    last_arrival = tileg_arrive<NT == 2>(p.ws, p.n_chunks, c, grp, gpc, (gpc + 15u) / 16u, V, false, raw,
                                                any_ne) ? 1u : 0u;
                } else {  // more than 256 workgroups per chunk: xor, then count arrivals
                    uint32_t* accw = p.ws + 4ull * c;
                    const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
                    const uint32_t tk = __hip_atomic_fetch_add(accw + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (tk + 1u == gpc) {
                        raw = __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        last_arrival = 1;
                    }
                }
                if (last_arrival) {
                    const uint32_t computed = ~(raw ^ p.c3);  // the lane constants carry c_inv
                    const uint32_t code = computed == stored ? ZHIP_ST_OK : ZHIP_ST_CRC_MISMATCH;
                    zhip_status st = {code, stored, computed, 0u};
                    p.status[c] = st;
                    if (code != ZHIP_ST_OK) atomicOr(p.errflag, 1u << code);
                }
            }
        }
    }
    // statuses not produced by the CRC finalize
    if (grp == 0 && t == 0 && !ok) {
        zhip_status st = {U.mode, 0u, 0u, 0u};
        p.status[c] = st;
        if (U.mode != ZHIP_ST_MISSING) atomicOr(p.errflag, 1u << U.mode);
    }
}

// k_decode_tileg: k_decode_tile4 for the transposed layouts it declines
// (partial tiles, more tiles per chunk, irregular steps between consecutive
// tiles), as long as some stored dim gd other than tq and the innermost has
// shape % 4 == 0: tiles are grouped by four along gd (a uniform stored and out
// step inside every group), partial tiles masked with the group's row / byte
// extent.  Same structure as k_decode_tile4 -- every load first, per tile LDS
// image -> out pieces -> 16-byte stores (failed chunks to a sink, a static
// count) -> Horner steps, the state carried by one table multiply -- and one
// lane multiply, one reduction and one XOR + arrival pair per workgroup (any
// number of groups per chunk).  PUB as in k_decode_tile4 (2: deferred CRC
// verdicts, production; 0: the returning two-level arrival, arm 2).
template <bool CRC, int ITEM, bool SWAP, int PUB = 2>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_decode_tileg(
    const DecodeParams p) {
    constexpr int kPer = 16 / ITEM;
    constexpr int kPiecesPerCol = kTileRows / kPer;
    __shared__ uint32_t s_tab[CRC ? 16 * 256 : 1];
    __shared__ uint32_t s_tz[CRC ? 1024 : 1];
    __shared__ __attribute__((aligned(16))) uint8_t s_tile[kTileRows * 256];
    __shared__ uint32_t s_red[kThreads / 64];
    const int t = threadIdx.x;
    const uint32_t gpc = p.n_groups;
    const uint32_t c = blockIdx.x / gpc;
    const uint32_t grp = blockIdx.x - c * gpc;
    const uint32_t expected = p.g.nbytes + (CRC ? 4u : 0u);
    uint4 tv0, tv1, tv2, tv3, tzv;
    uint32_t kth = 0;
    if constexpr (CRC) {
        const uint4* gt = reinterpret_cast<const uint4*>(p.horner);
        tv0 = gt[t];
        tv1 = gt[t + kThreads];
        tv2 = gt[t + 2 * kThreads];
        tv3 = gt[t + 3 * kThreads];
        tzv = reinterpret_cast<const uint4*>(p.gtz)[t];
        kth = p.kthread[t];
    }
    uint64_t dvprev = 0;
    if constexpr (CRC && PUB == 2) dvprev = dv_prev(p, c, grp == 0, g_tile_zero);
    const Unit U = resolve_unit(p, c * p.nseg, expected);
    const GroupEnt ge = load_uniform<GroupEnt>(p.gmap + grp);
    const bool ok = U.mode == ZHIP_ST_OK;
    const uint32_t sq = p.sstride[p.tq];
    const int32_t rows = ge.rows, cols = ge.cols;
    const uint32_t row0 = (uint32_t)t >> 4, col = 16u * (uint32_t)(t & 15);
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_tile_zero);
    const bool lane_in = (int32_t)col < cols;
    uint4 blk[kTiles][kPasses];
#pragma unroll
    for (int j = 0; j < kTiles; ++j)
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint32_t row = row0 + 16u * k;
            blk[j][k] = load_stream16_a1(ok && lane_in && (int32_t)row < rows
                                         ? U.cp + ge.tbase + (size_t)j * p.g_step_t + row * sq + col
                                         : zero);
        }
    uint32_t stored = 0;
    if (CRC && ok) stored = load_trailer_uniform(U.cp, p.g.nbytes);
    if constexpr (CRC) {
        uint4* st = reinterpret_cast<uint4*>(s_tab);
        st[t] = tv0;
        st[t + kThreads] = tv1;
        st[t + 2 * kThreads] = tv2;
        st[t + 3 * kThreads] = tv3;
        reinterpret_cast<uint4*>(s_tz)[t] = tzv;
    }
    const bool writes = ok || U.mode == ZHIP_ST_MISSING;
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
    const int32_t last = p.g.ndim - 1;
    const int64_t oq = p.g.ostride[p.tq];    // == ITEM
    const int64_t ocol = p.g.ostride[last];  // out stride of the innermost stored dim
    uint8_t* const obase = p.out + U.out_off + ge.orel;
    uint8_t* const sink = reinterpret_cast<uint8_t*>(g_tile_sink) + 16 * t;
    uint32_t S = 0;
#pragma unroll
    for (int j = 0; j < kTiles; ++j) {
        if (j > 0) __syncthreads();
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint4 v = swap_block<ITEM, SWAP>(blk[j][k]);
            tile_put16<ITEM>(s_tile, 16 * k + row0, col, v);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint32_t pc = (uint32_t)(k * kThreads + t);
            const uint32_t jc = pc / kPiecesPerCol;
            const uint32_t r0 = (pc % kPiecesPerCol) * kPer;
            uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int e = 0; e < kPer; ++e) {
                const uint8_t* src = s_tile + tile_byte<ITEM>(r0 + e, jc * ITEM);
                if constexpr (ITEM == 8) {
                    const uint2 v = *reinterpret_cast<const uint2*>(src);
                    w[2 * e] = v.x;
                    w[2 * e + 1] = v.y;
                } else if constexpr (ITEM == 4) {
                    w[e] = *reinterpret_cast<const uint32_t*>(src);
                } else if constexpr (ITEM == 2) {
                    w[e / 2] |= (uint32_t)(*reinterpret_cast<const uint16_t*>(src)) << (16 * (e & 1));
                } else {
                    w[e / 4] |= (uint32_t)(*src) << (8 * (e & 3));
                }
            }
            // pieces outside the tile (and failed chunks) store to the sink
            const bool in = writes && (int32_t)(jc * ITEM) < cols && (int32_t)r0 < rows;
            uint8_t* dst = in ? obase + (int64_t)j * p.g_step_o + (int64_t)jc * ocol + (int64_t)r0 * oq : sink;
            store_nt16(dst, ok ? make_uint4(w[0], w[1], w[2], w[3]) : f);
        }
        if constexpr (CRC) {
            if (ok) {
                uint32_t acc = 0;
#pragma unroll
                for (int k = 0; k < kPasses; ++k) {
                    const uint4 v = blk[j][k];
                    acc = tab_apply(s_tab, acc ^ v.x) ^ tab_apply(s_tab + 1024, v.y) ^
                          tab_apply(s_tab + 2048, v.z) ^ tab_apply(s_tab + 3072, v.w);
                }
                S = (j == 0 ? 0u : tab_apply(s_tz, S)) ^ acc;
            }
        }
    }
    if (CRC && ok) {
        uint32_t v = wave_xor(gf_mul(S, kth));
        if ((t & 63) == 0) s_red[t >> 6] = v;
        __syncthreads();
        if (t == 0 && PUB == 2) {
            dv_publish(p, c, grp == 0, gf_mul(s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3], ge.ku), stored);
        } else if (t == 0) {
            const uint32_t V = gf_mul(s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3], ge.ku);
            uint32_t raw = 0;
            bool last_one = false;
            if (gpc <= 16u || p.n_sub) {
                bool any_ne;
                last_one = tileg_arrive(p.ws, p.n_chunks, c, grp, gpc, p.n_sub, V, false, raw, any_ne);
            } else {  // more than 256 groups per chunk: XOR, then count arrivals
                uint32_t* accw = p.ws + 4ull * c;
                const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
                const uint32_t tk = __hip_atomic_fetch_add(accw + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (tk + 1u == gpc) {
                    raw = __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    last_one = true;
                }
            }
            if (last_one) {
                const uint32_t computed = ~(raw ^ p.c3);  // ku carries t_c_inv
                const uint32_t code = computed == stored ? ZHIP_ST_OK : ZHIP_ST_CRC_MISMATCH;
                zhip_status st = {code, stored, computed, 0u};
                p.status[c] = st;
                if (code != ZHIP_ST_OK) atomicOr(p.errflag, 1u << code);
            }
        }
    }
    if (grp == 0 && t == 0) {
        if (ok) {
            if (!CRC || PUB == 2) {
                zhip_status st = {ZHIP_ST_OK, 0u, 0u, 0u};
                p.status[c] = st;
            }
        } else {
            zhip_status st = {U.mode, 0u, 0u, 0u};
            p.status[c] = st;
            if (U.mode != ZHIP_ST_MISSING) atomicOr(p.errflag, 1u << U.mode);
        }
        if constexpr (CRC && PUB == 2) dv_settle(p, c, dvprev);
    }
}

// k_decode_tilegw: k_decode_tileg with k_decode_tile4w's chains: wave w owns
// tile w of its group (lane l: rows l/16 + 4 m, column block l % 16; rows
// and columns past a partial tile load zeros, which the chain steps over like
// absent bytes), one A_(4 sq) chain per lane, the group's and lane's frame in
// the host-built lane constant; the publication of k_decode_tileg (deferred
// verdicts).  Production for grouped CRC layouts since round 4: C3 in 128^3
// chunks 28.7-28.9 vs 30.2-30.3 us graph-timed (profiles/r04/l/); arms 2 / 5
// take k_decode_tileg.  (Taking the previous tile's Horner steps before the
// barrier, while one wave writes the image, measured the same in
// k_decode_tile4w.)
// PUB: 2 = deferred verdicts (ZHIP_DF_DEFER, the Python path's choice), 0 =
// the returning two-level arrival of k_decode_tileg (the C-ABI default: the
// launch itself sets the chunk's status and the error word).
// NT: tiles per workgroup -- 4, or 2 (two workgroups per group of four, two
// waves per tile as in k_decode_tile4w's two-tile form; the returning
// publication then xors and counts per chunk)
// LT (four tiles, tuning arm 40): lanes, not waves, pick the tile -- lane l of
// wave w loads rows w + 4 m of tile l / 16 (column block l % 16), so one load
// instruction reads one row of all four tiles (four 256-byte pieces one
// group step apart) instead of four rows of one tile (a stored-row stride
// apart: 64 KiB in 128^3 chunks); the chain is the same A_(4 sq) one, the lane
// constants swap the roles of w and l / 16, and in tile iteration j the 16
// lanes of every wave that hold tile j write the image.
// LB (tuning arm 62): the returning arrival replaced by tileg_arrive_lb (the
//   chunk's last workgroup polls, the others retire after a non-returning xor)
// BT (tuning arm 66): the chain through byte tables (crc_block4_t), 24 KiB of
//   LDS instead of 40
template <int ITEM, bool SWAP, int PUB = 2, int NT = kTiles, bool LT = false, bool SPR = false, bool LB = false,
          bool BT = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_decode_tilegw(
    const DecodeParams p) {
    static_assert(!LT || NT == kTiles, "lane-tile mapping: four tiles per workgroup");
    constexpr int kPer = 16 / ITEM;
    constexpr int kPiecesPerCol = kTileRows / kPer;
    constexpr int WPT = kTiles / NT;        // waves per tile
    constexpr int RPW = kTileRows / WPT;    // tile rows per wave
    constexpr int KB = RPW / 4;             // blocks per lane
    constexpr int HS = KB / NT;             // Horner steps per tile iteration
    constexpr uint32_t PG = kTiles / NT;    // workgroups per group of four tiles
    constexpr int TW = BT ? kByteTabWords : kPairTabWords;  // table words
    __shared__ __attribute__((aligned(16))) uint32_t s_mem[TW + kTileRows * 64];
    uint32_t* const s_tab = s_mem;
    uint8_t* const s_tile = reinterpret_cast<uint8_t*>(s_mem + TW);
    uint32_t* const s_red = s_mem + TW;  // after the last out-order pass
    const int t = threadIdx.x;
    const uint32_t wv = __builtin_amdgcn_readfirstlane((uint32_t)t >> 6);
    const uint32_t ln = (uint32_t)t & 63u, cl = 16u * (ln & 15u);
    // the lane's tile (of the workgroup's), row band and first row
    const uint32_t tj = LT ? (ln >> 4) : wv / WPT, hh = LT ? 0u : wv % WPT;
    const uint32_t rg = LT ? wv : (ln >> 4);
    const uint32_t gpc = p.n_groups * PG;  // workgroups per chunk
    const uint32_t c = blockIdx.x / gpc;
    const uint32_t wg = blockIdx.x - c * gpc;
    const uint32_t grp = wg / PG, t0 = (wg % PG) * NT;  // the group and its first tile here
    const uint32_t expected = p.g.nbytes + 4u;
    // (six uint4 table pieces per thread, two for the byte tables; named
    // registers -- an indexed array of them was placed in scratch)
    const uint4* gt = reinterpret_cast<const uint4*>(BT ? p.tbt_tab : p.t4w_tab);
    const uint4 tv0 = gt[t], tv1 = gt[t + kThreads];
    uint4 tv2, tv3, tv4, tv5;
    if constexpr (!BT) {
        tv2 = gt[t + 2 * kThreads];
        tv3 = gt[t + 3 * kThreads];
        tv4 = gt[t + 4 * kThreads];
        tv5 = gt[t + 5 * kThreads];
    }
    const uint32_t kq = p.t4w_kq[(size_t)wg * kThreads + t];
    // (the two-tile form always reports in-launch: twice the workgroups per
    // chunk made the deferred verdicts' one same-address word per chunk the
    // tail -- 36.8 vs 29.8 us on C3 in 128^3 chunks; its two-level returning
    // arrival keeps every word at 16 arrivals)
    constexpr bool kDefer = PUB == 2 && NT == kTiles;
    uint64_t dvprev = 0;
    if constexpr (kDefer) dvprev = dv_prev(p, c, wg == 0, g_tile_zero);
    const Unit U = resolve_unit(p, c * p.nseg, expected);
    const GroupEnt ge = load_uniform<GroupEnt>(p.gmap + grp);
    const bool ok = U.mode == ZHIP_ST_OK;
    const uint32_t sq = p.sstride[p.tq];
    const int32_t rows = ge.rows, cols = ge.cols;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_tile_zero);
    const bool lane_in = (int32_t)cl < cols;
    const uint8_t* const tb = U.cp + ge.tbase + (size_t)(t0 + tj) * p.g_step_t;
    uint4 blk[KB];
#pragma unroll
    for (int m = 0; m < KB; ++m) {
        const uint32_t row = hh * RPW + rg + 4u * (uint32_t)m;
        blk[m] = load_stream16_a1(ok && lane_in && (int32_t)row < rows ? tb + row * sq + cl : zero);
    }
    uint32_t stored = 0;
    if (ok) stored = load_trailer_uniform(U.cp, p.g.nbytes);
    {
        uint4* st = reinterpret_cast<uint4*>(s_tab);
        st[t] = tv0;
        st[t + kThreads] = tv1;
        if constexpr (!BT) {
            st[t + 2 * kThreads] = tv2;
            st[t + 3 * kThreads] = tv3;
            st[t + 4 * kThreads] = tv4;
            st[t + 5 * kThreads] = tv5;
        }
    }
    const bool writes = ok || U.mode == ZHIP_ST_MISSING;
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
    const int32_t last = p.g.ndim - 1;
    const int64_t oq = p.g.ostride[p.tq];
    const int64_t ocol = p.g.ostride[last];
    uint8_t* const obase = p.out + U.out_off + ge.orel;
    uint8_t* const sink = reinterpret_cast<uint8_t*>(g_tile_sink) + 16 * t;
    Acc4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        if (j > 0) __syncthreads();
        if (tj == (uint32_t)j) {
#pragma unroll
            for (int m = 0; m < KB; ++m)
                tile_put16<ITEM>(s_tile, hh * RPW + rg + 4u * (uint32_t)m, cl, swap_block<ITEM, SWAP>(blk[m]));
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint32_t pc = (uint32_t)(k * kThreads + t);
            const uint32_t jc = pc / kPiecesPerCol;
            const uint32_t r0 = (pc % kPiecesPerCol) * kPer;
            uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int e = 0; e < kPer; ++e) {
                const uint8_t* src = s_tile + tile_byte<ITEM>(r0 + e, jc * ITEM);
                if constexpr (ITEM == 8) {
                    const uint2 v = *reinterpret_cast<const uint2*>(src);
                    w[2 * e] = v.x;
                    w[2 * e + 1] = v.y;
                } else if constexpr (ITEM == 4) {
                    w[e] = *reinterpret_cast<const uint32_t*>(src);
                } else if constexpr (ITEM == 2) {
                    w[e / 2] |= (uint32_t)(*reinterpret_cast<const uint16_t*>(src)) << (16 * (e & 1));
                } else {
                    w[e / 4] |= (uint32_t)(*src) << (8 * (e & 3));
                }
            }
            const bool in = writes && (int32_t)(jc * ITEM) < cols && (int32_t)r0 < rows;
            uint8_t* dst = in ? obase + (int64_t)(t0 + j) * p.g_step_o + (int64_t)jc * ocol + (int64_t)r0 * oq : sink;
            store_nt16(dst, ok ? make_uint4(w[0], w[1], w[2], w[3]) : f);
        }
        if (ok) {
#pragma unroll
            for (int m = HS * j; m < HS * j + HS; ++m) crc_block4_t<BT>(s_tab, acc, blk[m]);
        }
    }
    if (ok) {
        const uint32_t v = wave_xor(lanemul_reg(kq, fold4_t<BT>(s_tab, acc)));
        __syncthreads();  // every out-order read of the last tile is done: s_red reuses the image
        if ((t & 63) == 0) s_red[t >> 6] = v;
        __syncthreads();
        if (t == 0 && kDefer) {
            dv_publish(p, c, wg == 0, s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3], stored);
        } else if (t == 0) {  // the returning arrival of k_decode_tileg (V in the same frame)
            const uint32_t V = s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3];
            uint32_t raw = 0;
            bool last_one = false;
            // subgroups of 16 workgroups (the plan's n_sub for four tiles; for two,
            // zhip_plan_info sizes the workspace tail for twice as many)
            const uint32_t nsub = NT == kTiles ? p.n_sub : ((gpc > 16u && gpc <= 256u) ? (gpc + 15u) / 16u : 0u);
            if (LB && (gpc <= 16u || nsub)) {
                bool any_ne;
                last_one = tileg_arrive_lb(p.ws, p.n_chunks, c, wg, gpc, nsub, V, false, raw, any_ne);
            } else if (gpc <= 16u || nsub) {
                bool any_ne;
                last_one = tileg_arrive<SPR>(p.ws, p.n_chunks, c, wg, gpc, nsub, V, false, raw, any_ne);
            } else {  // more than 256 groups per chunk: XOR, then count arrivals
                uint32_t* accw = p.ws + 4ull * c;
                const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
                const uint32_t tk = __hip_atomic_fetch_add(accw + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (tk + 1u == gpc) {
                    raw = __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    last_one = true;
                }
            }
            if (last_one) {
                const uint32_t computed = ~(raw ^ p.c3);
                const uint32_t code = computed == stored ? ZHIP_ST_OK : ZHIP_ST_CRC_MISMATCH;
                zhip_status st = {code, stored, computed, 0u};
                p.status[c] = st;
                if (code != ZHIP_ST_OK) atomicOr(p.errflag, 1u << code);
            }
        }
    }
    if (wg == 0 && t == 0) {
        if (ok) {
            if constexpr (kDefer) {
                zhip_status st = {ZHIP_ST_OK, 0u, 0u, 0u};
                p.status[c] = st;
            }
        } else {
            zhip_status st = {U.mode, 0u, 0u, 0u};
            p.status[c] = st;
            if (U.mode != ZHIP_ST_MISSING) atomicOr(p.errflag, 1u << U.mode);
        }
        if constexpr (kDefer) dv_settle(p, c, dvprev);
    }
}

// k_encode_tile4: the same four tiles per workgroup in reverse (TransposeCodec
// _encode_sync, transpose.py:113-118): 16-byte pieces of the source array's
// out-contiguous rows are gathered (all 16 per thread issued first), written
// into the LDS image at their transposed place, read back in stored order,
// fill-tested, byteswapped, stored as whole 256-byte rows of the stored chunk
// and run through the tile's Horner steps.  One 64-bit atomic per workgroup
// carries CRC | tile-group arrival | tile-group non-empty bits (at most 16
// workgroups per chunk); the last arrival writes trailer, status and the
// chunk's non-empty flag.
// NT: tiles per workgroup -- 4, or 2 (twice the workgroups: two residency
// rounds, as k_decode_tile4w's two-tile form; up to 32 workgroups per chunk
// publish per half-chunk word with a second level, as k_encode_il)
template <bool CRC, int ITEM, bool SWAP, int NT = kTiles>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_encode_tile4(
    const EncodeParams p) {
    constexpr int kPer = 16 / ITEM;
    constexpr int kPiecesPerCol = kTileRows / kPer;
    __shared__ uint32_t s_tab[CRC ? 16 * 256 : 1];
    __shared__ uint32_t s_tz[CRC ? 1024 : 1];
    __shared__ __attribute__((aligned(16))) uint8_t s_tile[kTileRows * 256];
    __shared__ uint32_t s_red[kThreads / 64];
    __shared__ uint32_t s_ne[kThreads / 64];
    const int t = threadIdx.x;
    const uint32_t g = blockIdx.x;
    const uint32_t gpc = p.t_per_chunk / NT;
    const uint32_t c = g / gpc;
    const uint32_t grp = g - c * gpc;
    uint4 tv0, tv1, tv2, tv3, tzv;
    uint32_t kq = 0;
    if constexpr (CRC) {
        const uint4* gt = reinterpret_cast<const uint4*>(p.horner);
        tv0 = gt[t];
        tv1 = gt[t + kThreads];
        tv2 = gt[t + 2 * kThreads];
        tv3 = gt[t + 3 * kThreads];
        tzv = reinterpret_cast<const uint4*>(p.tz)[t];
        kq = p.kq4[(size_t)grp * kThreads + t];  // (NT = 2: the two-tile constants, launch_encode)
    }
    const zhip_chunk ch = load_uniform<zhip_chunk>(p.chunks + c);  // src: dst offset, out_off: source offset
    const TileMapN<NT> tm = load_uniform<TileMapN<NT>>(p.tmap + (size_t)grp * NT);
    const int32_t last = p.g.ndim - 1;
    const int64_t oq = p.g.ostride[p.tq];    // == ITEM (source stride of the out-contiguous dim)
    const int64_t ocol = p.g.ostride[last];  // source stride of the innermost stored dim
    const uint8_t* const abase = p.arr + ch.out_off;
    uint8_t* const cp = p.dst + ch.src;
    const uint32_t sq = p.sstride[p.tq];
    const uint32_t row0 = (uint32_t)t >> 4, col = 16u * (uint32_t)(t & 15);
    // 1. gather every piece of the four tiles
    uint4 pcs[NT][kPasses];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint32_t pc = (uint32_t)(k * kThreads + t);
            const uint32_t jc = pc / kPiecesPerCol;
            const uint32_t r0 = (pc % kPiecesPerCol) * kPer;
            pcs[j][k] = load_stream16_a1(abase + tm.e[j].orel + (int64_t)jc * ocol + (int64_t)r0 * oq);
        }
    if constexpr (CRC) {
        uint4* st = reinterpret_cast<uint4*>(s_tab);
        st[t] = tv0;
        st[t + kThreads] = tv1;
        st[t + 2 * kThreads] = tv2;
        st[t + 3 * kThreads] = tv3;
        reinterpret_cast<uint4*>(s_tz)[t] = tzv;
    }
    uint32_t S = 0;
    bool eq = true;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        if (j > 0) __syncthreads();  // the previous tile's LDS reads are done
        // 2. pieces into the LDS image at their stored (row, column) place
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint32_t pc = (uint32_t)(k * kThreads + t);
            const uint32_t jc = pc / kPiecesPerCol;
            const uint32_t r0 = (pc % kPiecesPerCol) * kPer;
            const uint32_t w[4] = {pcs[j][k].x, pcs[j][k].y, pcs[j][k].z, pcs[j][k].w};
#pragma unroll
            for (int e = 0; e < kPer; ++e) {
                uint8_t* dst = s_tile + tile_byte<ITEM>(r0 + e, jc * ITEM);
                if constexpr (ITEM == 8) {
                    *reinterpret_cast<uint2*>(dst) = make_uint2(w[2 * e], w[2 * e + 1]);
                } else if constexpr (ITEM == 4) {
                    *reinterpret_cast<uint32_t*>(dst) = w[e];
                } else if constexpr (ITEM == 2) {
                    *reinterpret_cast<uint16_t*>(dst) = (uint16_t)(w[e / 2] >> (16 * (e & 1)));
                } else {
                    *dst = (uint8_t)(w[e / 4] >> (8 * (e & 3)));
                }
            }
        }
        __syncthreads();  // tile j (and, first time, the tables) in LDS
        // 3. stored-order blocks: fill test, byteswap, store, Horner steps
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint4 v = tile_get16<ITEM>(s_tile, 16 * k + row0, col);
            eq = eq && block_eq_fill_e<ITEM>(v, p);
            const uint4 e = swap_block<ITEM, SWAP>(v);
            store_nt16_a1(cp + tm.e[j].tbase + (row0 + 16u * k) * sq + col, e);
            if constexpr (CRC)
                acc = tab_apply(s_tab, acc ^ e.x) ^ tab_apply(s_tab + 1024, e.y) ^ tab_apply(s_tab + 2048, e.z) ^
                      tab_apply(s_tab + 3072, e.w);
        }
        if constexpr (CRC) S = (j == 0 ? 0u : tab_apply(s_tz, S)) ^ acc;
    }
    // 4. run end
    uint32_t v = 0;
    if constexpr (CRC) v = wave_xor(gf_mul(S, kq));
    const bool wne = __any(!eq);
    if ((t & 63) == 0) {
        s_red[t >> 6] = v;
        s_ne[t >> 6] = wne ? 1u : 0u;
    }
    __syncthreads();
    if (t != 0) return;
    const uint32_t V = CRC ? (s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3]) : 0u;
    const bool ne = (s_ne[0] | s_ne[1] | s_ne[2] | s_ne[3]) != 0u;
    uint64_t* w = reinterpret_cast<uint64_t*>(p.ws) + (uint64_t)p.pub_stride * c;
    // halves of at most 16 workgroups: CRC | arrival bits 32..47 | non-empty
    // bits 48..63 per half word, the last of a half folds it into the line's
    // third word (one half up to 16 workgroups: no second level)
    const uint32_t h = grp >> 4, b = grp & 15u;
    const uint32_t n_h = h ? gpc - 16u : (gpc < 16u ? gpc : 16u);
    const uint64_t pb = 1ull << b;
    const uint64_t word = (pb << 32) | (ne ? pb << 48 : 0ull) | V;
    const uint64_t prev = __hip_atomic_fetch_xor(w + h, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((((prev ^ word) >> 32) & 0xFFFFull) != (1ull << n_h) - 1ull) return;
    __hip_atomic_store(w + h, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t all = prev ^ word;
    if (gpc > 16u) {
        const uint64_t hb = 1ull << h;
        const uint64_t w2 = (hb << 32) | ((all >> 48) ? hb << 48 : 0ull) | (uint32_t)all;
        const uint64_t p2 = __hip_atomic_fetch_xor(w + 2, w2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((((p2 ^ w2) >> 32) & 0xFFFFull) != 3ull) return;
        __hip_atomic_store(w + 2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        all = p2 ^ w2;
    }
    p.nonempty[c] = (all >> 48) != 0ull ? 1u : 0u;
    uint32_t crc = 0;
    if constexpr (CRC) {
        crc = ~((uint32_t)all ^ p.c3);  // kq4 carries t_c_inv
        uint8_t* tr = cp + p.g.nbytes;  // LE trailer (crc32c_.py:64-68)
        tr[0] = (uint8_t)crc;
        tr[1] = (uint8_t)(crc >> 8);
        tr[2] = (uint8_t)(crc >> 16);
        tr[3] = (uint8_t)(crc >> 24);
    }
    zhip_status st = {ZHIP_ST_OK, crc, crc, 0u};
    p.status[c] = st;
}

// k_encode_tile: the general transposed encode (TransposeCodec._encode_sync,
// transpose.py:113-118) for layouts k_encode_tile4 does not take -- partial
// tiles (shape[tq] % 64, row_bytes % 256), any number of tiles per chunk, any
// base steps -- and for edge chunks whose selection is a prefix box (start 0,
// unit steps: the array covers [0, count) of every stored dim, the rest of the
// chunk is fill, as _merge_chunk_array writes it).  Up to four consecutive
// 64-row x 256-byte tiles of one chunk per workgroup, every gather issued
// first: the array's out-contiguous 16-byte pieces (kPer rows of the tq dim at
// one column element) go into the LDS image at their stored place and come
// back as stored 16-byte blocks (fill test, byteswap, store, Horner steps with
// k_decode_tile's stride tables).  A thread's per-tile states are shifted by
// the tile constants and summed (CRC linearity), so one reduction and one
// XOR + arrival pair per workgroup remain; the last arrival writes the
// trailer and the status.
namespace {
struct TileGeo {
    uint32_t tbase;
    int64_t aoff;
    int32_t rows_here, cols_here, rows_sel, cols_sel;  // cols_sel in elements
};
}  // namespace

template <int ITEM>
__device__ __forceinline__ TileGeo encode_tile_geo(const EncodeParams& p, uint32_t ti, const int32_t (&cnt)[ZHIP_MAX_DIMS],
                                                   int32_t cnt_q, int32_t cnt_l) {
    const int32_t last = p.g.ndim - 1;
    const uint32_t sq = p.sstride[p.tq];
    uint32_t r = ti;
    const uint32_t rq = fdiv_apply(r, p.d_cb.m, p.d_cb.s);
    const uint32_t cb = r - rq * p.n_cb;
    r = rq;
    const uint32_t rr = fdiv_apply(r, p.d_qb.m, p.d_qb.s);
    const uint32_t qb = r - rr * p.n_qb;
    r = rr;
    TileGeo g;
    g.tbase = qb * (uint32_t)kTileRows * sq + cb * (uint32_t)kTileCols;
    g.aoff = (int64_t)qb * kTileRows * p.g.ostride[p.tq] + (int64_t)(cb * (kTileCols / ITEM)) * p.g.ostride[last];
    bool inside = true;
#pragma unroll
    for (int d = ZHIP_MAX_DIMS - 1; d >= 0; --d) {
        if (d >= last || d == p.tq) continue;
        const uint32_t qd = fdiv_apply(r, p.g.dshape[d].m, p.g.dshape[d].s);
        const uint32_t sd = r - qd * (uint32_t)p.g.shape[d];
        r = qd;
        g.tbase += sd * p.sstride[d];
        g.aoff += (int64_t)sd * p.g.ostride[d];
        inside = inside && (int32_t)sd < cnt[d];
    }
    g.rows_here = min(kTileRows, p.g.shape[p.tq] - (int32_t)qb * kTileRows);
    g.cols_here = min(kTileCols, (int32_t)p.g.row_bytes - (int32_t)cb * kTileCols);
    g.rows_sel = inside ? max(0, min(g.rows_here, cnt_q - (int32_t)qb * kTileRows)) : 0;
    g.cols_sel = max(0, min(g.cols_here / ITEM, cnt_l - (int32_t)cb * (kTileCols / ITEM)));
    return g;
}

template <bool CRC, int ITEM, bool SWAP>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_encode_tile(
    const EncodeParams p) {
    constexpr int kPer = 16 / ITEM;
    constexpr int kPiecesPerCol = kTileRows / kPer;
    constexpr int G = kTiles;  // tiles per workgroup
    __shared__ uint32_t s_tab[CRC ? 16 * 256 : 1];
    __shared__ __attribute__((aligned(16))) uint8_t s_tile[kTileRows * 256];
    __shared__ uint32_t s_red[kThreads / 64];
    __shared__ uint32_t s_ne[kThreads / 64];
    struct Counts {
        int32_t v[ZHIP_MAX_DIMS];
    };
    const int t = threadIdx.x;
    const uint32_t T = p.t_per_chunk;
    const uint32_t gpc = (T + G - 1) / G;  // workgroups per chunk
    const uint32_t c = blockIdx.x / gpc;
    const uint32_t grp = blockIdx.x - c * gpc;
    const uint32_t ti0 = grp * G;
    const uint32_t nt = min((uint32_t)G, T - ti0);  // tiles of this workgroup
    uint4 tv0, tv1, tv2, tv3;
    uint32_t kth = 0;
    if constexpr (CRC) {
        const uint4* gt = reinterpret_cast<const uint4*>(p.horner);
        tv0 = gt[t];
        tv1 = gt[t + kThreads];
        tv2 = gt[t + 2 * kThreads];
        tv3 = gt[t + 3 * kThreads];
        kth = p.kthread[t];
    }
    const zhip_chunk ch = load_uniform<zhip_chunk>(p.chunks + c);  // src: dst offset, out_off: array offset
    const Counts cs = load_uniform<Counts>(&p.sels[ch.sel].count[0]);
    const int32_t last = p.g.ndim - 1;
    int32_t cnt_q = 0, cnt_l = 0;  // (select by compile-time index: no dynamic indexing of registers)
#pragma unroll
    for (int d = 0; d < ZHIP_MAX_DIMS; ++d) {
        cnt_q = d == p.tq ? cs.v[d] : cnt_q;
        cnt_l = d == last ? cs.v[d] : cnt_l;
    }
    TileGeo geo[G];
#pragma unroll
    for (int j = 0; j < G; ++j) geo[j] = encode_tile_geo<ITEM>(p, ti0 + min((uint32_t)j, nt - 1u), cs.v, cnt_q, cnt_l);
    const uint32_t sq = p.sstride[p.tq];
    const int64_t oq = p.g.ostride[p.tq];    // == ITEM
    const int64_t ocol = p.g.ostride[last];  // array stride of the innermost stored dim
    const uint8_t* const abase = p.arr + ch.out_off;
    uint8_t* const cp = p.dst + ch.src;
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
    // 1. gather every whole piece of the workgroup's tiles (the rest: fill;
    //    pieces crossing the selection's row end are completed in step 2)
    //    Every lane issues every load (a dummy address where the piece is not
    //    whole) and picks the fill only when the tile is consumed: a select
    //    right after a conditional load would wait for it, serialising them.
    uint4 pcs[G][kPasses];
    uint32_t wmask = 0;  // bit j * kPasses + k: piece (j, k) was loaded whole
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_tile_zero);
#pragma unroll
    for (int j = 0; j < G; ++j)
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const int32_t pc = k * kThreads + t;
            const int32_t jc = pc / kPiecesPerCol;
            const int32_t r0 = (pc % kPiecesPerCol) * kPer;
            const bool whole = (uint32_t)j < nt && jc < geo[j].cols_sel && r0 + kPer <= geo[j].rows_sel;
            wmask |= whole ? 1u << (j * kPasses + k) : 0u;
            pcs[j][k] = load_stream16_a1(whole ? abase + geo[j].aoff + (int64_t)jc * ocol + (int64_t)r0 * oq : zero);
        }
    if constexpr (CRC) {
        uint4* st = reinterpret_cast<uint4*>(s_tab);
        st[t] = tv0;
        st[t + kThreads] = tv1;
        st[t + 2 * kThreads] = tv2;
        st[t + 3 * kThreads] = tv3;
    }
    const uint32_t row0 = (uint32_t)t >> 4, col = 16u * (uint32_t)(t & 15);
    uint32_t S = 0;  // sum over tiles of this thread's tile state x tile constant
    bool eq = true;
#pragma unroll
    for (int j = 0; j < G; ++j) {
        if ((uint32_t)j >= nt) break;
        if (j > 0) __syncthreads();  // the previous tile's LDS reads are done
        // 2. pieces into the LDS image at their stored (row, column) place;
        //    pieces crossing the selection's row end are gathered element by
        //    element here (only this tile's loads are waited for)
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint32_t pc = (uint32_t)(k * kThreads + t);
            const uint32_t jc = pc / kPiecesPerCol;
            const uint32_t r0 = (pc % kPiecesPerCol) * kPer;
            const uint4 pv = (wmask >> (j * kPasses + k)) & 1u ? pcs[j][k] : f;
            uint32_t w[4] = {pv.x, pv.y, pv.z, pv.w};
            const int32_t rs = geo[j].rows_sel;
            if ((int32_t)jc < geo[j].cols_sel && (int32_t)r0 < rs && (int32_t)r0 + kPer > rs) {
                const uint8_t* a = abase + geo[j].aoff + (int64_t)jc * ocol + (int64_t)r0 * oq;
                for (int32_t e = 0; e < rs - (int32_t)r0; ++e) {
                    if constexpr (ITEM == 8) {
                        const uint2 v = *reinterpret_cast<const uint2*>(a + 8 * e);
                        w[2 * e] = v.x;
                        w[2 * e + 1] = v.y;
                    } else if constexpr (ITEM == 4) {
                        w[e] = *reinterpret_cast<const uint32_t*>(a + 4 * e);
                    } else if constexpr (ITEM == 2) {
                        const uint32_t sh = 16 * (e & 1);
                        w[e / 2] = (w[e / 2] & ~(0xFFFFu << sh)) |
                                   ((uint32_t)*reinterpret_cast<const uint16_t*>(a + 2 * e) << sh);
                    } else {
                        const uint32_t sh = 8 * (e & 3);
                        w[e / 4] = (w[e / 4] & ~(0xFFu << sh)) | ((uint32_t)a[e] << sh);
                    }
                }
            }
#pragma unroll
            for (int e = 0; e < kPer; ++e) {
                uint8_t* dst = s_tile + tile_byte<ITEM>(r0 + e, jc * ITEM);
                if constexpr (ITEM == 8) {
                    *reinterpret_cast<uint2*>(dst) = make_uint2(w[2 * e], w[2 * e + 1]);
                } else if constexpr (ITEM == 4) {
                    *reinterpret_cast<uint32_t*>(dst) = w[e];
                } else if constexpr (ITEM == 2) {
                    *reinterpret_cast<uint16_t*>(dst) = (uint16_t)(w[e / 2] >> (16 * (e & 1)));
                } else {
                    *dst = (uint8_t)(w[e / 4] >> (8 * (e & 3)));
                }
            }
        }
        __syncthreads();  // tile j (and, first time, the tables) in LDS
        // 3. stored-order blocks inside the chunk: fill test, byteswap, store,
        //    Horner steps (blocks past the chunk's rows / row end count as zeros)
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint32_t row = 16u * k + row0;
            uint4 e = make_uint4(0, 0, 0, 0);
            if ((int32_t)row < geo[j].rows_here && (int32_t)col < geo[j].cols_here) {
                const uint4 v = tile_get16<ITEM>(s_tile, row, col);
                eq = eq && block_eq_fill_e<ITEM>(v, p);
                e = swap_block<ITEM, SWAP>(v);
                store_nt16_a1(cp + geo[j].tbase + row * sq + col, e);
            }
            if constexpr (CRC)
                acc = tab_apply(s_tab, acc ^ e.x) ^ tab_apply(s_tab + 1024, e.y) ^ tab_apply(s_tab + 2048, e.z) ^
                      tab_apply(s_tab + 3072, e.w);
        }
        if constexpr (CRC) S ^= gf_mul(acc, __builtin_amdgcn_readfirstlane(p.kunit[ti0 + j]));
    }
    // 4. the workgroup's contribution and arrival
    uint32_t v = 0;
    if constexpr (CRC) v = wave_xor(gf_mul(S, kth));
    const bool wne = __any(!eq);
    if ((t & 63) == 0) {
        s_red[t >> 6] = v;
        s_ne[t >> 6] = wne ? 1u : 0u;
    }
    __syncthreads();
    if (t != 0) return;
    // arrival word: workgroups arrived (low 16 bits) | non-empty ones (high 16)
    const bool ne = (s_ne[0] | s_ne[1] | s_ne[2] | s_ne[3]) != 0u;
    uint32_t* accw = p.ws + 4ull * c;
    if constexpr (CRC) {
        const uint32_t V = s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3];
        const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
    }
    const uint32_t tk = __hip_atomic_fetch_add(accw + 2, ne ? 0x10001u : 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
    if ((tk & 0xFFFFu) + 1u != gpc) return;
    __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    p.nonempty[c] = ((tk >> 16) != 0u || ne) ? 1u : 0u;
    if constexpr (CRC) {
        const uint32_t raw = __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t crc = ~(gf_mul(raw, p.c_inv) ^ p.c3);
        uint8_t* tr = cp + p.g.nbytes;  // LE trailer (crc32c_.py:64-68)
        tr[0] = (uint8_t)crc;
        tr[1] = (uint8_t)(crc >> 8);
        tr[2] = (uint8_t)(crc >> 16);
        tr[3] = (uint8_t)(crc >> 24);
        zhip_status st = {ZHIP_ST_OK, crc, crc, 0u};
        p.status[c] = st;
    } else {
        zhip_status st = {ZHIP_ST_OK, 0u, 0u, 0u};
        p.status[c] = st;
    }
}

// k_encode_tileg: k_encode_tile4's recipe for every other transposed layout
// with full selections, as long as some stored dim gd (not tq, not the
// innermost) has shape % 4 == 0: the tiles are grouped by four along gd, so
// inside a group the stored (and array) offsets step uniformly -- one table
// multiply carries a thread's CRC state from tile to tile whatever the natural
// tile order -- and partial tiles (shape[tq] % 64, row_bytes % 256) are masked
// (the group's tiles share their row / byte extent).  Per workgroup: one
// 24-byte group record (scalar), all 16 loads per thread issued first (a dummy
// line outside the tile), per tile LDS image -> stored blocks -> fill test,
// byteswap, store, Horner; one lane multiply, one reduction, one XOR + arrival
// pair per workgroup (any number of groups per chunk).
// NT: tiles per workgroup -- 4, or 2 (two workgroups per group: two
// residency rounds; the first half's contribution shifted by p.g_z2 to the
// group's last-tile frame that ge.ku assumes; arrival subwords for twice the
// workgroups, zhip_plan_info)
// LB (tuning arm 63): tileg_arrive_lb instead of the returning arrival
// A4C (tuning arm 68): four word accumulators per lane through the ONE
//   operator A_(16 sq) (the first of the four byte-table operators) instead of
//   one accumulator through four, folded per tile by the A4 tables
//   (fold4_t: the state x^96 times the single accumulator's, undone by g_c96
//   in the lane multiply): 16 + 4 lookups per tile more, 8 KiB of tables
//   instead of 16 -- 28 KiB of LDS, five workgroups per CU instead of four
template <bool CRC, int ITEM, bool SWAP, int NT = kTiles, bool SPR = false, bool LB = false, bool A4C = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_encode_tileg(
    const EncodeParams p) {
    constexpr int kPer = 16 / ITEM;
    constexpr int kPiecesPerCol = kTileRows / kPer;
    __shared__ uint32_t s_tab[CRC ? (A4C ? 2048 : 16 * 256) : 1];
    __shared__ uint32_t s_tz[CRC ? 1024 : 1];
    __shared__ __attribute__((aligned(16))) uint8_t s_tile[kTileRows * 256];
    __shared__ uint32_t s_red[kThreads / 64];
    __shared__ uint32_t s_ne[kThreads / 64];
    const int t = threadIdx.x;
    constexpr uint32_t PG = kTiles / NT;  // workgroups per group of four tiles
    const uint32_t gpc = p.n_groups * PG;   // workgroups per chunk
    const uint32_t c = blockIdx.x / gpc;
    const uint32_t wg = blockIdx.x - c * gpc;
    const uint32_t grp = wg / PG, t0 = (wg % PG) * NT;  // the group and its first tile here
    uint4 tv0, tv1, tv2, tv3, tzv;
    uint32_t kth = 0;
    if constexpr (CRC) {
        const uint4* gt = reinterpret_cast<const uint4*>(p.horner);
        tv0 = gt[t];
        if constexpr (A4C) {
            tv1 = reinterpret_cast<const uint4*>(p.g_a4)[t];
        } else {
            tv1 = gt[t + kThreads];
            tv2 = gt[t + 2 * kThreads];
            tv3 = gt[t + 3 * kThreads];
        }
        tzv = reinterpret_cast<const uint4*>(p.gtz)[t];
        kth = p.kthread[t];
    }
    const zhip_chunk ch = load_uniform<zhip_chunk>(p.chunks + c);  // src: dst offset, out_off: array offset
    const GroupEnt ge = load_uniform<GroupEnt>(p.gmap + grp);
    const int32_t last = p.g.ndim - 1;
    const int64_t oq = p.g.ostride[p.tq];    // == ITEM
    const int64_t ocol = p.g.ostride[last];  // array stride of the innermost stored dim
    const uint32_t sq = p.sstride[p.tq];
    const uint8_t* const abase = p.arr + ch.out_off + ge.orel;
    uint8_t* const cp = p.dst + ch.src + ge.tbase;
    const int32_t rows = ge.rows, cols = ge.cols;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_tile_zero);
    // 1. every load of the workgroup's tiles (pieces outside the tile read a dummy line)
    uint4 pcs[NT][kPasses];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const int32_t pc = k * kThreads + t;
            const int32_t jc = pc / kPiecesPerCol;
            const int32_t r0 = (pc % kPiecesPerCol) * kPer;
            const bool in = jc * ITEM < cols && r0 < rows;  // rows % kPer == 0 (zhip_encode_mapped)
            pcs[j][k] = load_stream16_a1(in ? abase + (int64_t)(t0 + j) * p.g_step_o + (int64_t)jc * ocol +
                                                  (int64_t)r0 * oq
                                        : zero);
        }
    if constexpr (CRC) {
        uint4* st = reinterpret_cast<uint4*>(s_tab);
        st[t] = tv0;
        st[t + kThreads] = tv1;
        if constexpr (!A4C) {
            st[t + 2 * kThreads] = tv2;
            st[t + 3 * kThreads] = tv3;
        }
        reinterpret_cast<uint4*>(s_tz)[t] = tzv;
    }
    const uint32_t row0 = (uint32_t)t >> 4, col = 16u * (uint32_t)(t & 15);
    uint32_t S = 0;
    bool eq = true;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        if (j > 0) __syncthreads();  // the previous tile's LDS reads are done
        // 2. pieces into the LDS image at their stored (row, column) place
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint32_t pc = (uint32_t)(k * kThreads + t);
            const uint32_t jc = pc / kPiecesPerCol;
            const uint32_t r0 = (pc % kPiecesPerCol) * kPer;
            const uint32_t w[4] = {pcs[j][k].x, pcs[j][k].y, pcs[j][k].z, pcs[j][k].w};
#pragma unroll
            for (int e = 0; e < kPer; ++e) {
                uint8_t* dst = s_tile + tile_byte<ITEM>(r0 + e, jc * ITEM);
                if constexpr (ITEM == 8) {
                    *reinterpret_cast<uint2*>(dst) = make_uint2(w[2 * e], w[2 * e + 1]);
                } else if constexpr (ITEM == 4) {
                    *reinterpret_cast<uint32_t*>(dst) = w[e];
                } else if constexpr (ITEM == 2) {
                    *reinterpret_cast<uint16_t*>(dst) = (uint16_t)(w[e / 2] >> (16 * (e & 1)));
                } else {
                    *dst = (uint8_t)(w[e / 4] >> (8 * (e & 3)));
                }
            }
        }
        __syncthreads();  // tile j (and, first time, the tables) in LDS
        // 3. stored-order blocks inside the tile: fill test, byteswap, store,
        //    Horner steps (blocks outside the tile count as zeros)
        uint32_t acc = 0;
        Acc4 a4 = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < kPasses; ++k) {
            const uint32_t row = 16u * k + row0;
            uint4 e = make_uint4(0, 0, 0, 0);
            if ((int32_t)row < rows && (int32_t)col < cols) {
                const uint4 v = tile_get16<ITEM>(s_tile, row, col);
                eq = eq && block_eq_fill_e<ITEM>(v, p);
                e = swap_block<ITEM, SWAP>(v);
                store_nt16_a1(cp + (size_t)(t0 + j) * p.g_step_t + row * sq + col, e);
            }
            if constexpr (CRC && A4C) {
                crc_block4_t<true>(s_tab, a4, e);
            } else if constexpr (CRC) {
                acc = tab_apply(s_tab, acc ^ e.x) ^ tab_apply(s_tab + 1024, e.y) ^ tab_apply(s_tab + 2048, e.z) ^
                      tab_apply(s_tab + 3072, e.w);
            }
        }
        if constexpr (CRC && A4C) acc = fold4_t<true>(s_tab, a4);  // x^96 times the single accumulator
        if constexpr (CRC) S = (j == 0 ? 0u : tab_apply(s_tz, S)) ^ acc;
    }
    // 4. run end: lane shift, reduction, the group's tile / chunk-end shift
    uint32_t v = 0;
    if constexpr (CRC) v = wave_xor(gf_mul(S, A4C ? gf_mul(kth, p.g_c96) : kth));
    const bool wne = __any(!eq);
    if ((t & 63) == 0) {
        s_red[t >> 6] = v;
        s_ne[t >> 6] = wne ? 1u : 0u;
    }
    __syncthreads();
    if (t != 0) return;
    // the last arrival writes the chunk's non-empty flag (no zeroing pass)
    const bool ne = (s_ne[0] | s_ne[1] | s_ne[2] | s_ne[3]) != 0u;
    uint8_t* const chunk = p.dst + ch.src;
    uint32_t raw = 0;
    uint32_t V = 0;
    if constexpr (CRC) {
        const uint32_t ku = (NT == 2 && t0 == 0) ? gf_mul(ge.ku, p.g_z2) : ge.ku;
        V = gf_mul(s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3], ku);
    }
    const uint32_t nsub = NT == kTiles ? p.n_sub : ((gpc > 16u && gpc <= 256u) ? (gpc + 15u) / 16u : 0u);
    if (gpc <= 16u || nsub) {
        bool any_ne = false;
        if (LB) {
            if (!tileg_arrive_lb(p.ws, p.n_chunks, c, wg, gpc, nsub, V, ne, raw, any_ne)) return;
        } else if (!tileg_arrive<SPR>(p.ws, p.n_chunks, c, wg, gpc, nsub, V, ne, raw, any_ne)) {
            return;
        }
        p.nonempty[c] = any_ne ? 1u : 0u;
    } else {  // more than 256 groups per chunk: arrival count | non-empty count word
        uint32_t* accw = p.ws + 4ull * c;
        if constexpr (CRC) {
            const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
        }
        const uint32_t tk = __hip_atomic_fetch_add(accw + 2, ne ? 0x10001u : 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
        if ((tk & 0xFFFFu) + 1u != gpc) return;
        __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        p.nonempty[c] = ((tk >> 16) != 0u || ne) ? 1u : 0u;
        if constexpr (CRC) raw = __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (CRC) {
        const uint32_t crc = ~(raw ^ p.c3);  // ku carries t_c_inv
        uint8_t* tr = chunk + p.g.nbytes;    // LE trailer (crc32c_.py:64-68)
        tr[0] = (uint8_t)crc;
        tr[1] = (uint8_t)(crc >> 8);
        tr[2] = (uint8_t)(crc >> 16);
        tr[3] = (uint8_t)(crc >> 24);
        zhip_status st = {ZHIP_ST_OK, crc, crc, 0u};
        p.status[c] = st;
    } else {
        zhip_status st = {ZHIP_ST_OK, 0u, 0u, 0u};
        p.status[c] = st;
    }
}

using KernelFn = void (*)(const DecodeParams);
using EncodeFn = void (*)(const EncodeParams);

EncodeFn select_encode_tileg_kernel(bool crc, int item, bool swap, int nt) {
#if ZHIP_TUNING
    if (nt == 6 || nt == 7 || nt == 8 || nt == 9) {  // arms 47 / 50: four / two tiles, arrival words on
        // lines of their own; arm 63 (8): four tiles, the look-back finalizer; arm 68 (9): four
        // accumulators through one byte-table operator
        if (!crc) return nullptr;
#define ZHIP_ETG(I, W)                                                                                      \
    (nt == 6 ? k_encode_tileg<true, I, W, 4, true> : nt == 8 ? k_encode_tileg<true, I, W, 4, true, true>    \
     : nt == 9 ? k_encode_tileg<true, I, W, 4, false, false, true> : k_encode_tileg<true, I, W, 2, true>)
        switch (item) {
            case 1: return ZHIP_ETG(1, false);
            case 2: return swap ? ZHIP_ETG(2, true) : ZHIP_ETG(2, false);
            case 4: return swap ? ZHIP_ETG(4, true) : ZHIP_ETG(4, false);
            case 8: return swap ? ZHIP_ETG(8, true) : ZHIP_ETG(8, false);
            default: return nullptr;
        }
#undef ZHIP_ETG
    }
#endif
    if (nt == 2) {  // CRC layouts only
        if (!crc) return nullptr;
        switch (item) {
            case 1: return k_encode_tileg<true, 1, false, 2>;
            case 2: return swap ? k_encode_tileg<true, 2, true, 2> : k_encode_tileg<true, 2, false, 2>;
            case 4: return swap ? k_encode_tileg<true, 4, true, 2> : k_encode_tileg<true, 4, false, 2>;
            case 8: return swap ? k_encode_tileg<true, 8, true, 2> : k_encode_tileg<true, 8, false, 2>;
            default: return nullptr;
        }
    }
    switch (item) {
        case 1: return crc ? k_encode_tileg<true, 1, false> : k_encode_tileg<false, 1, false>;
        case 2: return crc ? (swap ? k_encode_tileg<true, 2, true> : k_encode_tileg<true, 2, false>)
                           : (swap ? k_encode_tileg<false, 2, true> : k_encode_tileg<false, 2, false>);
        case 4: return crc ? (swap ? k_encode_tileg<true, 4, true> : k_encode_tileg<true, 4, false>)
                           : (swap ? k_encode_tileg<false, 4, true> : k_encode_tileg<false, 4, false>);
        case 8: return crc ? (swap ? k_encode_tileg<true, 8, true> : k_encode_tileg<true, 8, false>)
                           : (swap ? k_encode_tileg<false, 8, true> : k_encode_tileg<false, 8, false>);
        default: return nullptr;
    }
}

EncodeFn select_encode_tile_kernel(bool crc, int item, bool swap) {
    switch (item) {
        case 1: return crc ? k_encode_tile<true, 1, false> : k_encode_tile<false, 1, false>;
        case 2: return crc ? (swap ? k_encode_tile<true, 2, true> : k_encode_tile<true, 2, false>)
                           : (swap ? k_encode_tile<false, 2, true> : k_encode_tile<false, 2, false>);
        case 4: return crc ? (swap ? k_encode_tile<true, 4, true> : k_encode_tile<true, 4, false>)
                           : (swap ? k_encode_tile<false, 4, true> : k_encode_tile<false, 4, false>);
        case 8: return crc ? (swap ? k_encode_tile<true, 8, true> : k_encode_tile<true, 8, false>)
                           : (swap ? k_encode_tile<false, 8, true> : k_encode_tile<false, 8, false>);
        default: return nullptr;
    }
}

// nt = 2: the two-tile form (CRC layouts whose plan built its constants)
EncodeFn select_encode_tile4_kernel(bool crc, int item, bool swap, int nt) {
    if (nt == 2) {
        if (!crc) return nullptr;
        switch (item) {
            case 1: return k_encode_tile4<true, 1, false, 2>;
            case 2: return swap ? k_encode_tile4<true, 2, true, 2> : k_encode_tile4<true, 2, false, 2>;
            case 4: return swap ? k_encode_tile4<true, 4, true, 2> : k_encode_tile4<true, 4, false, 2>;
            case 8: return swap ? k_encode_tile4<true, 8, true, 2> : k_encode_tile4<true, 8, false, 2>;
            default: return nullptr;
        }
    }
    switch (item) {
        case 1: return crc ? k_encode_tile4<true, 1, false> : k_encode_tile4<false, 1, false>;
        case 2: return crc ? (swap ? k_encode_tile4<true, 2, true> : k_encode_tile4<true, 2, false>)
                           : (swap ? k_encode_tile4<false, 2, true> : k_encode_tile4<false, 2, false>);
        case 4: return crc ? (swap ? k_encode_tile4<true, 4, true> : k_encode_tile4<true, 4, false>)
                           : (swap ? k_encode_tile4<false, 4, true> : k_encode_tile4<false, 4, false>);
        case 8: return crc ? (swap ? k_encode_tile4<true, 8, true> : k_encode_tile4<true, 8, false>)
                           : (swap ? k_encode_tile4<false, 8, true> : k_encode_tile4<false, 8, false>);
        default: return nullptr;
    }
}

// defer: ZHIP_DF_DEFER (deferred CRC verdicts, PUB 2); otherwise the returning
// publication (PUB 0), whose launch reports a mismatch itself
KernelFn select_tileg_kernel(bool crc, int item, bool swap, bool defer) {
    if (!crc) {
        switch (item) {
            case 1: return k_decode_tileg<false, 1, false>;
            case 2: return swap ? k_decode_tileg<false, 2, true> : k_decode_tileg<false, 2, false>;
            case 4: return swap ? k_decode_tileg<false, 4, true> : k_decode_tileg<false, 4, false>;
            case 8: return swap ? k_decode_tileg<false, 8, true> : k_decode_tileg<false, 8, false>;
            default: return nullptr;
        }
    }
#define ZHIP_TILEG(I, W) (defer ? k_decode_tileg<true, I, W, 2> : k_decode_tileg<true, I, W, 0>)
    switch (item) {
        case 1: return ZHIP_TILEG(1, false);
        case 2: return swap ? ZHIP_TILEG(2, true) : ZHIP_TILEG(2, false);
        case 4: return swap ? ZHIP_TILEG(4, true) : ZHIP_TILEG(4, false);
        case 8: return swap ? ZHIP_TILEG(8, true) : ZHIP_TILEG(8, false);
        default: return nullptr;
    }
#undef ZHIP_TILEG
}

KernelFn select_tilegw_kernel(int item, bool swap, bool defer, int nt) {  // CRC chains only
// (nt 2: the two-tile form, always the returning publication on spread lines;
// tuning: 6 the same on packed words, 5 lanes pick the tile)
#if ZHIP_TUNING
#define ZHIP_TILEGW(I, W)                                                                          \
    (nt == 2 ? k_decode_tilegw<I, W, 0, 2, false, true>                                             \
     : nt == 7 ? k_decode_tilegw<I, W, 0, 2, false, true, true>                                     \
     : nt == 8 ? k_decode_tilegw<I, W, 0, 2, false, true, false, true>                              \
     : nt == 5 ? (defer ? k_decode_tilegw<I, W, 2, 4, true> : k_decode_tilegw<I, W, 0, 4, true>)   \
     : nt == 6 ? k_decode_tilegw<I, W, 0, 2>                                                        \
             : (defer ? k_decode_tilegw<I, W, 2> : k_decode_tilegw<I, W, 0>))
#else
#define ZHIP_TILEGW(I, W)                                                                          \
    (nt == 2 ? k_decode_tilegw<I, W, 0, 2, false, true>                                             \
             : (defer ? k_decode_tilegw<I, W, 2> : k_decode_tilegw<I, W, 0>))
#endif
    switch (item) {
        case 1: return ZHIP_TILEGW(1, false);
        case 2: return swap ? ZHIP_TILEGW(2, true) : ZHIP_TILEGW(2, false);
        case 4: return swap ? ZHIP_TILEGW(4, true) : ZHIP_TILEGW(4, false);
        case 8: return swap ? ZHIP_TILEGW(8, true) : ZHIP_TILEGW(8, false);
        default: return nullptr;
    }
#undef ZHIP_TILEGW
}

KernelFn select_tile4w_kernel(int item, bool swap) {  // CRC chains only
    switch (item) {
        case 1: return k_decode_tile4w<1, false>;
        case 2: return swap ? k_decode_tile4w<2, true> : k_decode_tile4w<2, false>;
        case 4: return swap ? k_decode_tile4w<4, true> : k_decode_tile4w<4, false>;
        case 8: return swap ? k_decode_tile4w<8, true> : k_decode_tile4w<8, false>;
        default: return nullptr;
    }
}

// two tiles per workgroup (production where the plan built its constants);
// the tuning build adds one tile per workgroup (arm 37)
KernelFn select_tile2w_kernel(int item, bool swap, int nt) {  // CRC chains only
#if ZHIP_TUNING
#define ZHIP_T2W(I, W)                                                                                  \
    (nt == 1 ? k_decode_tile4w<I, W, 1> : nt == 3 ? k_decode_tile4w<I, W, 2, true>                       \
     : nt == 4 ? k_decode_tile4w<I, W, 2, false, true> : k_decode_tile4w<I, W, 2>)
#else
    if (nt != 2) return nullptr;
#define ZHIP_T2W(I, W) k_decode_tile4w<I, W, 2>
#endif
    switch (item) {
        case 1: return ZHIP_T2W(1, false);
        case 2: return swap ? ZHIP_T2W(2, true) : ZHIP_T2W(2, false);
        case 4: return swap ? ZHIP_T2W(4, true) : ZHIP_T2W(4, false);
        case 8: return swap ? ZHIP_T2W(8, true) : ZHIP_T2W(8, false);
        default: return nullptr;
    }
#undef ZHIP_T2W
}

#if ZHIP_TUNING
KernelFn select_tile4f_kernel(int item, bool swap) {  // CRC chains only
    switch (item) {
        case 1: return k_decode_tile4f<1, false>;
        case 2: return swap ? k_decode_tile4f<2, true> : k_decode_tile4f<2, false>;
        case 4: return swap ? k_decode_tile4f<4, true> : k_decode_tile4f<4, false>;
        case 8: return swap ? k_decode_tile4f<8, true> : k_decode_tile4f<8, false>;
        default: return nullptr;
    }
}
#endif

KernelFn select_tile4_kernel(bool crc, int item, bool swap) {
#if ZHIP_TUNING
    if (g_tune_arm == 1 && crc && item == 4 && !swap) return k_decode_tile4<true, 4, false, 0>;  // words 16 B apart
    if (g_tune_arm == 2 && crc && item == 4 && !swap) return k_decode_tile4<true, 4, false, 2>;  // deferred arm
#endif
    switch (item) {
        case 1: return crc ? k_decode_tile4<true, 1, false> : k_decode_tile4<false, 1, false>;
        case 2: return crc ? (swap ? k_decode_tile4<true, 2, true> : k_decode_tile4<true, 2, false>)
                           : (swap ? k_decode_tile4<false, 2, true> : k_decode_tile4<false, 2, false>);
        case 4: return crc ? (swap ? k_decode_tile4<true, 4, true> : k_decode_tile4<true, 4, false>)
                           : (swap ? k_decode_tile4<false, 4, true> : k_decode_tile4<false, 4, false>);
        case 8: return crc ? (swap ? k_decode_tile4<true, 8, true> : k_decode_tile4<true, 8, false>)
                           : (swap ? k_decode_tile4<false, 8, true> : k_decode_tile4<false, 8, false>);
        default: return nullptr;
    }
}

}  // namespace zhip
