// Fused zarr v3 encode for MI355X (gfx950): gather each chunk from a device
// array (transpose folded into the stored-dim strides), byteswap to the stored
// endian, write the encoded bytes, append the CRC-32C trailer and flag chunks
// that equal the fill value; plus the shard packer (Morton-ordered layout,
// empty-chunk elision, index + index CRC).
//
// Reference behaviour restated (file:line under /root/reference):
//   _merge_chunk_array (edge chunks: outside the selection = fill)
//                                   src/zarr/core/chunk_utils.py:115-162
//   chunk_is_empty / all_equal      chunk_utils.py:74-85, src/zarr/core/buffer/core.py:534-558
//   TransposeCodec._encode_sync     src/zarr/codecs/transpose.py:113-118
//   BytesCodec._encode_sync         src/zarr/codecs/bytes.py:140-158
//   Crc32cCodec._encode_sync        src/zarr/codecs/crc32c_.py:59-68
//   ShardingCodec._build_shard_layout / _assemble_shard / _encode_shard_index_sync
//                                   src/zarr/codecs/sharding.py:887-950, 633-640
//   Morton order                    src/zarr/core/indexing.py:1578-1643 (rank table from host)
//
// The unit decomposition and CRC combine are those of decode.hip (see there):
// the stored byte stream [0, N) is cut into end-aligned units of 4 KiB * K,
// thread t of a unit owns the 16-byte blocks at lo + 16t + 4096k.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/zarrhip.h"
#include "zhip_device.h"
#include "zhip_gf2.h"
#include "zhip_internal.h"
#include "zhip_decode_common.h"

namespace zhip {

// Element equality with the fill value as NDBuffer.all_equal defines it:
// bitwise, except that any NaN equals a NaN fill (equal_nan=True); a 0.0 fill
// compares bit patterns (so -0.0 != 0.0), which bitwise equality gives.
template <int ITEM>
__device__ __forceinline__ bool item_eq_fill(uint32_t lo, uint32_t hi, const EncodeParams& p) {
    if constexpr (ITEM == 8) {
        const bool eq = lo == p.fill[0] && hi == p.fill[1];
        if (!p.fill_nan) return eq;
        const uint64_t v = ((uint64_t)hi << 32) | lo;
        return eq || (v & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull;
    } else {
        constexpr uint32_t mask = ITEM == 4 ? 0xFFFFFFFFu : ((1u << (8 * ITEM)) - 1u);
        const bool eq = (lo & mask) == (p.fill[0] & mask);
        if (!p.fill_nan) return eq;
        if constexpr (ITEM == 4) return eq || (lo & 0x7FFFFFFFu) > 0x7F800000u;
        if constexpr (ITEM == 2) return eq || (lo & 0x7FFFu) > 0x7C00u;
        return eq;
    }
}

template <int ITEM>
__device__ __forceinline__ bool block_eq_fill(uint4 v, uint32_t valid, const EncodeParams& p) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    bool all = true;
    constexpr int kItems = 16 / ITEM;
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        if ((uint32_t)(j * ITEM) >= valid) break;
        uint32_t lo, hi = 0;
        if constexpr (ITEM == 8) {
            lo = w[2 * j];
            hi = w[2 * j + 1];
        } else {
            lo = w[(j * ITEM) / 4] >> (8 * ((j * ITEM) % 4));
        }
        all = all && item_eq_fill<ITEM>(lo, hi, p);
    }
    return all;
}

template <int ITEM>
__device__ __forceinline__ void load_item(const uint8_t* src, uint32_t& lo, uint32_t& hi) {
    if constexpr (ITEM == 1) lo = *src;
    else if constexpr (ITEM == 2) lo = *reinterpret_cast<const uint16_t*>(src);
    else if constexpr (ITEM == 4) lo = *reinterpret_cast<const uint32_t*>(src);
    else {
        const uint2 v = *reinterpret_cast<const uint2*>(src);
        lo = v.x;
        hi = v.y;
    }
}

// Gather the 16 stored bytes [o, o+16) of a chunk from the array (native
// order): selected elements from `arr`, the rest = fill.
template <int ITEM, bool FAST>
__device__ __forceinline__ uint4 gather_block(const EncodeParams& p, const zhip_sel& s, int64_t arr_off,
                                              int32_t o) {
    if constexpr (FAST) {
        const uint32_t r = fdiv_apply((uint32_t)o, p.g.drow.m, p.g.drow.s);
        const uint32_t col = (uint32_t)o - r * p.g.row_bytes;
        int64_t src = arr_off + col;
        if (!sel_offset(p.g, s, r, p.g.ndim - 2, src)) return make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
        return *reinterpret_cast<const uint4*>(p.arr + src);
    } else {
        uint32_t w[4] = {p.fill[0], p.fill[1], p.fill[2], p.fill[3]};
        constexpr int kItems = 16 / ITEM;
        const uint32_t e0 = (uint32_t)o / ITEM;
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            if ((uint32_t)o + (uint32_t)(j * ITEM) >= p.g.nbytes) break;
            int64_t src = arr_off;
            if (!sel_offset(p.g, s, e0 + j, p.g.ndim - 1, src)) continue;
            uint32_t lo = 0, hi = 0;
            load_item<ITEM>(p.arr + src, lo, hi);
            if constexpr (ITEM == 8) {
                w[2 * j] = lo;
                w[2 * j + 1] = hi;
            } else if constexpr (ITEM == 4) {
                w[j] = lo;
            } else {
                constexpr uint32_t m = (1u << (8 * ITEM)) - 1u;
                const int sh = 8 * ((j * ITEM) % 4);
                w[(j * ITEM) / 4] = (w[(j * ITEM) / 4] & ~(m << sh)) | ((lo & m) << sh);
            }
        }
        return make_uint4(w[0], w[1], w[2], w[3]);
    }
}

// Store the 16 encoded bytes at dst (chunk-relative block o), only [0, valid).
__device__ __forceinline__ void store_block(uint8_t* cp, int32_t o, uint4 v, uint32_t valid, bool al4) {
    if (valid >= 16u && al4) {
        *reinterpret_cast<uint4*>(cp + o) = v;
        return;
    }
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    const uint32_t n = valid < 16u ? valid : 16u;
    for (uint32_t i = 0; i < n; ++i) cp[o + i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3u)));
}

__device__ __forceinline__ void put_le_u32(uint8_t* d, uint32_t v) {  // any alignment
    d[0] = (uint8_t)v;
    d[1] = (uint8_t)(v >> 8);
    d[2] = (uint8_t)(v >> 16);
    d[3] = (uint8_t)(v >> 24);
}

template <bool CRC, bool FAST, int ITEM, bool SWAP>
__global__ __launch_bounds__(kThreads) void k_encode(const EncodeParams p) {
    constexpr int K = kDefaultBlocks;
    __shared__ uint32_t s_tab[CRC ? 16 * 256 : 1];
    __shared__ uint32_t s_red[2][kThreads / 64];
    const int t = threadIdx.x;
    uint32_t kth = 0;
    if constexpr (CRC) {
        const uint4* g = reinterpret_cast<const uint4*>(p.horner);
        uint4* sv = reinterpret_cast<uint4*>(s_tab);
        for (int i = t; i < 1024; i += kThreads) sv[i] = g[i];
        kth = p.kthread[t];
        __syncthreads();
    }
    const uint32_t G = gridDim.x, gi = blockIdx.x;
    const uint32_t per = p.n_units / G, rem = p.n_units % G;
    const uint32_t q0 = gi * per + (gi < rem ? gi : rem);
    const uint32_t q1 = q0 + per + (gi < rem ? 1u : 0u);
    uint32_t acc = 0, parity = 0;
    bool alleq = true;
    for (uint32_t q = q0; q < q1; ++q) {
        const uint32_t c = q / p.nseg;
        const uint32_t sidx = p.nseg - 1u - (q - c * p.nseg);
        const zhip_chunk ch = p.chunks[c];
        const zhip_sel& sel = p.sels[ch.sel];
        uint8_t* cp = p.dst + ch.src;
        const bool al4 = __builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<uintptr_t>(cp) & 3u)) == 0u;
        const int32_t seg_lo = (int32_t)p.E - (int32_t)((sidx + 1u) * p.seg);
        uint4 blk[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int32_t o = seg_lo + kWgStride * k + 16 * t;
            blk[k] = (o < 0 || (uint32_t)o >= p.g.nbytes) ? make_uint4(0, 0, 0, 0)
                                                          : gather_block<ITEM, FAST>(p, sel, ch.out_off, o);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int32_t o = seg_lo + kWgStride * k + 16 * t;
            if (o < 0 || (uint32_t)o >= p.g.nbytes) continue;
            const uint32_t valid = p.g.nbytes - (uint32_t)o;
            alleq = alleq && block_eq_fill<ITEM>(blk[k], valid, p);
            blk[k] = mask_tail(swap_block<ITEM, SWAP>(blk[k]), o, p.g.nbytes);
            store_block(cp, o, blk[k], valid, al4);
        }
        if constexpr (CRC) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint4 v = blk[k];
                acc = tab_apply(s_tab, acc ^ v.x) ^ tab_apply(s_tab + 1024, v.y) ^ tab_apply(s_tab + 2048, v.z) ^
                      tab_apply(s_tab + 3072, v.w);
            }
        }
        const bool run_end = (q + 1 >= q1) || ((q + 1) / p.nseg != c);
        if (run_end) {
            // chunk_is_empty: any element != fill anywhere in the chunk -> non-empty
            if (__any(!alleq) && (t & 63) == 0) atomicOr(p.nonempty + c, 1u);
            alleq = true;
            if constexpr (CRC) {
                uint32_t v = gf_mul(acc, kth);
                v = wave_xor(v);
                if ((t & 63) == 0) s_red[parity][t >> 6] = v;
                __syncthreads();
                if (t == 0) {
                    uint32_t V = s_red[parity][0] ^ s_red[parity][1] ^ s_red[parity][2] ^ s_red[parity][3];
                    V = gf_mul(V, p.kunit[sidx]);
                    uint32_t* accw = p.ws + 4ull * c;
                    const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
                    const uint32_t run_len = q + 1u - (q0 > c * p.nseg ? q0 : c * p.nseg);
                    const uint32_t tk =
                        __hip_atomic_fetch_add(accw + 2, run_len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (tk + run_len == p.nseg) {
                        const uint32_t raw = __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const uint32_t crc = ~(gf_mul(raw, p.c_inv) ^ p.c3);
                        uint8_t* tr = cp + p.g.nbytes;  // LE trailer (crc32c_.py:64-68)
                        tr[0] = (uint8_t)crc;
                        tr[1] = (uint8_t)(crc >> 8);
                        tr[2] = (uint8_t)(crc >> 16);
                        tr[3] = (uint8_t)(crc >> 24);
                        zhip_status st = {ZHIP_ST_OK, crc, crc, 0u};
                        p.status[c] = st;
                    }
                }
                parity ^= 1u;
                acc = 0;
            } else if (t == 0 && sidx == 0) {
                zhip_status st = {ZHIP_ST_OK, 0u, 0u, 0u};
                p.status[c] = st;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// k_encode_pair: whole-row layouts with a row map (zhip_encode_mapped).  The
// two-unit structure of k_decode_pair (decode_rows.hip) run in reverse: every
// gather load of both units first (source rows from the row map; lanes outside
// the selection read one dummy line and take the fill value), then per block
// the fill-equality test, byteswap, store and Horner step, then one run end
// per chunk run whose last arrival writes the CRC trailer.
// ---------------------------------------------------------------------------
__device__ uint4 g_enc_zero[1];
__device__ uint4 g_enc_sink[kThreads];

typedef unsigned int zhip_v4u_ae __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) const zhip_v4u_ae zhip_gv4u_ae;
typedef __attribute__((address_space(1))) zhip_v4u_ae zhip_gv4u_aew;

__device__ __forceinline__ uint4 enc_load16(const uint8_t* a) {  // any alignment, one dwordx4 (kNtLoads)
    zhip_v4u_ae w;
    if constexpr (kNtLoads) w = __builtin_nontemporal_load((zhip_gv4u_ae*)(reinterpret_cast<uintptr_t>(a)));
    else w = *(zhip_gv4u_ae*)(reinterpret_cast<uintptr_t>(a));
    return make_uint4(w.x, w.y, w.z, w.w);
}

__device__ __forceinline__ void enc_store16(uint8_t* a, uint4 v) {  // any alignment, one dwordx4 nt
    zhip_v4u_ae w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, (zhip_gv4u_aew*)(reinterpret_cast<uintptr_t>(a)));
}

struct EncRowSteps {
    zhip_rowblk e[kDefaultBlocks];
};

// ACC: uint32_t (one chain, the 16 byte-position tables: p.horner) or Acc4
// (one accumulator per word through A4096, the 11/11/10 pair tables: 12
// lookups per block instead of 16, folded at the run end -- k_decode_pair's
// CRC, zhip_decode_common.h)
template <bool CRC, int ITEM, bool SWAP, typename ACC>
__device__ __forceinline__ void enc_unit(const EncodeParams& p, const zhip_chunk& ch, uint32_t sidx, bool live,
                                        const EncRowSteps& m, uint32_t lane_row, const uint4 (&blk)[kDefaultBlocks],
                                        const uint32_t* s_tab, ACC& acc, bool& alleq, int t) {
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
    const int32_t seg_lo = (int32_t)p.E - (int32_t)((sidx + 1u) * p.seg);
    uint8_t* const cp = p.dst + ch.src;
    uint8_t* const sink = reinterpret_cast<uint8_t*>(g_enc_sink) + 16 * t;
#pragma unroll
    for (int k = 0; k < kDefaultBlocks; ++k) {
        const int32_t o = seg_lo + kWgStride * k;
        const bool in_sel = lane_row - m.e[k].lo < (uint32_t)(m.e[k].hi - m.e[k].lo);
        const uint4 v = in_sel ? blk[k] : f;  // _merge_chunk_array: outside the selection = fill
        alleq = alleq && block_eq_fill<ITEM>(v, 16u, p);
        const uint4 e = swap_block<ITEM, SWAP>(v);
        enc_store16(live && o >= 0 ? cp + o + 16 * t : sink, e);  // every path stores: static count
        if constexpr (CRC) {
            if (live && o >= 0) {
                if constexpr (sizeof(ACC) == sizeof(Acc4)) crc_block4(s_tab, acc, e);
                else
                    acc = tab_apply(s_tab, acc ^ e.x) ^ tab_apply(s_tab + 1024, e.y) ^
                          tab_apply(s_tab + 2048, e.z) ^ tab_apply(s_tab + 3072, e.w);
            }
        }
    }
}

template <typename ACC>
__device__ __forceinline__ uint32_t enc_state(const uint32_t* s_tab, const ACC& acc) {
    if constexpr (sizeof(ACC) == sizeof(Acc4)) return fold4(s_tab, acc);
    else return acc;
}

template <bool CRC>
__device__ __forceinline__ void enc_run_end(const EncodeParams& p, const zhip_chunk& ch, uint32_t c, uint32_t acc,
                                           uint32_t klane, uint32_t bits, uint32_t n_run, uint32_t* red, int t) {
    if constexpr (!CRC) {
        if (t == 0 && (bits & 1u)) {  // the unit ending at E is in this run: one status per chunk
            zhip_status st = {ZHIP_ST_OK, 0u, 0u, 0u};
            p.status[c] = st;
        }
        return;
    } else {
        const uint32_t v = wave_xor(gf_mul(acc, klane));
        __syncthreads();  // red may still be read by the previous run end
        if ((t & 63) == 0) red[t >> 6] = v;
        __syncthreads();
        if (t != 0) return;
        const uint32_t V = red[0] ^ red[1] ^ red[2] ^ red[3];
        uint32_t raw = 0, last = 0;
        if (p.nseg <= 32) {
            const uint64_t full = p.nseg >= 32 ? 0xFFFFFFFFull : ((1ull << p.nseg) - 1ull);
            uint64_t* w = reinterpret_cast<uint64_t*>(p.ws) + (uint64_t)p.pub_stride * c;
            const uint64_t prev =
                __hip_atomic_fetch_xor(w, ((uint64_t)bits << 32) | V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (((prev >> 32) ^ bits) == full) {
                __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                raw = (uint32_t)prev ^ V;
                last = 1;
            }
        } else {
            uint32_t* accw = p.ws + 4ull * c;
            const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
            const uint32_t tk = __hip_atomic_fetch_add(accw + 2, n_run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tk + n_run == p.nseg) {
                raw = __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = 1;
            }
        }
        if (last) {
            const uint32_t crc = ~(raw ^ p.c3);  // kpair carries c_inv
            put_le_u32(p.dst + ch.src + p.g.nbytes, crc);  // LE trailer (crc32c_.py:64-68)
            zhip_status st = {ZHIP_ST_OK, crc, crc, 0u};
            p.status[c] = st;
        }
    }
}

// Run end of a workgroup whose two units are pair `pr` of chunk c (regular
// pairing, see k_encode_pair): word = CRC contribution | arrival bit of the
// pair (bits 32..47) | non-empty bit of the pair (bits 48..63).  Each pair
// sets its bits once per launch, so XOR accumulates them like OR.
template <bool CRC>
__device__ __forceinline__ void enc_run_end_pair(const EncodeParams& p, const zhip_chunk& ch, uint32_t c, uint32_t acc,
                                                uint32_t klane, uint32_t pr, bool wave_ne, uint32_t* red, int t) {
    uint32_t v = 0;
    if constexpr (CRC) v = wave_xor(gf_mul(acc, klane));
    if ((t & 63) == 0) red[t >> 6] = v | 0u;
    __shared__ uint32_t s_ne[kThreads / 64];
    if ((t & 63) == 0) s_ne[t >> 6] = wave_ne ? 1u : 0u;
    __syncthreads();
    if (t != 0) return;
    const uint32_t V = CRC ? (red[0] ^ red[1] ^ red[2] ^ red[3]) : 0u;
    const bool ne = (s_ne[0] | s_ne[1] | s_ne[2] | s_ne[3]) != 0u;
    const uint64_t pb = 1ull << pr;
    const uint64_t full = (1ull << (p.nseg >> 1)) - 1ull;
    uint64_t* w = reinterpret_cast<uint64_t*>(p.ws) + (uint64_t)p.pub_stride * c;
    const uint64_t word = (pb << 32) | (ne ? pb << 48 : 0ull) | V;
    const uint64_t prev = __hip_atomic_fetch_xor(w, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((((prev >> 32) & 0xFFFFull) ^ pb) != full) return;
    __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    p.nonempty[c] = (((prev >> 48) ^ (ne ? pb : 0ull)) != 0ull) ? 1u : 0u;
    uint32_t crc = 0;
    if constexpr (CRC) {
        crc = ~(((uint32_t)prev ^ V) ^ p.c3);  // kpair carries c_inv
        put_le_u32(p.dst + ch.src + p.g.nbytes, crc);  // LE trailer (crc32c_.py:64-68)
    }
    zhip_status st = {ZHIP_ST_OK, crc, crc, 0u};
    p.status[c] = st;
}

// T11: the CRC through the 11/11/10 pair tables (arm ZHIP_TUNE_ARM = 1)
// instead of the byte-position tables: 12 lookups per block instead of 16,
// graph-timed on C2 30.7-30.9 vs 30.5-30.6 us (profiles/r04/g/enc_arms.jsonl):
// the encode is not bound by its lookups
template <bool CRC, int ITEM, bool SWAP, bool T11 = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_encode_pair(const EncodeParams p) {
    constexpr int K = kDefaultBlocks;
    using ACC = typename std::conditional<T11, Acc4, uint32_t>::type;
    __shared__ uint32_t s_tab[CRC ? (T11 ? kPairTabWords : 16 * 256) : 1];
    __shared__ uint32_t s_red[2][kThreads / 64];
    const int t = threadIdx.x;
    // XCD-contiguous runs for a one-wave grid (launch_encode's xcd_run, as k_decode_pair)
    const uint32_t b = p.xcd_run ? ((blockIdx.x >> 3) / p.xcd_run * 8u + (blockIdx.x & 7u)) * p.xcd_run +
                                       (blockIdx.x >> 3) % p.xcd_run
                                 : blockIdx.x;
    const uint32_t q0 = 2u * b;
    const bool has_b = q0 + 1u < p.n_units;
    auto unit_of = [&](uint32_t q) {
        const uint32_t c = q / p.nseg;
        return c * p.nseg + (p.nseg - 1u - (q - c * p.nseg));
    };
    const uint32_t u_a = unit_of(q0), u_b = has_b ? unit_of(q0 + 1u) : u_a;
    const uint32_t ca = u_a / p.nseg, sa = u_a - ca * p.nseg, cb = u_b / p.nseg, sb = u_b - cb * p.nseg;
    uint4 tv0, tv1, tv2, tv3, tv4, tv5;
    uint32_t ka = 0, kb = 0;
    if constexpr (CRC) {
        const uint4* gt = reinterpret_cast<const uint4*>(T11 ? p.pair_tab : p.horner);
        tv0 = gt[t];
        tv1 = gt[t + kThreads];
        tv2 = gt[t + 2 * kThreads];
        tv3 = gt[t + 3 * kThreads];
        if constexpr (T11) {
            tv4 = gt[t + 4 * kThreads];
            tv5 = gt[t + 5 * kThreads];
        }
        const uint32_t* kp = T11 ? p.kpair11 : p.kpair;
        ka = kp[(size_t)sa * kThreads + t];
        kb = kp[(size_t)sb * kThreads + t];
    }
    const zhip_chunk cha = load_uniform<zhip_chunk>(p.chunks + ca);
    const zhip_chunk chb = load_uniform<zhip_chunk>(p.chunks + cb);
    const EncRowSteps ma = load_uniform<EncRowSteps>(p.rowmap + ((size_t)cha.sel * p.nseg + sa) * K);
    const EncRowSteps mb = load_uniform<EncRowSteps>(p.rowmap + ((size_t)chb.sel * p.nseg + sb) * K);
    const uint32_t lane_row = (16u * (uint32_t)t) >> p.row_shift;
    const uint32_t lane_col = (16u * (uint32_t)t) & ((1u << p.row_shift) - 1u);
    const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_enc_zero);
    // 1. gather loads of both units (static count: outside the selection -> dummy line)
    uint4 A[K], B[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const bool in = lane_row - ma.e[k].lo < (uint32_t)(ma.e[k].hi - ma.e[k].lo);
        A[k] = enc_load16(in ? p.arr + cha.out_off + ma.e[k].rel + lane_off : zero);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const bool in = has_b && lane_row - mb.e[k].lo < (uint32_t)(mb.e[k].hi - mb.e[k].lo);
        B[k] = enc_load16(in ? p.arr + chb.out_off + mb.e[k].rel + lane_off : zero);
    }
    if constexpr (CRC) {
        uint4* st = reinterpret_cast<uint4*>(s_tab);
        st[t] = tv0;
        st[t + kThreads] = tv1;
        st[t + 2 * kThreads] = tv2;
        st[t + 3 * kThreads] = tv3;
        if constexpr (T11) {
            st[t + 4 * kThreads] = tv4;
            st[t + 5 * kThreads] = tv5;
        }
        __syncthreads();
    }
    // 2. per block: fill test, byteswap, store, Horner step
    const bool same = has_b && cb == ca;
    ACC acc_a{}, acc_b{};
    bool eq_a = true, eq_b = true;
    enc_unit<CRC, ITEM, SWAP>(p, cha, sa, true, ma, lane_row, A, s_tab, acc_a, eq_a, t);
    if (same) {
        acc_b = acc_a;
        eq_b = eq_a;
    }
    enc_unit<CRC, ITEM, SWAP>(p, chb, sb, has_b, mb, lane_row, B, s_tab, acc_b, eq_b, t);
    // 3./4. regular pairing (an even number of units per chunk, at most 32): the
    //    two units always share a chunk and the workgroup publishes CRC, its
    //    pair's arrival bit and its pair's non-empty bit in ONE 64-bit atomic;
    //    the last arrival writes trailer, status and the chunk's non-empty flag
    //    (so the flags need no zeroing and no same-address atomic storm)
    if (p.nseg % 2u == 0u && p.nseg <= 32u) {
        enc_run_end_pair<CRC>(p, chb, cb, CRC ? enc_state(s_tab, acc_b) : 0u, kb, (p.nseg - 1u - sb) >> 1,
                              __any(!eq_b), s_red[1], t);
        return;
    }
    // 3. chunk_is_empty (chunk_utils.py:74-85): any element != fill -> non-empty
    if (!(p.tune & kTuneEncNoFlags)) {  // (ablation: no flag atomics; results invalid)
        if (!same && __any(!eq_a) && (t & 63) == 0) atomicOr(p.nonempty + ca, 1u);
        if (has_b && __any(!eq_b) && (t & 63) == 0) atomicOr(p.nonempty + cb, 1u);
    }
    // 4. run ends: A alone when B starts another chunk, then B (or A+B)
    if (!same) enc_run_end<CRC>(p, cha, ca, CRC ? enc_state(s_tab, acc_a) : 0u, ka, 1u << (sa & 31u), 1u, s_red[0], t);
    if (has_b)
        enc_run_end<CRC>(p, chb, cb, CRC ? enc_state(s_tab, acc_b) : 0u, kb,
                         (same ? 1u << (sa & 31u) : 0u) | (1u << (sb & 31u)), same ? 2u : 1u, s_red[1], t);
}

// k_encode_il: k_decode_il in reverse (chunks whose 4 KiB steps tile into
// groups of eight workgroups: the headline's 1 MiB chunks).  Workgroup r of
// chunk c gathers the K = 8 steps st0 + 8 k (st0 = (r / 8) 64 + r % 8) of its
// chunk -- rows from the row map, as k_encode_pair -- tests them against the
// fill, stores them and carries their CRC through the A_(4096 * 8) 11/11/10
// tables with k_decode_il's lane constants (the same plan tables: the CRC is
// over the same stored bytes at the same positions).  One unit per workgroup
// (2 048 on the headline instead of 1 024 pairs).  Publication without extra
// same-address atomics (a non-empty OR per wave doubled the launch): the
// chunk's workgroups split into halves of at most 16, each half publishing
// CRC | arrival bits 32..47 | non-empty bits 48..63 in one 64-bit word (the
// pair kernel's format); the last arrival of a half folds the half's word into
// the line's third word the same way (bits 32 / 48 + half), and the last of
// those writes trailer, status and the non-empty flag.  Chunks of at most 16
// units have one half and no second level.
// AFF (tuning arm 46): ZHIP_DF_WHOLE launches of plans with aff_ok take the
// destinations from aff_rowblk instead of the row map (k_decode_il's AFF);
// graph-timed 0.5 us slower on the C2 encode, not adopted.
template <int ITEM, bool SWAP, bool AFF = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_encode_il(const EncodeParams p) {
    constexpr int K = kDefaultBlocks;
    __shared__ uint32_t s_tab[kPairTabWords];
    __shared__ uint32_t s_mul[12 * kThreads];
    __shared__ uint32_t s_red[kThreads / 64];
    __shared__ uint32_t s_ne[kThreads / 64];
    const int t = threadIdx.x;
    const uint32_t g = blockIdx.x;
    const uint32_t wpc = p.nseg, S = p.il_S;
    const uint32_t c = g / wpc, r = g - c * wpc;
    // 1. tables and the lane constant (the oldest loads), the chunk record and
    //    the row map (scalar), then the gather loads
    const uint4* gt = reinterpret_cast<const uint4*>(p.il_tab);
    const uint4 tv0 = gt[t], tv1 = gt[t + kThreads], tv2 = gt[t + 2 * kThreads], tv3 = gt[t + 3 * kThreads],
                tv4 = gt[t + 4 * kThreads], tv5 = gt[t + 5 * kThreads];
    const uint32_t kl = p.il_klane[(size_t)r * kThreads + t];
    const zhip_chunk ch = load_uniform<zhip_chunk>(p.chunks + c);
    const uint32_t st0 = (r / S) * S * (uint32_t)K + (r % S);
    const int32_t lo_frame = (int32_t)p.E - (int32_t)(p.nseg * p.seg);
    zhip_rowblk m[K];
    if (AFF && sel_whole(p, ch.sel)) {  // (checked, not trusted: sel_whole)
#pragma unroll
        for (int k = 0; k < K; ++k) m[k] = aff_rowblk(p, st0 + S * (uint32_t)k);
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t st = st0 + S * (uint32_t)k;
            const uint32_t sidx = p.nseg - 1u - st / (uint32_t)K;
            m[k] = load_uniform<zhip_rowblk>(p.rowmap + ((size_t)ch.sel * p.nseg + sidx) * K + (st % (uint32_t)K));
        }
    }
    const uint32_t lane_row = (16u * (uint32_t)t) >> p.row_shift;
    const uint32_t lane_col = (16u * (uint32_t)t) & ((1u << p.row_shift) - 1u);
    const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_enc_zero);
    uint4 A[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const bool in = lane_row - m[k].lo < (uint32_t)(m[k].hi - m[k].lo);
        A[k] = enc_load16(in ? p.arr + ch.out_off + m[k].rel + lane_off : zero);
    }
    // 2. tables into LDS, the lane-multiply column
    {
        uint4* stt = reinterpret_cast<uint4*>(s_tab);
        stt[t] = tv0;
        stt[t + kThreads] = tv1;
        stt[t + 2 * kThreads] = tv2;
        stt[t + 3 * kThreads] = tv3;
        stt[t + 4 * kThreads] = tv4;
        stt[t + 5 * kThreads] = tv5;
        lanemul3_init(s_mul, t, kl);
    }
    __syncthreads();
    // 3. per block: fill test (chunk_is_empty, chunk_utils.py:74-85; outside
    //    the selection = fill, _merge_chunk_array), byteswap, store, Horner step
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
    uint8_t* const cp = p.dst + ch.src;
    uint8_t* const sink = reinterpret_cast<uint8_t*>(g_enc_sink) + 16 * t;
    Acc4 acc = {0u, 0u, 0u, 0u};
    bool eq = true;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int32_t o = lo_frame + kWgStride * (int32_t)(st0 + S * (uint32_t)k);
        const bool in = lane_row - m[k].lo < (uint32_t)(m[k].hi - m[k].lo);
        const uint4 v = in ? A[k] : f;
        eq = eq && block_eq_fill<ITEM>(v, 16u, p);
        const uint4 e = swap_block<ITEM, SWAP>(v);
        enc_store16(o >= 0 ? cp + o + 16 * t : sink, e);
        if (o >= 0) crc_block4(s_tab, acc, e);
    }
    // 4. run end: one chain per workgroup, one publication
    const uint32_t v = wave_xor(lanemul3(s_mul, t, fold4(s_tab, acc)));
    const bool wave_ne = __any(!eq);
    if ((t & 63) == 0) {
        s_red[t >> 6] = v;
        s_ne[t >> 6] = wave_ne ? 1u : 0u;
    }
    __syncthreads();
    if (t != 0) return;
    const uint32_t V = s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3];
    const bool ne = (s_ne[0] | s_ne[1] | s_ne[2] | s_ne[3]) != 0u;
    uint64_t* const w = reinterpret_cast<uint64_t*>(p.ws) + (uint64_t)p.pub_stride * c;
    const uint32_t h = r >> 4, b = r & 15u;
    const uint32_t n_h = h ? wpc - 16u : (wpc < 16u ? wpc : 16u);  // workgroups of this half
    const uint64_t bit = 1ull << b;
    const uint64_t word = (bit << 32) | (ne ? bit << 48 : 0ull) | V;
    const uint64_t prev = __hip_atomic_fetch_xor(w + h, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((((prev ^ word) >> 32) & 0xFFFFull) != (1ull << n_h) - 1ull) return;
    __hip_atomic_store(w + h, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t all = prev ^ word;  // the half: CRC | arrivals | non-empty bits
    if (wpc > 16u) {  // second level: the halves into the line's third word
        const uint64_t hb = 1ull << h;
        const uint64_t w2 = (hb << 32) | ((all >> 48) ? hb << 48 : 0ull) | (uint32_t)all;
        const uint64_t p2 = __hip_atomic_fetch_xor(w + 2, w2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((((p2 ^ w2) >> 32) & 0xFFFFull) != 3ull) return;
        __hip_atomic_store(w + 2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        all = p2 ^ w2;
    }
    // the chunk's last arrival: trailer, status, non-empty flag
    p.nonempty[c] = (all >> 48) != 0ull ? 1u : 0u;
    const uint32_t crc = ~((uint32_t)all ^ p.c3);   // the lane constants carry c_inv
    put_le_u32(p.dst + ch.src + p.g.nbytes, crc);  // LE trailer (crc32c_.py:64-68)
    zhip_status st = {ZHIP_ST_OK, crc, crc, 0u};
    p.status[c] = st;
}

using EncodeFn = void (*)(const EncodeParams);

static EncodeFn pick_encode_il(int item, bool swap, bool aff) {
#if ZHIP_TUNING
#define ZHIP_EIL(I, W) (aff ? k_encode_il<I, W, true> : k_encode_il<I, W>)  // (arm 46)
#else
#define ZHIP_EIL(I, W) k_encode_il<I, W>
#endif
    switch (item) {
        case 1: return ZHIP_EIL(1, false);
        case 2: return swap ? ZHIP_EIL(2, true) : ZHIP_EIL(2, false);
        case 4: return swap ? ZHIP_EIL(4, true) : ZHIP_EIL(4, false);
        case 8: return swap ? ZHIP_EIL(8, true) : ZHIP_EIL(8, false);
        default: return nullptr;
    }
#undef ZHIP_EIL
}

// k_encode_quad: k_encode_pair for chunks of at most 16 KiB (one unit per
// chunk; the reference example's 64 x 64 int32 inner chunks).  Such a unit's
// first four steps lie before the chunk start, so the pair kernel gathers and
// stores half its blocks for nothing; here a workgroup encodes four chunks with
// only the last four steps of each.  The workgroup owns its chunks whole: CRC
// and non-empty bit reduce in LDS and lanes 0..3 write trailer, status and flag
// of one chunk each (no publication word, no zeroed flags).
template <bool CRC, int ITEM, bool SWAP>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_encode_quad(const EncodeParams p) {
    constexpr int NQ = 4, KS = kDefaultBlocks / 2, K0 = kDefaultBlocks - KS;
    __shared__ uint32_t s_tab[CRC ? 16 * 256 : 1];
    __shared__ uint32_t s_red[NQ][kThreads / 64];
    __shared__ uint32_t s_ne[NQ][kThreads / 64];
    const int t = threadIdx.x;
    const uint32_t c0 = (uint32_t)NQ * blockIdx.x;  // nseg == 1: unit = chunk
    uint4 tv0, tv1, tv2, tv3;
    uint32_t kl = 0;
    if constexpr (CRC) {
        const uint4* gt = reinterpret_cast<const uint4*>(p.horner);
        tv0 = gt[t];
        tv1 = gt[t + kThreads];
        tv2 = gt[t + 2 * kThreads];
        tv3 = gt[t + 3 * kThreads];
        kl = p.kpair[t];  // unit 0's lane constants
    }
    bool live[NQ];
    zhip_chunk ch[NQ];
    EncRowSteps m[NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        live[i] = c0 + (uint32_t)i < p.n_units;
        ch[i] = load_uniform<zhip_chunk>(p.chunks + (live[i] ? c0 + i : c0));
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i) m[i] = load_uniform<EncRowSteps>(p.rowmap + (size_t)ch[i].sel * kDefaultBlocks);
    const uint32_t lane_row = (16u * (uint32_t)t) >> p.row_shift;
    const uint32_t lane_col = (16u * (uint32_t)t) & ((1u << p.row_shift) - 1u);
    const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_enc_zero);
    uint4 blk[NQ][KS];
#pragma unroll
    for (int i = 0; i < NQ; ++i)
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            const zhip_rowblk& e = m[i].e[K0 + k];
            const bool in = live[i] && lane_row - e.lo < (uint32_t)(e.hi - e.lo);
            blk[i][k] = enc_load16(in ? p.arr + ch[i].out_off + e.rel + lane_off : zero);
        }
    if constexpr (CRC) {
        uint4* st = reinterpret_cast<uint4*>(s_tab);
        st[t] = tv0;
        st[t + kThreads] = tv1;
        st[t + 2 * kThreads] = tv2;
        st[t + 3 * kThreads] = tv3;
        __syncthreads();
    }
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
    const int32_t seg_lo = (int32_t)p.E - (int32_t)p.seg;
    uint8_t* const sink = reinterpret_cast<uint8_t*>(g_enc_sink) + 16 * t;
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        uint8_t* const cp = p.dst + ch[i].src;
        uint32_t acc = 0;
        bool eq = true;
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            const zhip_rowblk& e = m[i].e[K0 + k];
            const int32_t o = seg_lo + kWgStride * (K0 + k);
            const bool in_sel = lane_row - e.lo < (uint32_t)(e.hi - e.lo);
            const uint4 v = in_sel ? blk[i][k] : f;  // _merge_chunk_array: outside the selection = fill
            eq = eq && block_eq_fill<ITEM>(v, 16u, p);
            const uint4 w = swap_block<ITEM, SWAP>(v);
            enc_store16(live[i] && o >= 0 ? cp + o + 16 * t : sink, w);
            if constexpr (CRC)
                if (o >= 0)
                    acc = tab_apply(s_tab, acc ^ w.x) ^ tab_apply(s_tab + 1024, w.y) ^ tab_apply(s_tab + 2048, w.z) ^
                          tab_apply(s_tab + 3072, w.w);
        }
        uint32_t v = 0;
        // (the lane multiply in registers: four per workgroup here, 31.8-33.0 vs
        // 33.5-33.9 us with gf_mul's bit loop, profiles/r04/lmr/)
        if constexpr (CRC) v = wave_xor(lanemul_reg(kl, acc));
        const bool ne = __any(!eq);
        if ((t & 63) == 0) {
            s_red[i][t >> 6] = v;
            s_ne[i][t >> 6] = ne ? 1u : 0u;
        }
    }
    __syncthreads();
    if (t < NQ && c0 + (uint32_t)t < p.n_units) {  // lane i: chunk c0 + i
        const uint32_t c = c0 + (uint32_t)t;
        p.nonempty[c] = (s_ne[t][0] | s_ne[t][1] | s_ne[t][2] | s_ne[t][3]) != 0u ? 1u : 0u;
        uint32_t crc = 0;
        if constexpr (CRC) {
            crc = ~((s_red[t][0] ^ s_red[t][1] ^ s_red[t][2] ^ s_red[t][3]) ^ p.c3);  // kpair carries c_inv
            put_le_u32(p.dst + p.chunks[c].src + p.g.nbytes, crc);  // LE trailer (crc32c_.py:64-68)
        }
        zhip_status st = {ZHIP_ST_OK, crc, crc, 0u};
        p.status[c] = st;
    }
}


template <bool CRC, int ITEM>
static EncodeFn pick_encode_quad_item(bool swap) {
    if constexpr (ITEM == 1) return k_encode_quad<CRC, 1, false>;
    else return swap ? k_encode_quad<CRC, ITEM, true> : k_encode_quad<CRC, ITEM, false>;
}

static EncodeFn pick_encode_quad(bool crc, int item, bool swap) {
    switch (item) {
        case 1: return crc ? pick_encode_quad_item<true, 1>(swap) : pick_encode_quad_item<false, 1>(swap);
        case 2: return crc ? pick_encode_quad_item<true, 2>(swap) : pick_encode_quad_item<false, 2>(swap);
        case 4: return crc ? pick_encode_quad_item<true, 4>(swap) : pick_encode_quad_item<false, 4>(swap);
        case 8: return crc ? pick_encode_quad_item<true, 8>(swap) : pick_encode_quad_item<false, 8>(swap);
        default: return nullptr;
    }
}

template <bool CRC, bool FAST>
static EncodeFn pick_encode(int item, bool swap) {
    switch (item) {
        case 1: return k_encode<CRC, FAST, 1, false>;
        case 2: return swap ? k_encode<CRC, FAST, 2, true> : k_encode<CRC, FAST, 2, false>;
        case 4: return swap ? k_encode<CRC, FAST, 4, true> : k_encode<CRC, FAST, 4, false>;
        case 8: return swap ? k_encode<CRC, FAST, 8, true> : k_encode<CRC, FAST, 8, false>;
        default: return nullptr;
    }
}

static EncodeFn pick_encode_pair(bool crc, int item, bool swap) {
#if ZHIP_TUNING
    if (g_tune_arm == 1 && crc && item == 4 && !swap) return k_encode_pair<true, 4, false, true>;  // 11/11/10 tables
#endif
    switch (item) {
        case 1: return crc ? k_encode_pair<true, 1, false> : k_encode_pair<false, 1, false>;
        case 2: return crc ? (swap ? k_encode_pair<true, 2, true> : k_encode_pair<true, 2, false>)
                           : (swap ? k_encode_pair<false, 2, true> : k_encode_pair<false, 2, false>);
        case 4: return crc ? (swap ? k_encode_pair<true, 4, true> : k_encode_pair<true, 4, false>)
                           : (swap ? k_encode_pair<false, 4, true> : k_encode_pair<false, 4, false>);
        case 8: return crc ? (swap ? k_encode_pair<true, 8, true> : k_encode_pair<true, 8, false>)
                           : (swap ? k_encode_pair<false, 8, true> : k_encode_pair<false, 8, false>);
        default: return nullptr;
    }
}

EncodeFn select_encode_tile4_kernel(bool crc, int item, bool swap, int nt);  // decode_tile.hip
EncodeFn select_encode_tile_kernel(bool crc, int item, bool swap);   // decode_tile.hip
EncodeFn select_encode_tileg_kernel(bool crc, int item, bool swap, int nt);  // decode_tile.hip

int launch_encode(const EncodeParams& p, hipStream_t stream, int max_grid) {
    const bool crc = (p.lflags & ZHIP_LF_CRC) != 0;
    const bool swap = (p.lflags & ZHIP_LF_SWAP) != 0;
    if (p.tile4) {  // transposed layouts with full tiles (k_encode_tile4)
        // two tiles per workgroup where the plan built their constants (tuning
        // arm 38 keeps four)
        const int nt = (crc && p.kq2 && g_tune_arm != 38) ? 2 : 4;
        EncodeFn fn = select_encode_tile4_kernel(crc, p.g.itemsize, swap, nt);
        if (!fn) return ZHIP_E_UNSUPPORTED;
        if (p.n_chunks == 0) return ZHIP_OK;
        EncodeParams q = p;
        if (nt == 2) q.kq4 = p.kq2;
        g_last_kernel = nt == 2 ? "k_encode_tile2" : "k_encode_tile4";
        hipLaunchKernelGGL(fn, dim3(p.n_chunks * (p.t_per_chunk / (uint32_t)nt)), dim3(kThreads), 0, stream, q);
        return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
    }
    if (p.tile == 2) {  // full selections, tiles grouped by four at a uniform step (k_encode_tileg)
        // (tuning arm 36: two workgroups per group, two tiles each -- C3 in 128^3
        // chunks 33.1-34.1 vs 32.8-33.6 us graph-timed, no gain, profiles/r05/p/)
        const int nt = (crc && (g_tune_arm == 36 || g_tune_arm == 50)) ? 2 : 4;
        // (tuning arms 47 / 50: four / two tiles, arrival words on lines of their own)
        const bool spr = ZHIP_TUNING && crc && (g_tune_arm == 47 || g_tune_arm == 50);
        // (tuning arm 63: four tiles, the look-back finalizer, while fewer chunks than CUs)
        const bool lb = ZHIP_TUNING && crc && g_tune_arm == 63 && p.n_chunks < (uint32_t)(max_grid / 8) &&
                        (p.n_groups <= 16u || p.n_sub);
        // (tuning arm 68: four accumulators through one byte-table operator)
        const bool a4c = ZHIP_TUNING && crc && g_tune_arm == 68 && p.g_a4 != nullptr;
        EncodeFn fn = select_encode_tileg_kernel(crc, p.g.itemsize, swap,
                                                 a4c ? 9 : lb ? 8 : spr ? (nt == 4 ? 6 : 7) : nt);
        if (!fn) return ZHIP_E_UNSUPPORTED;
        if (p.n_chunks == 0) return ZHIP_OK;
        const uint64_t grid = (uint64_t)p.n_chunks * p.n_groups * (uint32_t)(4 / nt);
        if (grid >= (1ull << 31) || p.n_groups >= 65536u) return ZHIP_E_UNSUPPORTED;
        // (the last arrival of each chunk writes its non-empty flag)
        g_last_kernel = nt == 2 ? (spr ? "k_encode_tileg2s" : "k_encode_tileg2") : spr ? "k_encode_tilegs" : "k_encode_tileg";
        if (lb) g_last_kernel = "k_encode_tileg_lb";
        if (a4c) g_last_kernel = "k_encode_tileg_a4";
        hipLaunchKernelGGL(fn, dim3((uint32_t)grid), dim3(kThreads), 0, stream, p);
        return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
    }
    if (p.tile) {  // other transposed layouts / prefix selections (k_encode_tile)
        EncodeFn fn = select_encode_tile_kernel(crc, p.g.itemsize, swap);
        if (!fn) return ZHIP_E_UNSUPPORTED;
        if (p.n_chunks == 0) return ZHIP_OK;
        const uint64_t gpc = (p.t_per_chunk + 3u) / 4u;  // four tiles per workgroup
        if ((uint64_t)p.n_chunks * gpc >= (1ull << 31) || gpc >= 65536u) return ZHIP_E_UNSUPPORTED;
        // (the last arrival of each chunk writes its non-empty flag)
        hipLaunchKernelGGL(fn, dim3((uint32_t)(p.n_chunks * gpc)), dim3(kThreads), 0, stream, p);
        return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
    }
    if (p.rowmap && p.seg == (uint32_t)kWgStride * kDefaultBlocks && !(p.tune & kTunePersist) && p.nseg == 1u &&
        p.E <= 4u * kWgStride && g_tune_arm != 11) {  // chunks of <= 16 KiB: four per workgroup (arm 11: pairs)
        EncodeFn fn = pick_encode_quad(crc, p.g.itemsize, swap);
        if (!fn) return ZHIP_E_UNSUPPORTED;
        if (p.n_units == 0) return ZHIP_OK;
        hipLaunchKernelGGL(fn, dim3((p.n_units + 3u) / 4u), dim3(kThreads), 0, stream, p);
        return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
    }
    if (p.rowmap && p.seg == (uint32_t)kWgStride * kDefaultBlocks && !(p.tune & kTunePersist) && crc &&
        p.il_S >= 8u && p.nseg <= 32u && g_tune_arm != 34) {
        // one unit per workgroup, steps interleaved in groups of eight (k_encode_il;
        // tuning arm 34 keeps k_encode_pair)
        EncodeFn fn = pick_encode_il(p.g.itemsize, swap, p.aff_ok != 0);
        if (!fn) return ZHIP_E_UNSUPPORTED;
        if (p.n_units == 0) return ZHIP_OK;
        g_last_kernel = "k_encode_il";
        hipLaunchKernelGGL(fn, dim3(p.n_units), dim3(kThreads), 0, stream, p);
        return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
    }
    if (p.rowmap && p.seg == (uint32_t)kWgStride * kDefaultBlocks && !(p.tune & kTunePersist)) {
        g_last_kernel = "k_encode_pair";
        EncodeFn fn = pick_encode_pair(crc, p.g.itemsize, swap);
        if (!fn) return ZHIP_E_UNSUPPORTED;
        if (p.n_units == 0) return ZHIP_OK;
        // an even unit count <= 32 per chunk: the last arrival of each chunk writes
        // its non-empty flag; otherwise the kernel ORs into the flags -> zero them
        if ((p.nseg & 1u) || p.nseg > 32u) {
            if (hipMemsetAsync(p.nonempty, 0, (size_t)p.n_chunks * sizeof(uint32_t), stream) != hipSuccess)
                return ZHIP_E_HIP;
        }
        const uint32_t grid = (p.n_units + 1u) / 2u;
        EncodeParams q = p;
        q.xcd_run = (!(p.tune & kTuneNoXcd) && grid % 8u == 0u && grid <= (uint32_t)(max_grid / 8) * 4u) ? grid / 8u
                                                                                                      : 0u;
        hipLaunchKernelGGL(fn, dim3(grid), dim3(kThreads), 0, stream, q);
        return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
    }
    EncodeFn fn = crc ? (p.fast ? pick_encode<true, true>(p.g.itemsize, swap) : pick_encode<true, false>(p.g.itemsize, swap))
                      : (p.fast ? pick_encode<false, true>(p.g.itemsize, swap) : pick_encode<false, false>(p.g.itemsize, swap));
    if (!fn) return ZHIP_E_UNSUPPORTED;
    if (p.n_units == 0) return ZHIP_OK;
    // the persistent encode ORs each unit's non-empty bit into its chunk's flag
    if (hipMemsetAsync(p.nonempty, 0, (size_t)p.n_chunks * sizeof(uint32_t), stream) != hipSuccess)
        return ZHIP_E_HIP;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(fn), kThreads, 0) ==
            hipSuccess && per_cu > 0)
        max_grid = (max_grid / 8) * per_cu;
    if (g_tune_max_grid > 0) max_grid = g_tune_max_grid;
    const uint32_t grid = p.n_units < (uint32_t)max_grid ? p.n_units : (uint32_t)max_grid;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kThreads), 0, stream, p);
    return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
}

// ---------------------------------------------------------------------------
// Shard packing: one workgroup per shard.
//   in : inner chunks already encoded densely in Morton-rank order at
//        blob + data_start + rank * elen; nonempty flags per inner chunk
//   out: present chunks compacted (rare path: only when some inner chunk is
//        empty), index (LE u64 offset/length, MAX_UINT_64 for absent) + CRC
//        written, blob length reported (0 = all empty: delete the shard key).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void put_u32_bytes(uint8_t* d, uint32_t v) {
    d[0] = (uint8_t)v;
    d[1] = (uint8_t)(v >> 8);
    d[2] = (uint8_t)(v >> 16);
    d[3] = (uint8_t)(v >> 24);
}

__global__ __launch_bounds__(kThreads) void k_shard_pack(const PackParams p) {
    __shared__ uint32_t s_tab[16 * 256];
    __shared__ uint32_t s_scan[kThreads];
    __shared__ uint32_t s_red[kThreads / 64];
    __shared__ uint32_t s_total;
    const int t = threadIdx.x;
    const uint32_t sh = blockIdx.x;
    const zhip_shard ps = p.shards[sh];
    uint8_t* blob = p.dst + ps.blob;
    const uint32_t n = p.n_inner;
    const uint32_t data_start = p.index_start ? p.index_size : 0u;
    if (p.index_crc) {
        const uint4* g = reinterpret_cast<const uint4*>(p.horner);
        uint4* sv = reinterpret_cast<uint4*>(s_tab);
        for (int i = t; i < 1024; i += kThreads) sv[i] = g[i];
    }
    // 1. present flags in rank order -> exclusive scan (chunks of 256 ranks)
    const uint32_t* ne = p.nonempty + ps.first_chunk;  // indexed by rank
    uint32_t carry = 0;
    for (uint32_t base = 0; base < n; base += kThreads) {
        const uint32_t r = base + t;
        const uint32_t pr = (r < n) ? ((p.keep_empty || ne[r]) ? 1u : 0u) : 0u;
        s_scan[t] = pr;
        __syncthreads();
        for (int off = 1; off < kThreads; off <<= 1) {
            const uint32_t v = t >= off ? s_scan[t - off] : 0u;
            __syncthreads();
            s_scan[t] += v;
            __syncthreads();
        }
        const uint32_t incl = s_scan[t];
        const uint32_t tot = s_scan[kThreads - 1];
        __syncthreads();
        if (r < n) {
            const uint32_t newrank = carry + incl - pr;
            p.newrank[ps.first_chunk + r] = pr ? newrank : 0xFFFFFFFFu;
        }
        carry += tot;
    }
    if (t == 0) s_total = carry;
    __syncthreads();
    const uint32_t n_present = s_total;
    const bool dense = n_present == n;
    // 2. compaction (only when some inner chunk is empty), in increasing rank
    //    order so a move never overwrites a chunk that has not moved yet
    if (!dense) {
        for (uint32_t r = 0; r < n; ++r) {
            const uint32_t nr = p.newrank[ps.first_chunk + r];
            __syncthreads();
            if (nr == 0xFFFFFFFFu || nr == r) continue;
            uint8_t* from = blob + data_start + (uint64_t)r * p.elen;
            uint8_t* to = blob + data_start + (uint64_t)nr * p.elen;
            for (uint32_t i = t; i < p.elen; i += kThreads) to[i] = from[i];
        }
        __syncthreads();
    }
    if (n_present == 0) {
        if (t == 0) p.blob_len[sh] = 0;
        return;
    }
    const uint64_t blen = (uint64_t)n_present * p.elen + p.index_size;
    uint8_t* ix = blob + (p.index_start ? 0ull : (uint64_t)n_present * p.elen);
    // 3. index entries in C order: entry i at ix + 16 i; Horner CRC over them
    //    with the 4096-byte-stride tables (thread t owns entries t + 256 k)
    __syncthreads();
    uint32_t acc = 0;
    const uint32_t kiters = (n + kThreads - 1) / kThreads;
    for (uint32_t k = 0; k < kiters; ++k) {
        const uint32_t i = k * kThreads + t;
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        if (i < n) {
            const uint32_t r = p.rank_of_slot[i];
            const uint32_t nr = p.newrank[ps.first_chunk + r];
            if (nr == 0xFFFFFFFFu) {
                w[0] = w[1] = w[2] = w[3] = 0xFFFFFFFFu;
            } else {
                const uint64_t off = (uint64_t)data_start + (uint64_t)nr * p.elen;
                w[0] = (uint32_t)off;
                w[1] = (uint32_t)(off >> 32);
                w[2] = p.elen;
                w[3] = 0u;
            }
            uint8_t* e = ix + 16ull * i;
            put_u32_bytes(e, w[0]);
            put_u32_bytes(e + 4, w[1]);
            put_u32_bytes(e + 8, w[2]);
            put_u32_bytes(e + 12, w[3]);
        }
        if (p.index_crc)
            acc = tab_apply(s_tab, acc ^ w[0]) ^ tab_apply(s_tab + 1024, w[1]) ^ tab_apply(s_tab + 2048, w[2]) ^
                  tab_apply(s_tab + 3072, w[3]);
    }
    if (p.index_crc) {
        uint32_t v = gf_mul(acc, p.kthread[t]);
        v = wave_xor(v);
        if ((t & 63) == 0) s_red[t >> 6] = v;
        __syncthreads();
        if (t == 0) {
            const uint32_t V = s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3];
            const uint32_t crc = ~(gf_mul(V, p.idx_c_inv) ^ p.idx_c3);
            put_u32_bytes(ix + 16ull * n, crc);
        }
    }
    if (t == 0) p.blob_len[sh] = blen;
}

int launch_shard_pack(const PackParams& p, uint32_t n_shards, hipStream_t stream) {
    if (n_shards == 0) return ZHIP_OK;
    hipLaunchKernelGGL(k_shard_pack, dim3(n_shards), dim3(kThreads), 0, stream, p);
    return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
}

}  // namespace zhip
