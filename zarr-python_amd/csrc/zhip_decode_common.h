// Decode building blocks shared by k_decode (decode.hip) and k_decode_rows
// (decode_rows.hip): unit resolution through the shard index, unit loads,
// CRC finalisation, fused shard-index verification and the deferred arrival
// retire.  See decode.hip for the work decomposition and the CRC algebra.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/zarrhip.h"
#include "zhip_gf2.h"
#include "zhip_internal.h"
#include "zhip_device.h"

namespace zhip {

// Per-unit context (wave-uniform).
struct Unit {
    uint32_t c;       // chunk
    uint32_t sidx;    // unit index inside the chunk (0 = the one ending at E)
    uint32_t mode;    // ZHIP_ST_OK / MISSING / error code
    const uint8_t* cp;
    int32_t seg_lo;
    uint32_t sel;
    int64_t out_off;
};

__device__ __forceinline__ Unit resolve_unit(const DecodeParams& p, uint32_t u, uint32_t expected) {
    Unit U;
    U.c = u / p.nseg;
    U.sidx = u - U.c * p.nseg;
    const zhip_chunk ch = p.chunks[U.c];
    U.mode = ZHIP_ST_OK;
    uint64_t base = ch.src;
    if (ch.flags & ZHIP_CF_MISSING) {
        U.mode = ZHIP_ST_MISSING;
    } else if (p.lflags & ZHIP_LF_SHARDED) {
        // _ShardIndex.get_chunk_slice (sharding.py:248-254): LE u64 (offset, nbytes),
        // (2^64-1, 2^64-1) = missing; offsets are absolute within the blob.
        const uint64_t ipos = (p.lflags & ZHIP_LF_INDEX_START) ? 0ull : ch.src_len - p.index_size;
        const uint8_t* e = p.src + ch.src + ipos + 16ull * ch.slot;
        const uint64_t off = load_u64_le_bytes(e);
        const uint64_t len = load_u64_le_bytes(e + 8);
        if (off == ~0ull && len == ~0ull) U.mode = ZHIP_ST_MISSING;
        else if (off > ch.src_len || len > ch.src_len - off) U.mode = ZHIP_ST_INDEX_OOB;
        else if (len != expected) U.mode = ZHIP_ST_LENGTH_MISMATCH;
        else base = ch.src + off;
    } else if (ch.src_len != expected) {
        U.mode = ZHIP_ST_LENGTH_MISMATCH;
    }
    U.cp = p.src + base;
    U.seg_lo = (int32_t)p.E - (int32_t)((U.sidx + 1u) * p.seg);
    U.sel = ch.sel;
    U.out_off = ch.out_off;
    return U;
}

template <int K>
__device__ __forceinline__ void load_unit(const DecodeParams& p, const Unit& U, int t, uint4 (&blk)[K]) {
    // uniform branches (SGPR conditions): never if-convert the two load forms
    const uint32_t ok = __builtin_amdgcn_readfirstlane(U.mode == ZHIP_ST_OK ? 1u : 0u);
    const uint32_t al4 = __builtin_amdgcn_readfirstlane(
        (uint32_t)(reinterpret_cast<uintptr_t>(U.cp) & 3u) == 0u ? 1u : 0u);
    const uint32_t nt = __builtin_amdgcn_readfirstlane((p.tune & kTuneNT) && ((reinterpret_cast<uintptr_t>(U.cp) & 15u) == 0u) ? 1u : 0u);
    if (!ok) {
#pragma unroll
        for (int k = 0; k < K; ++k) blk[k] = make_uint4(0, 0, 0, 0);
    } else if (nt) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            blk[k] = load_block_t<true, true>(U.cp, U.seg_lo + kWgStride * k + 16 * t, p.g.nbytes);
    } else if (al4) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            blk[k] = load_block<true>(U.cp, U.seg_lo + kWgStride * k + 16 * t, p.g.nbytes);
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k)
            blk[k] = load_block<false>(U.cp, U.seg_lo + kWgStride * k + 16 * t, p.g.nbytes);
    }
}

// Last unit of chunk c has arrived: turn the accumulator into the CRC-32C value
// and compare with the stored little-endian trailer (crc32c_.py:41-49).
__device__ __forceinline__ void finalize_chunk(const DecodeParams& p, uint32_t c, uint32_t stored,
                                               uint32_t raw) {
    const uint32_t computed = ~(gf_mul(raw, p.c_inv) ^ p.c3);
    const uint32_t code = computed == stored ? ZHIP_ST_OK : ZHIP_ST_CRC_MISMATCH;
    zhip_status st;
    st.code = code;
    st.stored = stored;
    st.computed = computed;
    st.aux = 0;
    p.status[c] = st;
    if (code != ZHIP_ST_OK) atomicOr(p.errflag, 1u << code);
}

__device__ __forceinline__ uint32_t load_trailer(const uint8_t* cp, uint32_t n) {
    const uint8_t* tr = cp + n;
    return (uint32_t)tr[0] | ((uint32_t)tr[1] << 8) | ((uint32_t)tr[2] << 16) | ((uint32_t)tr[3] << 24);
}

// CRC-32C check of one shard index (payload idx_nbytes + LE trailer) by one
// workgroup: the same per-thread Horner chain as a data unit ending at idx_E
// (reference point idx_E + 4096), reduced over the workgroup.  `red` is a
// 4-word LDS scratch the caller does not use concurrently.
__device__ __forceinline__ void verify_index(const DecodeParams& p, uint32_t j, int t, uint32_t kth,
                                          const uint32_t* s_tab, uint32_t* red) {
    const zhip_chunk ch = p.idx_chunks[j];
    const uint32_t ok = ch.src_len == (uint64_t)p.idx_nbytes + 4u;
    const uint8_t* cp = p.src + ch.src;
    const uint32_t nk = (p.idx_E + kWgStride - 1) / kWgStride;
    const int32_t lo = (int32_t)p.idx_E - (int32_t)(nk * kWgStride);
    uint32_t acc = 0;
    if (ok) {
        for (uint32_t k = 0; k < nk; ++k) {
            const uint4 v = load_block<false>(cp, lo + kWgStride * (int32_t)k + 16 * t, p.idx_nbytes);
            acc = tab_apply(s_tab, acc ^ v.x) ^ tab_apply(s_tab + 1024, v.y) ^
                  tab_apply(s_tab + 2048, v.z) ^ tab_apply(s_tab + 3072, v.w);
        }
    }
    uint32_t v = gf_mul(acc, kth);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off, 64);
    __syncthreads();  // red may still be read from a previous index
    if ((t & 63) == 0) red[t >> 6] = v;
    __syncthreads();
    if (t == 0) {
        zhip_status st = {ZHIP_ST_LENGTH_MISMATCH, 0u, 0u, 0u};
        if (ok) {
            const uint32_t V = red[0] ^ red[1] ^ red[2] ^ red[3];
            st.stored = load_trailer(cp, p.idx_nbytes);
            st.computed = ~(gf_mul(V, p.idx_c_inv) ^ p.idx_c3);
            st.code = st.computed == st.stored ? ZHIP_ST_OK : ZHIP_ST_CRC_MISMATCH;
        }
        p.idx_status[j] = st;
        if (st.code != ZHIP_ST_OK) atomicOr(p.errflag, 1u << st.code);
    }
}

struct Pending {  // thread 0's outstanding arrival for one run, checked one run later
    uint64_t prev;
    uint32_t stored, c, bits, V, valid;
};

__device__ __forceinline__ void retire(const DecodeParams& p, Pending& q, uint64_t full) {
    if (!q.valid) return;
    q.valid = 0;
    if (((q.prev >> 32) ^ q.bits) == full) {
        uint64_t* w = reinterpret_cast<uint64_t*>(p.ws) + 2ull * q.c;
        __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        finalize_chunk(p, q.c, q.stored, (uint32_t)q.prev ^ q.V);
    }
}

}  // namespace zhip
