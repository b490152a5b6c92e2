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

// Wave-uniform 16-byte read through the scalar data cache (read only): the
// constant address space makes the compiler emit s_load_dwordx4, which is
// tracked by lgkmcnt, so waiting for it never waits for the wave's in-flight
// vector loads or stores.  `a` must be 4-byte aligned and uniform.
typedef __attribute__((address_space(4))) const uint32_t zhip_const_u32;

// A POD object of T read dword by dword through the scalar cache (T's size a
// multiple of 4, `a` 4-byte aligned).
template <typename T>
__device__ __forceinline__ T load_uniform(const void* a) {
    static_assert(sizeof(T) % 4 == 0, "dword-sized objects only");
    const uint64_t v = reinterpret_cast<uintptr_t>(a);
    const uint64_t u = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    const zhip_const_u32* w = (const zhip_const_u32*)u;
    uint32_t d[sizeof(T) / 4];
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) d[i] = w[i];
    T r;
    __builtin_memcpy(&r, d, sizeof(T));
    return r;
}


// A wave-uniform pointer into read-only tables, in the constant address space
// (scalar loads for fields read with compile-time offsets).
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* uniform_ptr(const T* a) {
    const uint64_t v = reinterpret_cast<uintptr_t>(a);
    const uint64_t u = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    return (const __attribute__((address_space(4))) T*)u;
}

// The same address, provably wave-uniform (SGPR pair): lets the compiler use the
// SGPR-base + VGPR-offset addressing form.
template <typename T>
__device__ __forceinline__ T* uniform_addr(T* a) {
    const uint64_t v = reinterpret_cast<uintptr_t>(a);
    return reinterpret_cast<T*>(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
                                (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v));
}

// Thread t's lane-shift constant x^(8(4096 - 16t)) (the value build_tables
// stores in kthread[t]) from 32 kernel-argument constants: with t = 16a + b it
// is kq[a] * kq[16 + b], kq[a] = x^(8(4096 - 256a)), kq[16 + b] = x^(-128b).
// Computed, not loaded: nothing waits for the unit loads in flight.
__device__ __forceinline__ uint32_t lane_kthread(const DecodeParams& p, int t) {
    const uint32_t a = (uint32_t)t >> 4, b = (uint32_t)t & 15u;
    uint32_t qa = 0, pb = 0;
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) {
        qa = a == i ? p.kq[i] : qa;
        pb = b == i ? p.kq[16 + i] : pb;
    }
    return gf_mul(qa, pb);
}

// (offset, nbytes) of one shard-index entry (LE u64 pair), any alignment: the
// five aligned dwords covering it through the scalar cache, funnel-shifted.
__device__ __forceinline__ void load_index_entry(const uint8_t* e, uint64_t& off, uint64_t& len) {
    struct D5 { uint32_t d[5]; };
    const uint64_t a = reinterpret_cast<uintptr_t>(e);
    const uint32_t sh = (uint32_t)(a & 3u) * 8u;
    const D5 w = load_uniform<D5>(reinterpret_cast<const void*>(a & ~3ull));
    uint32_t x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = (uint32_t)((((uint64_t)w.d[i + 1] << 32) | w.d[i]) >> sh);
    off = ((uint64_t)x[1] << 32) | x[0];
    len = ((uint64_t)x[3] << 32) | x[2];
}

// a > b for wave-uniform u64 on the scalar ALU (it has no 64-bit ordered
// compare; the opaque halves keep LLVM from re-forming a VALU i64 compare)
__device__ __forceinline__ bool u64_gt(uint64_t a, uint64_t b) {
    uint32_t ah = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)), al = __builtin_amdgcn_readfirstlane((uint32_t)a);
    uint32_t bh = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)), bl = __builtin_amdgcn_readfirstlane((uint32_t)b);
    asm volatile("" : "+s"(ah), "+s"(al), "+s"(bh), "+s"(bl));
    return ah > bh || (ah == bh && al > bl);
}

__device__ __forceinline__ Unit resolve_unit(const DecodeParams& p, uint32_t u, uint32_t expected) {
    Unit U;
    U.c = u / p.nseg;
    U.sidx = u - U.c * p.nseg;
    const zhip_chunk ch = load_uniform<zhip_chunk>(p.chunks + U.c);
    U.mode = ZHIP_ST_OK;
    uint64_t base = ch.src;
    if (ch.flags & ZHIP_CF_MISSING) {
        U.mode = ZHIP_ST_MISSING;
    } else if (p.lflags & ZHIP_LF_SHARDED) {
        // _ShardIndex.get_chunk_slice (sharding.py:248-254): LE u64 (offset, nbytes),
        // (2^64-1, 2^64-1) = missing; offsets are absolute within the blob.
        const uint64_t ipos = (p.lflags & ZHIP_LF_INDEX_START) ? 0ull : ch.src_len - p.index_size;
        const uint8_t* e = p.src + ch.src + ipos + 16ull * ch.slot;
        uint64_t off, len;
        load_index_entry(e, off, len);
        // (64-bit compares spelled in 32-bit halves: scalar ALU, no VGPR temporaries
        // that could alias registers with loads in flight)
        if (off == ~0ull && len == ~0ull) U.mode = ZHIP_ST_MISSING;
        else if (u64_gt(off, ch.src_len) || u64_gt(len, ch.src_len - off)) U.mode = ZHIP_ST_INDEX_OOB;
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

// Unit u given the previous unit: a unit of the same chunk reuses its
// resolution (no memory access); otherwise resolve from the tables.
__device__ __forceinline__ Unit advance_unit(const DecodeParams& p, const Unit& prev, uint32_t u,
                                             uint32_t expected) {
    const uint32_t c = u / p.nseg;
    if (c == prev.c) {
        Unit U = prev;
        U.sidx = u - c * p.nseg;
        U.seg_lo = (int32_t)p.E - (int32_t)((U.sidx + 1u) * p.seg);
        return U;
    }
    return resolve_unit(p, u, expected);
}

// The Horner operator tables [op][slice][256] (op k = A_(4096 - 4k), see
// build_horner in capi.cpp) computed in LDS: entry b of (op, slice) is
// gf_mul(x_op, b << 8*slice), linear in b, so thread t = b xors the basis
// values x_op * x^(31-j) (j = 8*slice + bit) of its set bits.  The basis chain
// is wave-uniform (scalar ALU); no memory reads, so nothing here waits for the
// unit loads already in flight.
__device__ __forceinline__ uint32_t mulx1_u(uint32_t b) { return (b >> 1) ^ (kPoly & (0u - (b & 1u))); }

__device__ __forceinline__ void build_horner_lds(uint32_t* s_tab, int t, const uint32_t (&hx)[4]) {
    uint32_t m[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = 0u - (((uint32_t)t >> i) & 1u);
#pragma unroll
    for (int op = 0; op < 4; ++op) {
        uint32_t v = hx[op];
        uint32_t e[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 31; j >= 0; --j) {
            e[j >> 3] ^= v & m[j & 7];
            v = mulx1_u(v);
        }
#pragma unroll
        for (int sl = 0; sl < 4; ++sl) s_tab[op * 1024 + sl * 256 + t] = e[sl];
    }
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

// The LE u32 CRC trailer at cp + n through the scalar cache: the aligned dword
// pair covering it (the arena keeps readable slack past every blob), shifted.
__device__ __forceinline__ uint32_t load_trailer_uniform(const uint8_t* cp, uint32_t n) {
    const uint64_t a = reinterpret_cast<uintptr_t>(cp + n);
    const uint32_t sh = (uint32_t)(a & 3u) * 8u;
    const uint2 w = load_uniform<uint2>(reinterpret_cast<const void*>(a & ~3ull));
    return (uint32_t)((((uint64_t)w.y << 32) | w.x) >> sh);
}

// The whole-chunk row map's entry for step st (ZHIP_DF_WHOLE launches, plans
// with aff_ok): rel = (st >> aff_sh) B + (st & aff_mask) C + D, every row of
// the step (zhip_plan aff_*, plan_affine in capi.cpp).  DecodeParams or
// EncodeParams.
template <class P>
__device__ __forceinline__ zhip_rowblk aff_rowblk(const P& p, uint32_t st) {
    zhip_rowblk e;
    e.rel = (int32_t)(st >> p.aff_sh) * p.aff_B + (int32_t)(st & p.aff_mask) * p.aff_C + p.aff_D;
    e.lo = 0;
    e.hi = (uint16_t)((uint32_t)kWgStride >> p.row_shift);
    return e;
}

// ZHIP_DF_WHOLE is checked in the kernel, not trusted (round 6): the
// selection record of the unit's chunk must be the whole chunk -- start 0,
// count = shape, step 1 in every dimension (chunk_utils.py:88-214,
// is_complete_chunk) -- before a launch computes destinations instead of
// loading them from the row map.  Scalar loads (3 x 32 bytes) issued beside
// the data loads; a C caller's partial selection under the flag falls back to
// the map, so nothing lands outside its selection.
template <class P>
__device__ __forceinline__ bool sel_whole(const P& p, uint32_t sel) {
    struct S3 {
        int32_t v[3 * ZHIP_MAX_DIMS];
    };
    const S3 s = load_uniform<S3>(p.sels + sel);
    bool w = true;
#pragma unroll
    for (int d = 0; d < ZHIP_MAX_DIMS; ++d)
        if (d < p.g.ndim)
            w = w && s.v[d] == 0 && s.v[ZHIP_MAX_DIMS + d] == p.g.shape[d] && s.v[2 * ZHIP_MAX_DIMS + d] == 1;
    return w;
}

__device__ __forceinline__ uint32_t load_trailer(const uint8_t* cp, uint32_t n) {
    const uint8_t* tr = cp + n;
    return (uint32_t)tr[0] | ((uint32_t)tr[1] << 8) | ((uint32_t)tr[2] << 16) | ((uint32_t)tr[3] << 24);
}

// ---- deferred CRC verdicts (zarrhip.h), shared by the decode kernels that
// publish without a returning atomic ----
// {word, stored} of chunk c in the OTHER bank (the previous launch's verdict),
// read by the chunk's first workgroup; one address for every lane (`zero`
// otherwise), so every path issues the same vector load.
__device__ __forceinline__ uint64_t dv_prev(const DecodeParams& p, uint32_t c, bool first, const void* zero) {
    return __hip_atomic_load(reinterpret_cast<const uint64_t*>(
                                 first ? p.ws + 4ull * c + 2u * (p.dv_bank ^ 1u) : static_cast<const uint32_t*>(zero)),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One lane: xor the workgroup's (chunk-referenced) contribution into this
// launch's bank word -- the first workgroup also folds in c3 ^ ~stored, so
// the word ends as computed ^ stored -- and record the trailer.  The atomic's
// result is unused: nobody waits for its round trip.
__device__ __forceinline__ void dv_publish(const DecodeParams& p, uint32_t c, bool first, uint32_t V,
                                           uint32_t stored) {
    uint32_t* w = p.ws + 4ull * c + 2u * p.dv_bank;
    __hip_atomic_fetch_xor(w, V ^ (first ? (p.c3 ^ ~stored) : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (first) __hip_atomic_store(w + 1, stored, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One lane of the first workgroup, after the chunk's own status: a nonzero
// previous verdict is the previous launch's mismatch (sticky status + error
// bit); its word is cleared for the launch after this one.
__device__ __forceinline__ void dv_settle(const DecodeParams& p, uint32_t c, uint64_t prev) {
    const uint32_t pw = (uint32_t)prev, ps = (uint32_t)(prev >> 32);
    if (pw != 0u) {
        zhip_status st = {ZHIP_ST_CRC_MISMATCH, ps, pw ^ ps, 0u};
        p.status[c] = st;
        atomicOr(p.errflag, 1u << ZHIP_ST_CRC_MISMATCH);
        __hip_atomic_store(p.ws + 4ull * c + 2u * (p.dv_bank ^ 1u), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// CRC-32C check of one shard index (payload idx_nbytes + LE trailer) by one
// workgroup: the same per-thread Horner chain as a data unit ending at idx_E
// (reference point idx_E + 4096), reduced over the workgroup.  `red` is a
// 4-word LDS scratch the caller does not use concurrently.
// The first 16-byte block thread t reads for index j, loaded with exactly one
// vector load whatever the lane or index state (`dummy` when out of range), so
// it can be issued early without making the kernel's load counts path-dependent.
// Consumed by verify_index(..., &pre).
__device__ __forceinline__ uint4 index_prefetch(const DecodeParams& p, uint32_t j, bool has, int t,
                                                const uint8_t* dummy) {
    const uint8_t* a = dummy;
    if (has) {
        const zhip_chunk ch = load_uniform<zhip_chunk>(p.idx_chunks + j);
        const uint32_t nk = (p.idx_E + kWgStride - 1) / kWgStride;
        const int32_t o = (int32_t)p.idx_E - (int32_t)(nk * kWgStride) + 16 * t;
        if (ch.src_len == (uint64_t)p.idx_nbytes + 4u && o >= 0 && (uint32_t)o < p.idx_nbytes)
            a = p.src + ch.src + o;
    }
    uint4 v;
    __builtin_memcpy(&v, a, 16);
    return v;
}

__device__ __forceinline__ void verify_index(const DecodeParams& p, uint32_t j, int t, uint32_t kth,
                                          const uint32_t* s_tab, uint32_t* red, bool has_pre = false,
                                          uint4 pre = make_uint4(0, 0, 0, 0)) {
    const zhip_chunk ch = p.idx_chunks[j];
    const uint32_t ok = ch.src_len == (uint64_t)p.idx_nbytes + 4u;
    const uint8_t* cp = p.src + ch.src;
    const uint32_t nk = (p.idx_E + kWgStride - 1) / kWgStride;
    const int32_t lo = (int32_t)p.idx_E - (int32_t)(nk * kWgStride);
    uint32_t acc = 0;
    if (ok) {
        for (uint32_t k = 0; k < nk; ++k) {
            const int32_t o = lo + kWgStride * (int32_t)k + 16 * t;
            uint4 v;
            if (k == 0 && has_pre) v = (o >= 0 && (uint32_t)o < p.idx_nbytes) ? mask_tail(pre, o, p.idx_nbytes)
                                                                         : make_uint4(0, 0, 0, 0);
            else v = load_block<false>(cp, o, p.idx_nbytes);
            acc = tab_apply(s_tab, acc ^ v.x) ^ tab_apply(s_tab + 1024, v.y) ^
                  tab_apply(s_tab + 2048, v.z) ^ tab_apply(s_tab + 3072, v.w);
        }
    }
    uint32_t v = gf_mul(acc, kth);
    v = wave_xor(v);
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

// ---- the pair kernel's CRC step (k_decode_pair / k_decode_il / k_decode_tile4f;
// tables in the kPairTab* layout, built by capi.cpp build_pair_tables) ----
struct Acc4 {
    uint32_t a0, a1, a2, a3;
};

__device__ __forceinline__ uint32_t t11(const uint32_t* s, uint32_t w) {
    return s[kPairT1 + (w & 2047u)] ^ s[kPairT2 + ((w >> 11) & 2047u)] ^ s[kPairT3 + (w >> 22)];
}

__device__ __forceinline__ void crc_block4(const uint32_t* s, Acc4& a, const uint4 v) {
    a.a0 = t11(s, a.a0 ^ v.x);
    a.a1 = t11(s, a.a1 ^ v.y);
    a.a2 = t11(s, a.a2 ^ v.z);
    a.a3 = t11(s, a.a3 ^ v.w);
}

__device__ __forceinline__ uint32_t fold4(const uint32_t* s, const Acc4& a) {
    const uint32_t* t4 = s + kPairA4;
    return tab_apply(t4, tab_apply(t4, tab_apply(t4, a.a0) ^ a.a1) ^ a.a2) ^ a.a3;
}

// The same chain step and fold over byte tables (kByteTabWords: A_D's four
// 256-entry tables, then A4's): 16 lookups per block instead of 12, 8 KiB of
// LDS instead of 24 (tuning arms 66 / 67: more resident tile workgroups)
template <bool BT>
__device__ __forceinline__ void crc_block4_t(const uint32_t* s, Acc4& a, const uint4 v) {
    if constexpr (BT) {
        a.a0 = tab_apply(s, a.a0 ^ v.x);
        a.a1 = tab_apply(s, a.a1 ^ v.y);
        a.a2 = tab_apply(s, a.a2 ^ v.z);
        a.a3 = tab_apply(s, a.a3 ^ v.w);
    } else {
        crc_block4(s, a, v);
    }
}

template <bool BT>
__device__ __forceinline__ uint32_t fold4_t(const uint32_t* s, const Acc4& a) {
    if constexpr (BT) {
        const uint32_t* t4 = s + 1024;
        return tab_apply(t4, tab_apply(t4, tab_apply(t4, a.a0) ^ a.a1) ^ a.a2) ^ a.a3;
    } else {
        return fold4(s, a);
    }
}

// Per-lane multiply by a lane constant k over 3-bit windows of the operand
// (bits 0..29) and a 2-bit top window (bits 30..31), Horner over the windows
// with x^3 / x^2 steps whose reductions (r3 / r2) are VALU; the window products
// come from a 12-entry LDS column (lanemul3, decode_rows.hip) or from
// registers (lanemul_reg).
constexpr uint32_t rbasis(uint32_t n, int steps) {
    for (int i = 0; i < steps; ++i) n = (n >> 1) ^ (kPoly & (0u - (n & 1u)));
    return n;
}

__device__ __forceinline__ uint32_t r3(uint32_t n) {
    return ((n & 1u) ? rbasis(1, 3) : 0u) ^ ((n & 2u) ? rbasis(2, 3) : 0u) ^ ((n & 4u) ? rbasis(4, 3) : 0u);
}

__device__ __forceinline__ uint32_t r2(uint32_t n) {
    return ((n & 1u) ? rbasis(1, 2) : 0u) ^ ((n & 2u) ? rbasis(2, 2) : 0u);
}

// The lane's 12-entry window column of k in LDS (12 KiB for 256 lanes; the
// 4-bit form needs 16), and the multiply over it (k_decode_il, k_encode_il).
__device__ __forceinline__ void lanemul3_init(uint32_t* s_mul, int t, uint32_t k) {
    const uint32_t k1 = mulx1_u(k), k2 = mulx1_u(k1);
#pragma unroll
    for (uint32_t v = 0; v < 8; ++v)
        s_mul[v * kThreads + t] = ((v & 4u) ? k : 0u) ^ ((v & 2u) ? k1 : 0u) ^ ((v & 1u) ? k2 : 0u);
#pragma unroll
    for (uint32_t v = 0; v < 4; ++v) s_mul[(8u + v) * kThreads + t] = ((v & 2u) ? k : 0u) ^ ((v & 1u) ? k1 : 0u);
}

__device__ __forceinline__ uint32_t lanemul3(const uint32_t* s_mul, int t, uint32_t a) {
    uint32_t m[11];
#pragma unroll
    for (int j = 0; j < 10; ++j) m[j] = s_mul[((a >> (3 * j)) & 7u) * kThreads + t];
    m[10] = s_mul[(8u + (a >> 30)) * kThreads + t];
    uint32_t q = m[0];
#pragma unroll
    for (int j = 1; j < 10; ++j) q = (q >> 3) ^ r3(q & 7u) ^ m[j];
    return (q >> 2) ^ r2(q & 3u) ^ m[10];
}

// The window products selected in registers from k, kx, kx^2 (no LDS column):
// ~130 VALU instructions once per run end instead of 11 LDS reads
// (k_decode_il arms LM = 1 / 2, k_decode_tile4f).
__device__ __forceinline__ uint32_t lanemul_reg(uint32_t k, uint32_t a) {
    const uint32_t k1 = mulx1_u(k), k2 = mulx1_u(k1);
    auto sel3 = [&](uint32_t w) {
        return (k & (0u - ((w >> 2) & 1u))) ^ (k1 & (0u - ((w >> 1) & 1u))) ^ (k2 & (0u - (w & 1u)));
    };
    uint32_t q = sel3(a & 7u);
#pragma unroll
    for (int j = 1; j < 10; ++j) q = (q >> 3) ^ r3(q & 7u) ^ sel3((a >> (3 * j)) & 7u);
    const uint32_t w = a >> 30;
    return (q >> 2) ^ r2(q & 3u) ^ (k & (0u - ((w >> 1) & 1u))) ^ (k1 & (0u - (w & 1u)));
}

// Arrival of one workgroup of a grouped tile kernel (k_decode_tileg /
// k_encode_tileg) with its CRC contribution v and non-empty bit: 64-bit words
// CRC (low 32) | arrival bits (32..47) | non-empty bits (48..63), one relaxed
// XOR per level.  Up to 16 groups per chunk the chunk word is the only level;
// up to 256 the groups first meet in words of 16 (the workspace tail after the
// 4 words per chunk), whose completing arrival carries the subgroup's XOR on
// to the chunk word.  True for the arrival completing the chunk, with the
// XOR of every contribution and whether any group was non-empty.
// SPR: every subword and the chunk's word on a 128-byte line of its own
// (chunk lines at ws + 32 c, subword lines after all chunk lines;
// zhip_plan_info sizes the workspace for it), so a chunk's arrivals do not
// meet on one line: production for k_decode_tilegw's two-tile form -- C3 in
// 128^3 chunks, 256 arrivals per chunk, 28.94 / 29.00 vs 29.57 / 29.28 us
// graph-timed (profiles/r05/aa/; tuning arm 48 keeps the packed words); in
// k_encode_tileg (128 arrivals per chunk) neutral, tuning arm 47.
template <bool SPR = false>
__device__ __forceinline__ bool tileg_arrive(uint32_t* ws, uint32_t n_chunks, uint32_t c, uint32_t grp,
                                             uint32_t gpc, uint32_t n_sub, uint32_t v, bool ne, uint32_t& raw,
                                             bool& any_ne) {
    if (n_sub) {
        const uint32_t sg = grp >> 4;
        const uint32_t in_sg = min(16u, gpc - (sg << 4));
        uint64_t* sw = SPR ? reinterpret_cast<uint64_t*>(ws + 32ull * n_chunks) + ((uint64_t)c * n_sub + sg) * 16u
                           : reinterpret_cast<uint64_t*>(ws + 4ull * n_chunks) + (uint64_t)c * n_sub + sg;
        const uint64_t b = 1ull << (grp & 15u);
        const uint64_t prev = __hip_atomic_fetch_xor(sw, (b << 32) | (ne ? b << 48 : 0ull) | v, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
        if ((((prev >> 32) & 0xFFFFull) ^ b) != (1ull << in_sg) - 1ull) return false;
        __hip_atomic_store(sw, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v ^= (uint32_t)prev;
        ne = ne || ((prev >> 48) & 0xFFFFull) != 0ull;
        grp = sg;
        gpc = n_sub;
    }
    uint64_t* cw = reinterpret_cast<uint64_t*>(ws) + (SPR ? 16ull : 2ull) * c;
    const uint64_t b = 1ull << grp;
    const uint64_t prev = __hip_atomic_fetch_xor(cw, (b << 32) | (ne ? b << 48 : 0ull) | v, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if ((((prev >> 32) & 0xFFFFull) ^ b) != (1ull << gpc) - 1ull) return false;
    __hip_atomic_store(cw, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    raw = (uint32_t)prev ^ v;
    any_ne = ne || ((prev >> 48) & 0xFFFFull) != 0ull;
    return true;
}

// tileg_arrive with the look-back finalizer (round 6; tuning arms 62 / 63):
// the subwords of 16 arrivals on lines of their own (tileg_arrive SPR's
// layout; one word of up to 16 when n_sub is 0).  Every workgroup but the
// chunk's last (grp = gpc - 1) xors its bit | non-empty bit | v with a
// NON-returning atomic and returns false; the last one polls every subword
// (one lane, relaxed agent loads) until all the other arrivals are in, resets
// them and returns true with the chunk's raw sum and non-empty flag.  The
// caller takes it only while fewer chunks than CUs are in the launch (the
// finalizers then never hold every slot; publish_lb, decode_rows.hip).
__device__ __forceinline__ bool tileg_arrive_lb(uint32_t* ws, uint32_t n_chunks, uint32_t c, uint32_t grp,
                                                uint32_t gpc, uint32_t n_sub, uint32_t v, bool ne, uint32_t& raw,
                                                bool& any_ne) {
    const uint32_t nsw = n_sub ? n_sub : 1u;
    uint64_t* const base = n_sub ? reinterpret_cast<uint64_t*>(ws + 32ull * n_chunks) + (uint64_t)c * n_sub * 16u
                                 : reinterpret_cast<uint64_t*>(ws) + 16ull * c;
    const uint32_t sg = n_sub ? grp >> 4 : 0u;
    const uint64_t b = 1ull << (n_sub ? (grp & 15u) : grp);
    if (grp + 1u < gpc) {
        (void)__hip_atomic_fetch_xor(base + 16ull * sg, (b << 32) | (ne ? b << 48 : 0ull) | v, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
        return false;
    }
    uint32_t acc = v;
    bool nn = ne;
    for (uint32_t s = 0; s < nsw; ++s) {
        const uint32_t in_s = n_sub ? min(16u, gpc - 16u * s) : gpc;
        uint64_t expect = (1ull << in_s) - 1ull;
        if (s == sg) expect ^= b;
        uint64_t* const w = base + 16ull * s;
        uint64_t cur;
        for (;;) {
            cur = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (((cur >> 32) & 0xFFFFull) == expect) break;
            __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc ^= (uint32_t)cur;
        nn = nn || ((cur >> 48) & 0xFFFFull) != 0ull;
    }
    raw = acc;
    any_ne = nn;
    return true;
}

}  // namespace zhip
