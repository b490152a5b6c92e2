// k_decode_rows: the whole-row decode with an affine per-step out mapping.
//
// Same work decomposition, CRC algebra, arrival protocol and fused shard-index
// checks as k_decode (decode.hip), for the layouts the headline configs use:
// every chunk selects whole innermost rows with unit steps, rows are
// 2^row_shift <= 4096 bytes and contiguous in out, and shape[ndim-2] is a
// multiple of the rows one workgroup step covers (4096 / row_bytes).  Then
// step k of a unit covers rows [R_k, R_k + 4096/row_bytes) of ONE dim-(ndim-2)
// run, so the out address of thread t's block is
//     base(R_k)  (wave-uniform, scalar ALU)  +  lane_off(t)  (per lane, once)
// and the per-block selection test is one compare on the dim-(ndim-2)
// coordinate.  Loads and stores are nontemporal (every byte is touched once).
//
// Reference behaviour restated: Crc32cCodec._decode_sync (crc32c_.py:34-50),
// BytesCodec._decode_sync (bytes.py:97-131), scatter_chunk /
// decode_and_scatter_chunk (chunk_utils.py:88-214), _ShardIndex.get_chunk_slice
// (sharding.py:248-254), _decode_shard_index_sync (sharding.py:624-631).
#include <hip/hip_runtime.h>

#include "../../include/zarrhip.h"
#include "zhip_gf2.h"
#include "zhip_internal.h"
#include "zhip_device.h"
#include "zhip_decode_common.h"

namespace zhip {

namespace {

template <int kRowsK>
__device__ __forceinline__ void load_unit_rows(const DecodeParams& p, const Unit& U, int t, uint4 (&blk)[kRowsK]) {
    const uint32_t ok = __builtin_amdgcn_readfirstlane(U.mode == ZHIP_ST_OK ? 1u : 0u);
    const uint32_t al4 = __builtin_amdgcn_readfirstlane(
        (uint32_t)(reinterpret_cast<uintptr_t>(U.cp) & 3u) == 0u ? 1u : 0u);
    if (!ok) {
#pragma unroll
        for (int k = 0; k < kRowsK; ++k) blk[k] = make_uint4(0, 0, 0, 0);
    } else if (al4) {
        // N is a multiple of 4096: a step is wholly inside [0, N) or wholly before it
#pragma unroll
        for (int k = 0; k < kRowsK; ++k) {
            const int32_t base = U.seg_lo + kWgStride * k;
            blk[k] = base >= 0 ? load_nt16(U.cp + base + 16 * t) : make_uint4(0, 0, 0, 0);
        }
    } else {
#pragma unroll
        for (int k = 0; k < kRowsK; ++k)
            blk[k] = load_block<false>(U.cp, U.seg_lo + kWgStride * k + 16 * t, p.g.nbytes);
    }
}

// Per-lane GF(2) multiply by the thread's fixed shift constant kth (4-bit
// windows): s_mul[v*256 + t] = (v << 28) * kth, s_r4[n] = n * x^4, so
// a * kth = Horner over the 8 nibbles of a with p <- p*x^4 ^ s_mul[nibble].
// 8 conflict-free LDS reads + 7 reduction reads instead of a 32-step loop.
__device__ __forceinline__ uint32_t mulx1(uint32_t b) { return (b >> 1) ^ (kPoly & (0u - (b & 1u))); }

__device__ __forceinline__ void lanemul_init(uint32_t* s_mul, uint32_t* s_r4, int t, uint32_t kth) {
    const uint32_t m8 = kth, m4 = mulx1(m8), m2 = mulx1(m4), m1 = mulx1(m2);
#pragma unroll
    for (uint32_t v = 0; v < 16; ++v)
        s_mul[v * kThreads + t] = ((v & 8u) ? m8 : 0u) ^ ((v & 4u) ? m4 : 0u) ^ ((v & 2u) ? m2 : 0u) ^
                                  ((v & 1u) ? m1 : 0u);
    if (t < 16) s_r4[t] = mulx1(mulx1(mulx1(mulx1((uint32_t)t))));
}

__device__ __forceinline__ uint32_t lanemul(const uint32_t* s_mul, const uint32_t* s_r4, int t, uint32_t a) {
    uint32_t p = s_mul[(a & 15u) * kThreads + t];
#pragma unroll
    for (int j = 1; j < 8; ++j)
        p = (p >> 4) ^ s_r4[p & 15u] ^ s_mul[((a >> (4 * j)) & 15u) * kThreads + t];
    return p;
}

// Wave-uniform multiply (scalar ALU): both operands are read from lane 0.
__device__ __forceinline__ uint32_t gf_mul_uniform(uint32_t a, uint32_t b) {
    return gf_mul(__builtin_amdgcn_readfirstlane(a), __builtin_amdgcn_readfirstlane(b));
}

// The arrival protocol of k_decode, executed wave-uniformly by wave 0 so the
// GF(2) work runs on the scalar unit; only lane 0 touches memory.
struct PendingU {
    uint64_t prev;  // lane 0: returned 64-bit arrival word (consumed one run later)
    uint32_t stored, c, bits, V, valid;
};

__device__ __forceinline__ void finalize_uniform(const DecodeParams& p, uint32_t c, uint32_t stored, uint32_t raw,
                                                 int t) {
    const uint32_t computed = ~(gf_mul_uniform(raw, p.c_inv) ^ p.c3);
    const uint32_t code = computed == stored ? ZHIP_ST_OK : ZHIP_ST_CRC_MISMATCH;
    if (t == 0) {
        zhip_status st = {code, stored, computed, 0u};
        p.status[c] = st;
        if (code != ZHIP_ST_OK) atomicOr(p.errflag, 1u << code);
    }
}

__device__ __forceinline__ void retire_uniform(const DecodeParams& p, PendingU& q, uint64_t full, int t) {
    if (!q.valid) return;
    q.valid = 0;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)q.prev);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(q.prev >> 32));
    if ((uint64_t)(hi ^ q.bits) == full) {
        if (t == 0) {
            uint64_t* w = reinterpret_cast<uint64_t*>(p.ws) + 2ull * q.c;
            __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        finalize_uniform(p, q.c, q.stored, lo ^ q.V, t);
    }
}

}  // namespace

template <bool CRC, int ITEM, bool SWAP, int K = 8>
__global__ __launch_bounds__(kThreads) void k_decode_rows(const DecodeParams p) {
    __shared__ uint32_t s_tab[CRC ? 16 * 256 : 1];
    __shared__ uint32_t s_mul[CRC ? 16 * kThreads : 1];
    __shared__ uint32_t s_r4[16];
    __shared__ uint32_t s_red[2][kThreads / 64];
    const int t = threadIdx.x;
    const uint32_t G = gridDim.x, g = blockIdx.x;
    const uint32_t per = p.n_units / G, rem = p.n_units % G;
    const uint32_t q0 = g * per + (g < rem ? g : rem);
    const uint32_t q1 = q0 + per + (g < rem ? 1u : 0u);
    if (q0 >= q1 && g >= p.n_idx) return;
    const uint32_t expected = p.g.nbytes + (CRC ? 4u : 0u);
    auto unit_of = [&](uint32_t q) {
        const uint32_t c = q / p.nseg;
        return c * p.nseg + (p.nseg - 1u - (q - c * p.nseg));
    };
    uint4 A[K], B[K];
    Unit ua;
    uint32_t stored = 0;
    // first unit's loads go out before anything else (tables, index checks)
    if (q0 < q1) {
        ua = resolve_unit(p, unit_of(q0), expected);
        load_unit_rows(p, ua, t, A);
        if (CRC && t == 0 && ua.mode == ZHIP_ST_OK) stored = load_trailer(ua.cp, p.g.nbytes);
    }
    uint32_t kth = 0;
    if constexpr (CRC) {
        const uint4* gt = reinterpret_cast<const uint4*>(p.horner);
        uint4* sv = reinterpret_cast<uint4*>(s_tab);
        for (int i = t; i < 1024; i += kThreads) sv[i] = gt[i];
        kth = p.kthread[t];
        lanemul_init(s_mul, s_r4, t, kth);
        __syncthreads();
        for (uint32_t j = g; j < p.n_idx; j += G) verify_index(p, j, t, kth, s_tab, s_red[1]);
    }
    if (q0 >= q1) return;

    // per-lane part of the out address: row t*16 >> row_shift of the step, column t*16 mod row
    const uint32_t lane_row = (16u * (uint32_t)t) >> p.row_shift;
    const uint32_t lane_col = (16u * (uint32_t)t) & ((1u << p.row_shift) - 1u);
    const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
    const bool one_atomic = p.nseg <= 32;
    const uint64_t full = p.nseg >= 32 ? 0xFFFFFFFFull : ((1ull << p.nseg) - 1ull);
    PendingU pend;
    pend.valid = 0;
    uint32_t acc = 0, run_bits = 0, parity = 0;
    for (uint32_t q = q0;;) {
        const uint32_t qn = q + 1;
        const bool more = qn < q1;
        Unit ub;
        if (more) {
            ub = resolve_unit(p, unit_of(qn), expected);
            load_unit_rows(p, ub, t, B);
        }
        const bool run_end = !more || ub.c != ua.c;
        const zhip_sel& sel = p.sels[ua.sel];
        const bool present = ua.mode == ZHIP_ST_OK;
        if (present || ua.mode == ZHIP_ST_MISSING) {
            // selection of dim ndim-2 (unit steps; innermost rows are whole)
            const int32_t sy0 = sel.start[p.nd2];
            const uint32_t cy = (uint32_t)sel.count[p.nd2];
            const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int32_t base_o = ua.seg_lo + kWgStride * k;
                if (base_o < 0) continue;
                const uint32_t R = (uint32_t)base_o >> p.row_shift;
                uint32_t r = fdiv_apply(R, p.r_dy.m, p.r_dy.s);
                const uint32_t y0 = R - r * p.r_sy;
                int64_t dst = ua.out_off + (int64_t)((int32_t)y0 - sy0) * p.r_oy;
                bool uok = true;
#pragma unroll
                for (int d = ZHIP_MAX_DIMS - 3; d >= 0; --d) {
                    if (d >= p.nd2) continue;
                    const uint32_t qd = d > 0 ? fdiv_apply(r, p.g.dshape[d].m, p.g.dshape[d].s) : 0u;
                    const int32_t rel = (int32_t)(r - qd * (uint32_t)p.g.shape[d]) - sel.start[d];
                    r = qd;
                    uok = uok && rel >= 0 && rel < sel.count[d];
                    dst += (int64_t)rel * p.g.ostride[d];
                }
                if (!uok) continue;
                if ((uint32_t)((int32_t)(y0 + lane_row) - sy0) >= cy) continue;
                store_nt16(p.out + dst + lane_off, present ? swap_block<ITEM, SWAP>(A[k]) : f);
            }
        }
        if (present) {
            if constexpr (CRC) {
                if (p.tune & kTuneSkipCrc) {  // ablation: lookups replaced by a plain xor
#pragma unroll
                    for (int k = 0; k < K; ++k) acc ^= A[k].x ^ A[k].y ^ A[k].z ^ A[k].w;
                } else {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const uint4 v = A[k];
                        acc = tab_apply(s_tab, acc ^ v.x) ^ tab_apply(s_tab + 1024, v.y) ^
                              tab_apply(s_tab + 2048, v.z) ^ tab_apply(s_tab + 3072, v.w);
                    }
                }
                run_bits |= 1u << (ua.sidx & 31u);
                if (run_end) {
                    uint32_t v = (p.tune & kTuneNoLaneMul) ? acc : lanemul(s_mul, s_r4, t, acc);
#pragma unroll
                    for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off, 64);
                    if ((t & 63) == 0) s_red[parity][t >> 6] = v;
                    __syncthreads();
                    if (t < 64) {  // wave 0, wave-uniform
                        const uint32_t V = gf_mul_uniform(
                            s_red[parity][0] ^ s_red[parity][1] ^ s_red[parity][2] ^ s_red[parity][3],
                            p.kunit[ua.sidx]);
                        if (p.tune & kTuneNoTicket) {  // ablation: no publication / last-arriver
                            if (t == 0 && V == 0x9E3779B9u) p.status[ua.c].aux = V;
                        } else if (one_atomic) {
                            retire_uniform(p, pend, full, t);  // the previous run's arrival returned by now
                            if (t == 0) {
                                uint64_t* w = reinterpret_cast<uint64_t*>(p.ws) + 2ull * ua.c;
                                pend.prev = __hip_atomic_fetch_xor(w, ((uint64_t)run_bits << 32) | V,
                                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            }
                            pend.stored = __builtin_amdgcn_readfirstlane(stored);
                            pend.c = ua.c;
                            pend.bits = run_bits;
                            pend.V = V;
                            pend.valid = 1;
                        } else {
                            // > 32 units per chunk: xor, then count arrivals
                            uint32_t raw = 0, last = 0;
                            const uint32_t n_run = __builtin_popcount(run_bits);
                            if (t == 0) {
                                uint32_t* accw = p.ws + 4ull * ua.c;
                                const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED,
                                                                             __HIP_MEMORY_SCOPE_AGENT);
                                asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
                                const uint32_t tk = __hip_atomic_fetch_add(accw + 2, n_run, __ATOMIC_RELAXED,
                                                                           __HIP_MEMORY_SCOPE_AGENT);
                                if (tk + n_run == p.nseg) {
                                    raw = __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                    __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                    last = 1;
                                }
                            }
                            if (__builtin_amdgcn_readfirstlane(last))
                                finalize_uniform(p, ua.c, __builtin_amdgcn_readfirstlane(stored),
                                                 __builtin_amdgcn_readfirstlane(raw), t);
                        }
                    }
                    parity ^= 1u;
                    acc = 0;
                    run_bits = 0;
                }
            } else {
                if (ua.sidx == 0 && t == 0) {
                    zhip_status st = {ZHIP_ST_OK, 0u, 0u, 0u};
                    p.status[ua.c] = st;
                }
            }
        } else if (ua.sidx == 0 && t == 0) {
            zhip_status st = {ua.mode, 0u, 0u, 0u};
            p.status[ua.c] = st;
            if (ua.mode != ZHIP_ST_MISSING) atomicOr(p.errflag, 1u << ua.mode);
        }
        if (!more) break;
        if (CRC && t == 0 && ub.c != ua.c && ub.mode == ZHIP_ST_OK) stored = load_trailer(ub.cp, p.g.nbytes);
        q = qn;
        ua = ub;
#pragma unroll
        for (int k = 0; k < K; ++k) A[k] = B[k];
    }
    if (t < 64) retire_uniform(p, pend, full, t);
}

using KernelFn = void (*)(const DecodeParams);

KernelFn select_rows_kernel(bool crc, int item, bool swap, int k) {
    if (k == 4) {  // 16 KiB units (tuning arm)
        if (crc && item == 4 && !swap) return k_decode_rows<true, 4, false, 4>;
        return nullptr;
    }
    if (k != 8) return nullptr;
    switch (item) {
        case 1: return crc ? k_decode_rows<true, 1, false> : k_decode_rows<false, 1, false>;
        case 2: return crc ? (swap ? k_decode_rows<true, 2, true> : k_decode_rows<true, 2, false>)
                           : (swap ? k_decode_rows<false, 2, true> : k_decode_rows<false, 2, false>);
        case 4: return crc ? (swap ? k_decode_rows<true, 4, true> : k_decode_rows<true, 4, false>)
                           : (swap ? k_decode_rows<false, 4, true> : k_decode_rows<false, 4, false>);
        case 8: return crc ? (swap ? k_decode_rows<true, 8, true> : k_decode_rows<true, 8, false>)
                           : (swap ? k_decode_rows<false, 8, true> : k_decode_rows<false, 8, false>);
        default: return nullptr;
    }
}

}  // namespace zhip
