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
// coordinate.  Stores are nontemporal (every byte is touched once); loads take
// the default policy (kNtLoads: measured faster).
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

// Every wave issues exactly K vector loads per unit, whatever the unit's state:
// blocks outside the chunk and units that are missing or failed read zeros
// from g_rows_zero (leading zeros do not change a CRC).  With a path-independent
// count the compiler can wait for a unit's data with vmcnt(N > 0), leaving the
// next unit's loads in flight (vmcnt counts in issue order; a path with fewer
// memory operations would force vmcnt(0)).  N is a multiple of 4096 here, so a
// step lies wholly inside [0, N) or wholly before it.
typedef unsigned int zhip_v4u_a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) const zhip_v4u_a1 zhip_gv4u_a1;

typedef __attribute__((address_space(1))) const uint32_t zhip_gu32_a1 __attribute__((aligned(1)));

__device__ __forceinline__ uint32_t load_u32_any(const uint8_t* a) {  // any alignment, one global dword
    return *(zhip_gu32_a1*)(reinterpret_cast<uintptr_t>(a));
}

__device__ __forceinline__ uint4 load16_any(const uint8_t* a) {  // any alignment, one global dwordx4, default policy
    const zhip_v4u_a1 w = *(zhip_gv4u_a1*)(reinterpret_cast<uintptr_t>(a));
    return make_uint4(w.x, w.y, w.z, w.w);
}

__device__ __forceinline__ uint4 load_stream16_any(const uint8_t* a) {  // any alignment, one global dwordx4 (kNtLoads)
    if constexpr (!kNtLoads) return load16_any(a);
    const zhip_v4u_a1 w = __builtin_nontemporal_load((zhip_gv4u_a1*)(reinterpret_cast<uintptr_t>(a)));
    return make_uint4(w.x, w.y, w.z, w.w);
}

// phase timestamps (diagnostics, kTuneStamp): [wg][slot]
__device__ uint64_t g_stamps[kStampWG * kStampSlots];

__device__ __forceinline__ void stamp(uint32_t tune, uint32_t g, int t, int slot) {
    if ((tune & kTuneStamp) && t == 0 && g < kStampWG) {
        uint64_t v = __builtin_amdgcn_s_memrealtime();
        if (slot == 0) {  // slot 0 also carries the hardware id (XCC / SE / CU) in the top bits
            uint32_t hw;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            uint32_t xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            v = (v & 0xFFFFFFFFull) | ((uint64_t)(hw & 0xFFFFFFu) << 32) | ((uint64_t)(xcc & 0xFu) << 56);
        }
        g_stamps[g * kStampSlots + slot] = v;
    }
}

__device__ __forceinline__ void stamp(const DecodeParams& p, uint32_t g, int t, int slot) { stamp(p.tune, g, t, slot); }

// zeros: blocks outside the chunk and units that are not present read here
__device__ uint4 g_rows_zero[kThreads];

template <int kRowsK>
__device__ __forceinline__ void load_unit_rows(const Unit& U, bool live, int t, uint4 (&blk)[kRowsK]) {
    const bool ok = live && U.mode == ZHIP_ST_OK;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_rows_zero);
#pragma unroll
    for (int k = 0; k < kRowsK; ++k) {
        // dummy loads: every lane reads the same 16 zero bytes (one cache line
        // per wave instruction, no traffic to speak of)
        const int32_t base = U.seg_lo + kWgStride * k;
        blk[k] = load_stream16_any(ok && base >= 0 ? U.cp + base + 16 * t : zero);
    }
}

// The unit a prediction (zhip_predict) says unit u is: present, at the
// predicted payload address.  Only its cp / seg_lo are used (for the loads).
__device__ __forceinline__ Unit predict_unit(const DecodeParams& p, uint32_t u) {
    Unit U;
    U.c = u / p.nseg;
    U.sidx = u - U.c * p.nseg;
    U.mode = ZHIP_ST_OK;
    const uint32_t grp = U.c / p.pred_per;
    const uint64_t off = p.pred_base + (uint64_t)grp * p.pred_outer + (uint64_t)(U.c - grp * p.pred_per) * p.pred_inner;
    U.cp = p.src + off;
    U.seg_lo = (int32_t)p.E - (int32_t)((U.sidx + 1u) * p.seg);
    U.sel = 0;
    U.out_off = 0;
    return U;
}

// The kernel arguments k_decode_pair needs before its first loads (PairHot),
// forced into SGPRs at one point: every s_load of the batch is issued before
// a single wait, instead of one dependent round trip per branch that first
// uses a field.
__device__ __forceinline__ void pair_hot(PairHot& h) {
    asm volatile("" : "+s"(h.n_units), "+s"(h.nseg), "+s"(h.n_idx), "+s"(h.xcd_run), "+s"(h.d_nseg.m),
                 "+s"(h.d_nseg.s), "+s"(h.d_xcd.m), "+s"(h.d_xcd.s), "+s"(h.d_per.m), "+s"(h.d_per.s), "+s"(h.pred),
                 "+s"(h.pred_per), "+s"(h.E), "+s"(h.seg), "+s"(h.tune));
    asm volatile("" : "+s"(h.pred_base), "+s"(h.pred_outer), "+s"(h.pred_inner), "+s"(h.src), "+s"(h.pair_tab),
                 "+s"(h.kpair11), "+s"(h.kthread11));
}

// k_decode_il's part of the batch (with pair_hot)
__device__ __forceinline__ void il_hot(PairHot& h) {
    asm volatile("" : "+s"(h.il_S), "+s"(h.n_chunks), "+s"(h.il_tab), "+s"(h.il_klane), "+s"(h.il_kidx));
}

// predict_unit from the PairHot batch (magic divisions, no kernarg reloads)
__device__ __forceinline__ Unit predict_unit_h(const PairHot& h, uint32_t u) {
    Unit U;
    U.c = fdiv_apply(u, h.d_nseg.m, h.d_nseg.s);
    U.sidx = u - U.c * h.nseg;
    U.mode = ZHIP_ST_OK;
    const uint32_t grp = fdiv_apply(U.c, h.d_per.m, h.d_per.s);
    const uint64_t off = h.pred_base + (uint64_t)grp * h.pred_outer + (uint64_t)(U.c - grp * h.pred_per) * h.pred_inner;
    U.cp = reinterpret_cast<const uint8_t*>(h.src) + off;
    U.seg_lo = (int32_t)h.E - (int32_t)((U.sidx + 1u) * h.seg);
    U.sel = 0;
    U.out_off = 0;
    return U;
}

// Stores that fall outside the selection go to this sink instead of being
// skipped, so every unit issues exactly K stores (see load_unit_rows).
__device__ uint4 g_rows_sink[kThreads];

// Per-lane GF(2) multiply by the thread's fixed shift constant kth (4-bit
// windows): s_mul[v*256 + t] = (v << 28) * kth, s_r4[n] = n * x^4, so
// a * kth = Horner over the 8 nibbles of a with p <- p*x^4 ^ s_mul[nibble].
// 8 conflict-free LDS reads + 7 reduction reads instead of a 32-step loop.
__device__ __forceinline__ uint32_t mulx1(uint32_t b) { return (b >> 1) ^ (kPoly & (0u - (b & 1u))); }

__device__ __forceinline__ void lanemul_init(uint32_t* s_mul, int t, uint32_t kth) {
    const uint32_t m8 = kth, m4 = mulx1(m8), m2 = mulx1(m4), m1 = mulx1(m2);
#pragma unroll
    for (uint32_t v = 0; v < 16; ++v)
        s_mul[v * kThreads + t] = ((v & 8u) ? m8 : 0u) ^ ((v & 4u) ? m4 : 0u) ^ ((v & 2u) ? m2 : 0u) ^
                                  ((v & 1u) ? m1 : 0u);
}


// n * x^4 for a nibble n (the reduction of a 4-bit right shift), from its
// four basis values: VALU only, so the Horner chain below has no LDS round
// trips (the s_mul reads do not depend on it and all go out first).
constexpr uint32_t r4_basis(uint32_t n) {
    for (int i = 0; i < 4; ++i) n = (n >> 1) ^ (kPoly & (0u - (n & 1u)));
    return n;
}

__device__ __forceinline__ uint32_t r4(uint32_t n) {
    return ((n & 1u) ? r4_basis(1) : 0u) ^ ((n & 2u) ? r4_basis(2) : 0u) ^ ((n & 4u) ? r4_basis(4) : 0u) ^
           ((n & 8u) ? r4_basis(8) : 0u);
}

__device__ __forceinline__ uint32_t lanemul(const uint32_t* s_mul, const uint32_t* /*s_r4*/, int t, uint32_t a) {
    uint32_t m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = s_mul[((a >> (4 * j)) & 15u) * kThreads + t];
    uint32_t p = m[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) p = (p >> 4) ^ r4(p & 15u) ^ m[j];
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
                                                 int t, bool scaled = false) {
    const uint32_t computed = ~((scaled ? raw : gf_mul_uniform(raw, p.c_inv)) ^ p.c3);
    const uint32_t code = computed == stored ? ZHIP_ST_OK : ZHIP_ST_CRC_MISMATCH;
    if (t == 0) {
        zhip_status st = {code, stored, computed, 0u};
        p.status[c] = st;
        if (code != ZHIP_ST_OK) atomicOr(p.errflag, 1u << code);
    }
}

__device__ __forceinline__ void retire_uniform(const DecodeParams& p, PendingU& q, uint64_t full, int t,
                                               bool scaled = false) {
    if (!q.valid) return;
    q.valid = 0;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)q.prev);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(q.prev >> 32));
    if ((uint64_t)(hi ^ q.bits) == full) {
        if (t == 0) {
            uint64_t* w = reinterpret_cast<uint64_t*>(p.ws) + 2ull * q.c;
            __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        finalize_uniform(p, q.c, q.stored, lo ^ q.V, t, scaled);
    }
}

}  // namespace

template <bool CRC, int ITEM, bool SWAP, int K = 8>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_decode_rows(const DecodeParams p) {
    __shared__ uint32_t s_tab[CRC ? 16 * 256 : 1];
    __shared__ uint32_t s_mul[CRC ? 16 * kThreads : 1];
    __shared__ uint32_t s_r4[16];
    __shared__ uint32_t s_red[2][kThreads / 64];
    __shared__ uint4 s_idx[CRC ? kThreads : 1];
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
    const uint8_t* dummy = reinterpret_cast<const uint8_t*>(g_rows_zero);
    uint8_t* sink = reinterpret_cast<uint8_t*>(g_rows_sink);  // one line: garbage for every lane

    // Prologue.  Memory order per wave: unit q0 (K loads), this workgroup's
    // first shard-index block (1 load), then at the loop top unit q0+1 (K
    // loads).  Unit headers (chunk record, shard-index entry, CRC trailer) are
    // scalar loads and the CRC tables are computed, so nothing here waits on
    // vector memory: the first wait (unit q0's data) leaves K + 1 loads in
    // flight.
    uint4 A[K], B[K];
    Unit ua, ub;
    uint32_t stored = 0;
    const bool units = q0 < q1;
    if (units) {
        ua = resolve_unit(p, unit_of(q0), expected);
        load_unit_rows(ua, true, t, A);
        if (CRC && ua.mode == ZHIP_ST_OK) stored = load_trailer_uniform(ua.cp, p.g.nbytes);
    }
    uint4 ipre = make_uint4(0, 0, 0, 0);
    uint32_t kth = 0;
    if constexpr (CRC) {
        ipre = index_prefetch(p, g, g < p.n_idx, t, dummy);
        build_horner_lds(s_tab, t, p.hx);
        kth = lane_kthread(p, t);
        if (t < 16) s_r4[t] = mulx1(mulx1(mulx1(mulx1((uint32_t)t))));
        lanemul_init(s_mul, t, kth);
        __syncthreads();
    }
    if (!units) {  // index checks only
        if constexpr (CRC)
            for (uint32_t j = g; j < p.n_idx; j += G) verify_index(p, j, t, kth, s_tab, s_red[1], j == g, ipre);
        return;
    }

    // per-lane part of the out address: row t*16 >> row_shift of the step, column t*16 mod row
    const uint32_t lane_row = (16u * (uint32_t)t) >> p.row_shift;
    const uint32_t lane_col = (16u * (uint32_t)t) & ((1u << p.row_shift) - 1u);
    const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
    const bool one_atomic = p.nseg <= 32;
    const uint64_t full = p.nseg >= 32 ? 0xFFFFFFFFull : ((1ull << p.nseg) - 1ull);
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
    PendingU pend;
    pend.valid = 0;
    uint32_t acc = 0, run_bits = 0, parity = 0;
    uint32_t first = 1u;
    ub = ua;
    for (uint32_t q = q0;;) {
        // the next unit's K loads go out before this one is processed (dummy
        // loads after the last unit keep the per-iteration count fixed)
        const uint32_t qn = q + 1;
        const bool more = qn < q1;
        if (more) ub = advance_unit(p, ua, unit_of(qn), expected);
        load_unit_rows(ub, more, t, B);
        if constexpr (CRC) {
            // the prefetched shard-index block (issued after unit q0, before
            // unit q0+1) parks in LDS until the index checks after the loop
            if (first) s_idx[t] = ipre;
            ipre = make_uint4(0, 0, 0, 0);
        }
        const bool run_end = !more || ub.c != ua.c;
        const auto& sel = *uniform_ptr(p.sels + ua.sel);
        const bool present = ua.mode == ZHIP_ST_OK;
        const bool writes = present || ua.mode == ZHIP_ST_MISSING;
        // selection of dim ndim-2 (unit steps; innermost rows are whole)
        const int32_t sy0 = sel.start[p.nd2];
        const uint32_t cy = (uint32_t)sel.count[p.nd2];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int32_t base_o = ua.seg_lo + kWgStride * k;
            const uint32_t R = (uint32_t)base_o >> p.row_shift;
            uint32_t r = fdiv_apply(R, p.r_dy.m, p.r_dy.s);
            const uint32_t y0 = R - r * p.r_sy;
            int64_t dst = ua.out_off + (int64_t)((int32_t)y0 - sy0) * p.r_oy;
            bool uok = writes && base_o >= 0;
#pragma unroll
            for (int d = ZHIP_MAX_DIMS - 3; d >= 0; --d) {
                if (d >= p.nd2) continue;
                const uint32_t qd = d > 0 ? fdiv_apply(r, p.g.dshape[d].m, p.g.dshape[d].s) : 0u;
                const int32_t rel = (int32_t)(r - qd * (uint32_t)p.g.shape[d]) - sel.start[d];
                r = qd;
                uok = uok && rel >= 0 && rel < sel.count[d];
                dst += (int64_t)rel * p.g.ostride[d];
            }
            // every lane stores (to the sink when outside the selection): K stores per unit
            const bool wr = uok && (uint32_t)((int32_t)(y0 + lane_row) - sy0) < cy;
            store_nt16(wr ? p.out + dst + lane_off : sink, present ? swap_block<ITEM, SWAP>(A[k]) : f);
        }
        if (present) {
            if constexpr (CRC) {
                if (p.tune & kTuneSkipCrc) {  // ablation: lookups replaced by a plain xor
#pragma unroll
                    for (int k = 0; k < K; ++k) acc ^= A[k].x ^ A[k].y ^ A[k].z ^ A[k].w;
                } else {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const uint4 v = A[k];  // blocks before the chunk start read zeros
                        acc = tab_apply(s_tab, acc ^ v.x) ^ tab_apply(s_tab + 1024, v.y) ^
                              tab_apply(s_tab + 2048, v.z) ^ tab_apply(s_tab + 3072, v.w);
                    }
                }
                run_bits |= 1u << (ua.sidx & 31u);
                if (run_end) {
                    uint32_t v = (p.tune & kTuneNoLaneMul) ? acc : lanemul(s_mul, s_r4, t, acc);
                    v = wave_xor(v);
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
                    // consume the returned value here (rare path): a register with a
                    // load still pending would make every later write to it wait
                    // for the wave's stores too
                    asm volatile("s_waitcnt vmcnt(0)" ::"v"(raw) : "memory");
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
        if constexpr (CRC) {
            first = 0u;
            asm volatile("" : "+s"(first));  // opaque: no first-iteration peeling
        }
        if (!more) break;
        if (CRC && ub.c != ua.c && ub.mode == ZHIP_ST_OK) stored = load_trailer_uniform(ub.cp, p.g.nbytes);
        q = qn;
        ua = ub;
#pragma unroll
        for (int k = 0; k < K; ++k) A[k] = B[k];
    }
    if constexpr (CRC) {
        // fused shard-index checks: the first block is resident in LDS
        __syncthreads();
        for (uint32_t j = g; j < p.n_idx; j += G) {
            verify_index(p, j, t, kth, s_tab, s_red[1], j == g, s_idx[t]);
        }
    }
    if (t < 64) retire_uniform(p, pend, full, t);
}

// ---------------------------------------------------------------------------
// k_decode_pair: the same decode with a non-persistent grid, one workgroup per
// pair of consecutive units (2 x 32 KiB).  Straight-line: both units' loads go
// out first, then both units' stores (as each arrives), then both units' CRC
// lookups — so the writes never queue behind LDS work, and the hardware
// dispatcher overlaps one workgroup's CRC tail with the next one's loads on
// the same CU.  The CRC tables are computed in LDS (no loads), so a short-lived
// workgroup costs no extra memory traffic.  Index checks run in the lowest
// workgroups (dispatched first, finished early).

__device__ __forceinline__ uint32_t crc_block(const uint32_t* s_tab, uint32_t acc, const uint4 v) {
    return tab_apply(s_tab, acc ^ v.x) ^ tab_apply(s_tab + 1024, v.y) ^ tab_apply(s_tab + 2048, v.z) ^
           tab_apply(s_tab + 3072, v.w);
}

// ---- k_decode_pair's CRC (tables: kPairTab* layout, built by capi.cpp) ----
// Every word of a 16-byte block is carried by its own accumulator through ONE
// operator, A4096 (multiply by x^(8*4096)), looked up by the word's 11 low,
// 11 middle and 10 high bits: 3 LDS reads per word instead of 4 byte reads
// into four per-position tables.  At a run end the four accumulators fold
// into one state with the A4 byte tables, a3 ^ A4(a2 ^ A4(a1 ^ A4(a0))), which
// sits 12 bytes after the single-chain state of the other kernels; the lane
// constants kpair11 / kthread11 carry the x^(-96) that undoes it.  (The CPU
// emulation zhip_emulate_chunk_crc_pair checks this decomposition.)  The step
// (Acc4, t11, crc_block4, fold4) lives in zhip_decode_common.h, shared with
// k_decode_tile4f.

// Timing arm (kTuneCfLookup): the same three lookups per word at addresses
// whose bank is the lane's own (index bits << 5 | lane % 32), so no ds_read_b32
// group conflicts -- the cost of the CRC lookups without bank conflicts.
// Results invalid.
__device__ __forceinline__ uint32_t t11_cf(const uint32_t* s, uint32_t w, uint32_t ln) {
    return s[kPairT1 + (((w & 63u) << 5) | ln)] ^ s[kPairT2 + ((((w >> 11) & 63u) << 5) | ln)] ^
           s[kPairT3 + ((((w >> 22) & 31u) << 5) | ln)];
}

__device__ __forceinline__ void crc_block4_cf(const uint32_t* s, Acc4& a, const uint4 v, uint32_t ln) {
    a.a0 = t11_cf(s, a.a0 ^ v.x, ln);
    a.a1 = t11_cf(s, a.a1 ^ v.y, ln);
    a.a2 = t11_cf(s, a.a2 ^ v.z, ln);
    a.a3 = t11_cf(s, a.a3 ^ v.w, ln);
}

// Shard-index CRC check by one workgroup with the pair tables (verify_index's
// chain, four accumulators, folded, shifted by kthread11).
// (`active` false: a second half-workgroup that only joins the barriers)
__device__ __forceinline__ void verify_index_pair(const DecodeParams& p, uint32_t j, int t, uint32_t kth11,
                                                  const uint32_t* s_tab, uint32_t* red, bool has_pre, uint4 pre,
                                                  bool active = true) {
    const zhip_chunk ch = p.idx_chunks[j];
    const uint32_t ok = active && ch.src_len == (uint64_t)p.idx_nbytes + 4u;
    const uint8_t* cp = p.src + ch.src;
    const uint32_t nk = (p.idx_E + kWgStride - 1) / kWgStride;
    const int32_t lo = (int32_t)p.idx_E - (int32_t)(nk * kWgStride);
    Acc4 a = {0u, 0u, 0u, 0u};
    if (ok) {
        for (uint32_t k = 0; k < nk; ++k) {
            const int32_t o = lo + kWgStride * (int32_t)k + 16 * t;
            uint4 v;
            if (k == 0 && has_pre) v = (o >= 0 && (uint32_t)o < p.idx_nbytes) ? mask_tail(pre, o, p.idx_nbytes)
                                                                         : make_uint4(0, 0, 0, 0);
            else v = load_block<false>(cp, o, p.idx_nbytes);
            crc_block4(s_tab, a, v);
        }
    }
    uint32_t v = wave_xor(gf_mul(fold4(s_tab, a), kth11));
    __syncthreads();  // red may still be read from a previous index
    if (active && (t & 63) == 0) red[t >> 6] = v;
    __syncthreads();
    if (active && t == 0) {
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

// The K = 8 steps of one unit in the row map (zhip_rows_map): 64 bytes, one
// scalar load per unit.
struct RowSteps {
    zhip_rowblk e[kDefaultBlocks];
};

__device__ __forceinline__ RowSteps load_row_steps(const DecodeParams& p, const Unit& U) {
    return load_uniform<RowSteps>(p.rowmap + ((size_t)U.sel * p.nseg + U.sidx) * kDefaultBlocks);
}

// Stores of one unit; with `crc` the Horner step of each block follows its
// store (the lookups spread over the data's arrival instead of trailing it).
// Destinations come from the row map: no per-step address arithmetic.
template <int ITEM, bool SWAP, int K, bool SKIP = false>
__device__ __forceinline__ void store_unit_rows(const DecodeParams& p, const Unit& U, const RowSteps& m, bool live,
                                                uint32_t lane_row, int64_t lane_off, uint8_t* sink,
                                                const uint4 (&blk)[K], bool crc = false,
                                                const uint32_t* s_tab = nullptr, Acc4* acc = nullptr) {
    static_assert(K == kDefaultBlocks, "the row map holds kDefaultBlocks steps per unit");
    const bool present = live && U.mode == ZHIP_ST_OK;
    const bool writes = live && (U.mode == ZHIP_ST_OK || U.mode == ZHIP_ST_MISSING);
    uint8_t* const base = p.out + U.out_off;
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t lo = m.e[k].lo, hi = m.e[k].hi;
        const bool wr = writes && lane_row - lo < hi - lo;  // unsigned: lo <= lane_row < hi
        store_nt16(wr ? base + m.e[k].rel + lane_off : sink, present ? swap_block<ITEM, SWAP>(blk[k]) : f);
        // (SKIP: ablation arm, lookups replaced by a plain xor; a compile-time
        // choice -- a runtime test here doubles the loop's branches)
        if (crc) {
            if constexpr (SKIP) acc->a0 ^= blk[k].x ^ blk[k].y ^ blk[k].z ^ blk[k].w;
            else crc_block4(s_tab, *acc, blk[k]);
        }
    }
}

// Publication of a run's reduced contribution V by wave 0 (wave-uniform, lane 0
// touches memory): one 64-bit atomic (contribution | arrival bits) when a chunk
// has <= 32 units, else xor + arrival count; the arrival that completes the
// chunk compares with the trailer.
__device__ __forceinline__ void publish_run(const DecodeParams& p, const Unit& U, uint32_t V, uint32_t run_bits,
                                            uint32_t stored, int t) {
    if (p.tune & kTuneNoTicket) {  // ablation: no publication / last-arriver
        if (t == 0 && V == 0x9E3779B9u) p.status[U.c].aux = V;
    } else if (p.nseg <= 32) {
        const uint64_t full = p.nseg >= 32 ? 0xFFFFFFFFull : ((1ull << p.nseg) - 1ull);
        uint64_t prev = 0;
        if (t == 0) {
            uint64_t* w = reinterpret_cast<uint64_t*>(p.ws) + 2ull * U.c;
            prev = __hip_atomic_fetch_xor(w, ((uint64_t)run_bits << 32) | V, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
        }
        PendingU q;
        q.prev = prev;
        q.stored = stored;
        q.c = U.c;
        q.bits = run_bits;
        q.V = V;
        q.valid = 1;
        retire_uniform(p, q, full, t, true);
    } else {  // > 32 units per chunk: xor, then count arrivals
        uint32_t raw = 0, last = 0;
        const uint32_t n_run = __builtin_popcount(run_bits);
        if (t == 0) {
            uint32_t* accw = p.ws + 4ull * U.c;
            const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
            const uint32_t tk = __hip_atomic_fetch_add(accw + 2, n_run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tk + n_run == p.nseg) {
                raw = __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // consume the returned value here (rare path): a register with a
                // load still pending would make every later write to it wait
                // for the wave's stores too
                asm volatile("s_waitcnt vmcnt(0)" ::"v"(raw) : "memory");
                __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = 1;
            }
        }
        if (__builtin_amdgcn_readfirstlane(last))
            finalize_uniform(p, U.c, stored, __builtin_amdgcn_readfirstlane(raw), t, true);
    }
}

// End of a run (consecutive units of one chunk in this workgroup): reduce the
// lanes' Horner states, shift to the chunk reference, publish with one 64-bit
// atomic (CRC contribution | arrival bits); the arrival that completes the
// chunk finalizes it.  `red` is a 4-word LDS scratch not used concurrently.
// End of a run (consecutive units of one chunk in this workgroup): shift every
// lane's Horner state by its kpair constant (lane shift x unit shift x c_inv,
// so no uniform multiply remains), xor-reduce over the workgroup, publish with
// one 64-bit atomic (contribution | arrival bits); the arrival that completes
// the chunk compares with the trailer.  `red` is a 4-word LDS scratch.
__device__ __forceinline__ void run_end_pair(const DecodeParams& p, const Unit& U, uint32_t acc, uint32_t run_bits,
                                             uint32_t stored, uint32_t klane, bool lds_mul, const uint32_t* s_mul,
                                             uint32_t* red, int t, uint32_t g = 0) {
    if (p.tune & kTuneNoRunEnd) {  // ablation: no reduction, no publication
        if (acc == 0x9E3779B9u) red[0] = acc;
        return;
    }
    // acc: the lane's folded state (fold4); klane / the s_mul column: kpair11
    uint32_t v = (p.tune & kTuneNoLaneMul) ? acc : lds_mul ? lanemul3(s_mul, t, acc) : gf_mul(acc, klane);
    v = wave_xor(v);
    if ((t & 63) == 0) red[t >> 6] = v;
    __syncthreads();
    stamp(p, g, t, 5);
    if (t < 64) {  // wave 0, wave-uniform
        const uint32_t V = __builtin_amdgcn_readfirstlane(red[0] ^ red[1] ^ red[2] ^ red[3]);
        stamp(p, g, t, 6);
        publish_run(p, U, V, run_bits, stored, t);
    }
}

__device__ __forceinline__ void unit_status_pair(const DecodeParams& p, const Unit& U, bool crc, int t) {
    // statuses not produced by the CRC finalize: non-CRC chains (OK), missing / failed units
    if (U.sidx != 0 || t != 0) return;
    if (U.mode == ZHIP_ST_OK) {
        if (!crc) {
            zhip_status st = {ZHIP_ST_OK, 0u, 0u, 0u};
            p.status[U.c] = st;
        }
    } else {
        zhip_status st = {U.mode, 0u, 0u, 0u};
        p.status[U.c] = st;
        if (U.mode != ZHIP_ST_MISSING) atomicOr(p.errflag, 1u << U.mode);
    }
}

// Unit B's loads issued one per stored block of unit A (VARIANT 7 / 8): at
// most K + 1 loads in flight per thread instead of 2K, so a wave's stores
// are not queued behind its own second unit's loads.
template <int ITEM, bool SWAP, int K>
__device__ __forceinline__ void store_a_load_b(const DecodeParams& p, const Unit& UA, const RowSteps& m,
                                               uint32_t lane_row, int64_t lane_off, uint8_t* sink,
                                               const uint4 (&blk)[K], bool crc, const uint32_t* s_tab, Acc4* acc,
                                               const Unit& UB, bool live_b, int t, uint4 (&nb)[K]) {
    const bool present = UA.mode == ZHIP_ST_OK;
    const bool writes = UA.mode == ZHIP_ST_OK || UA.mode == ZHIP_ST_MISSING;
    uint8_t* const base = p.out + UA.out_off;
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
    const bool okb = live_b && UB.mode == ZHIP_ST_OK;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_rows_zero);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t lo = m.e[k].lo, hi = m.e[k].hi;
        const bool wr = writes && lane_row - lo < hi - lo;
        store_nt16(wr ? base + m.e[k].rel + lane_off : sink, present ? swap_block<ITEM, SWAP>(blk[k]) : f);
        if (crc) crc_block4(s_tab, *acc, blk[k]);
        const int32_t bb = UB.seg_lo + kWgStride * k;
        nb[k] = load_stream16_any(okb && bb >= 0 ? UB.cp + bb + 16 * t : zero);
    }
}

// Shard-index check by a leading workgroup of a decode whose inner chunks carry
// no CRC (zarr's default sharding codecs: inner bytes only, index
// bytes + crc32c, sharding.py:423-427): the pair tables go into LDS for this
// workgroup alone, then verify_index_pair's chain.
__device__ __forceinline__ void index_lead(const DecodeParams& p, uint32_t j, int t, uint32_t* s_tab,
                                           uint32_t* red) {
    const uint4* gt = reinterpret_cast<const uint4*>(p.pair_tab);
    uint4 v[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) v[i] = gt[t + i * kThreads];
    const uint32_t kth = load_u32_any(reinterpret_cast<const uint8_t*>(p.kthread11 + t));
    uint4* st = reinterpret_cast<uint4*>(s_tab);
#pragma unroll
    for (int i = 0; i < 6; ++i) st[t + i * kThreads] = v[i];
    __syncthreads();
    verify_index_pair(p, j, t, kth, s_tab, red, false, make_uint4(0, 0, 0, 0));
}

// VARIANT (tuning arm, headline item type only): 0 production, 3 no CRC
// lookups (a plain xor; results invalid), 6 s_setprio(1) once every load of
// the wave is issued, 7 unit B's loads interleaved with unit A's stores, 8
// both.  (Round-1 arms 1 -- every store before the lookups -- and 2 --
// independent chains for the two units -- measured slower and were retired
// with the single-operator tables.)
template <bool CRC, int ITEM, bool SWAP, int NU, int K = 8, int VARIANT = 0>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(NU == 1 ? 8 : 4))) void k_decode_pair(const DecodeParams p) {
    // NU == 1: the lane shift is a VALU multiply (no s_mul), so that eight
    // workgroups fit a CU's LDS
    constexpr bool kLdsMul = CRC && NU == 2;
    constexpr bool SKIP = VARIANT == 3;
    constexpr bool PRIO = VARIANT == 6 || VARIANT == 8;
    constexpr bool DEFER_B = NU == 2 && (VARIANT == 7 || VARIANT == 8);
    __shared__ uint32_t s_tab[CRC ? kPairTabWords : 1];
    __shared__ uint32_t s_mul[kLdsMul ? 12 * kThreads : 1];
    __shared__ uint32_t s_red[2][kThreads / 64];
    const int t = threadIdx.x;
    const uint32_t G = gridDim.x;
    // XCD-contiguous runs (launch_decode sets xcd_run = G / 8 when the whole
    // grid is resident at once): the workgroups the dispatcher sends to one
    // XCD (blockIdx % 8) take one contiguous eighth of the batch instead of
    // every eighth pair; measured 1-2 us faster on the headline, slower on
    // multi-wave grids such as C4 (profiles/r02/kernel_arms_ab.jsonl)
    uint32_t g = blockIdx.x;
    if (p.xcd_run) {
        const uint32_t x = blockIdx.x & 7u, slot = blockIdx.x >> 3;
        g = ((slot / p.xcd_run) * 8u + x) * p.xcd_run + slot % p.xcd_run;
    }
    const uint32_t q0 = (uint32_t)NU * g;
    const bool has_a = q0 < p.n_units, has_b = NU == 2 && q0 + 1u < p.n_units;
    if (!has_a && g >= p.n_idx) return;
    const uint32_t expected = p.g.nbytes + (CRC ? 4u : 0u);
    auto unit_of = [&](uint32_t q) {
        const uint32_t c = q / p.nseg;
        return c * p.nseg + (p.nseg - 1u - (q - c * p.nseg));
    };
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_rows_zero);
    stamp(p, g, t, 0);
    // 1. vector loads, in this order and count on every path: [CRC: the pair
    //    tables (6), lane constants (3)], [CRC: the first shard-index block],
    //    unit A (K), unit B (K); unit headers and CRC trailers are scalar
    //    loads.  Waiting for any of them leaves the later ones in flight.
    const uint32_t u_a = has_a ? unit_of(q0) : 0u, u_b = has_b ? unit_of(q0 + 1u) : u_a;
    uint4 tv0, tv1, tv2, tv3, tv4, tv5;  // scalars, not an array: an array here lands in scratch
    uint32_t kth = 0, ka = 0, kb = 0;
    if constexpr (CRC) {
        // (ablation kTuneNoTables: read zero bytes instead; results invalid)
        const bool nt = (p.tune & kTuneNoTables) != 0;
        const uint4* gt = reinterpret_cast<const uint4*>(nt ? reinterpret_cast<const uint8_t*>(g_rows_zero)
                                                            : reinterpret_cast<const uint8_t*>(p.pair_tab));
        tv0 = gt[nt ? 0 : t];
        tv1 = gt[nt ? 0 : t + kThreads];
        tv2 = gt[nt ? 0 : t + 2 * kThreads];
        tv3 = gt[nt ? 0 : t + 3 * kThreads];
        tv4 = gt[nt ? 0 : t + 4 * kThreads];
        tv5 = gt[nt ? 0 : t + 5 * kThreads];
        if (!(p.tune & kTuneNoConsts)) {
            kth = load_u32_any(reinterpret_cast<const uint8_t*>(p.kthread11 + t));
            ka = load_u32_any(reinterpret_cast<const uint8_t*>(p.kpair11 + (size_t)(u_a % p.nseg) * kThreads + t));
            kb = load_u32_any(reinterpret_cast<const uint8_t*>(p.kpair11 + (size_t)(u_b % p.nseg) * kThreads + t));
        }
    }
    uint4 A[K], B[NU == 2 ? K : 1];
    Unit ua, ub;
    uint4 ipre = make_uint4(0, 0, 0, 0);
    if (p.pred) {
        // predicted addresses: the unit loads go out before the headers arrive
        Unit ga = predict_unit(p, u_a), gb = predict_unit(p, u_b);
        load_unit_rows(ga, has_a, t, A);
        if constexpr (NU == 2 && !DEFER_B) load_unit_rows(gb, has_b, t, B);
        ua = resolve_unit(p, u_a, expected);
        ub = ua;
        if constexpr (NU == 2)
            if (has_b) ub = advance_unit(p, ua, u_b, expected);
        // a wrong prediction (non-default packing, elided inner chunks) reloads
        // from the live index; the full drain keeps every later wait exact
        const bool bad_a = has_a && ua.mode == ZHIP_ST_OK && ua.cp != ga.cp;
        const bool bad_b = !DEFER_B && has_b && ub.mode == ZHIP_ST_OK && ub.cp != gb.cp;
        if (bad_a || bad_b) {
            if (bad_a) load_unit_rows(ua, true, t, A);
            if constexpr (NU == 2)
                if (bad_b) load_unit_rows(ub, true, t, B);
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        }
        if constexpr (CRC) ipre = index_prefetch(p, g, g < p.n_idx, t, zero);
    } else {
        ua = resolve_unit(p, u_a, expected);
        ub = ua;
        if constexpr (NU == 2)
            if (has_b) ub = advance_unit(p, ua, u_b, expected);
        if constexpr (CRC) ipre = index_prefetch(p, g, g < p.n_idx, t, zero);
        load_unit_rows(ua, has_a, t, A);
        if constexpr (NU == 2 && !DEFER_B) load_unit_rows(ub, has_b, t, B);
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);  // every load of this wave is out
    // destinations of both units' steps (scalar loads, consumed at the stores)
    const RowSteps ma = load_row_steps(p, ua), mb = load_row_steps(p, ub);
    uint32_t stored_a = 0, stored_b = 0;
    if constexpr (CRC) {
        const bool ta = has_a && ua.mode == ZHIP_ST_OK;
        const bool tb = has_b && ub.c != ua.c && ub.mode == ZHIP_ST_OK;
        // scalar loads (lgkmcnt): consuming them at the run end never waits
        // for this wave's stores, which a vector load issued before them would
        if (!(p.tune & kTuneNoConsts)) {
            if (ta) stored_a = load_trailer_uniform(ua.cp, p.g.nbytes);
            if (tb) stored_b = load_trailer_uniform(ub.cp, p.g.nbytes);
        }
    }
    stamp(p, g, t, 1);
    // 2. tables into LDS (waits for the table loads only), lane-multiply column
    if constexpr (CRC) {
        uint4* st = reinterpret_cast<uint4*>(s_tab);
        st[t] = tv0;
        st[t + kThreads] = tv1;
        st[t + 2 * kThreads] = tv2;
        st[t + 3 * kThreads] = tv3;
        st[t + 4 * kThreads] = tv4;
        st[t + 5 * kThreads] = tv5;
        if constexpr (kLdsMul) lanemul3_init(s_mul, t, kb);  // own column
        if (!(p.tune & kTuneNoBarrier)) __syncthreads();
    }
    stamp(p, g, t, 2);
    if (has_a) {
        if (p.tune & kTuneSerialize) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // ablation
        // 3. stores: A as soon as it arrives (B still in flight), then B; the
        //    Horner step of each block right after its store
        uint8_t* sink = reinterpret_cast<uint8_t*>(g_rows_sink);
        const uint32_t lane_row = (16u * (uint32_t)t) >> p.row_shift;
        const uint32_t lane_col = (16u * (uint32_t)t) & ((1u << p.row_shift) - 1u);
        const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
        const bool same = has_b && ub.c == ua.c;
        Acc4 acc_a = {0u, 0u, 0u, 0u}, acc_b = {0u, 0u, 0u, 0u};
        if constexpr (DEFER_B)
            store_a_load_b<ITEM, SWAP, K>(p, ua, ma, lane_row, lane_off, sink, A, CRC && ua.mode == ZHIP_ST_OK,
                                          s_tab, &acc_a, ub, has_b, t, B);
        else
            store_unit_rows<ITEM, SWAP, K, SKIP>(p, ua, ma, true, lane_row, lane_off, sink, A,
                                                 CRC && ua.mode == ZHIP_ST_OK, s_tab, &acc_a);
        stamp(p, g, t, 3);
        if constexpr (NU == 2) {
            if (same) acc_b = acc_a;
            store_unit_rows<ITEM, SWAP, K, SKIP>(p, ub, mb, has_b, lane_row, lane_off, sink, B,
                                                 CRC && has_b && ub.mode == ZHIP_ST_OK, s_tab, &acc_b);
        }
        stamp(p, g, t, 4);
        // 4. run ends (the CRC lookups ran with the stores): A alone when B
        //    starts another chunk, then B (or A+B).  Two straight-line call
        //    sites (a loop here merges the wait state of its back edge, and the
        //    compiler then drains the wave's stores before the reduction)
        if constexpr (CRC) {
            const uint32_t sa = __builtin_amdgcn_readfirstlane(stored_a);
            const uint32_t sb = same ? sa : __builtin_amdgcn_readfirstlane(stored_b);
            if (ua.mode == ZHIP_ST_OK && !same)
                run_end_pair(p, ua, SKIP ? acc_a.a0 : fold4(s_tab, acc_a), 1u << (ua.sidx & 31u), sa, ka, false,
                             s_mul, s_red[0], t, g);
            if (NU == 2 && has_b && ub.mode == ZHIP_ST_OK)
                run_end_pair(p, ub, SKIP ? acc_b.a0 : fold4(s_tab, acc_b),
                             (same ? 1u << (ua.sidx & 31u) : 0u) | (1u << (ub.sidx & 31u)), sb, kb, kLdsMul, s_mul,
                             s_red[1], t, g);
        }
        unit_status_pair(p, ua, CRC, t);
        if (has_b) unit_status_pair(p, ub, CRC, t);
    }
    // 5. fused shard-index checks (the lowest workgroups: dispatched first); the
    //    first block of this workgroup's index was prefetched with the units
    if constexpr (CRC)
        for (uint32_t j = g; j < p.n_idx; j += G) verify_index_pair(p, j, t, kth, s_tab, s_red[1], j == g, ipre);
    stamp(p, g, t, 7);
}

// ---------------------------------------------------------------------------
// k_decode_lead: k_decode_pair for chains whose inner chunks carry no CRC but
// whose shard indexes do (zarr's default sharding codecs: inner bytes only,
// index bytes + crc32c, sharding.py:423-427).  The first round_up(n_idx, 8)
// workgroups each verify one shard index (index_lead: pair tables in LDS) and
// return; the rest decode two units each with no tables at all -- one launch
// instead of an index launch ahead of the data.  With nothing to compute but
// addresses, the prologue is lean: the PairHot batch (one scalar round trip),
// magic divisions, and the unit loads at the addresses the default shard
// packing predicts (zhip_predict) before the header chain resolves; a wrong
// guess reloads.  (The same prologue measured slower in the CRC kernels, whose
// 24 KiB table loads then queue behind every workgroup's data loads:
// profiles/r03/lean/.)
template <int ITEM, bool SWAP, int K = kDefaultBlocks>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_decode_lead(const DecodeParams p) {
    __shared__ uint32_t s_tab[kPairTabWords];
    __shared__ uint32_t s_red[kThreads / 64];
    const int t = threadIdx.x;
    PairHot h = p.h;
    pair_hot(h);
    uint32_t bx = blockIdx.x;
    // a multiple of 8 leading workgroups keeps bx % 8 the dispatch XCD
    const uint32_t lead = (h.n_idx + 7u) & ~7u;
    if (bx < lead) {
        if (bx < h.n_idx) index_lead(p, bx, t, s_tab, s_red);
        return;
    }
    bx -= lead;
    uint32_t g = bx;
    {
        const uint32_t x = bx & 7u, slot = bx >> 3;
        const uint32_t r = fdiv_apply(slot, h.d_xcd.m, h.d_xcd.s);
        const uint32_t gx = (r * 8u + x) * h.xcd_run + (slot - r * h.xcd_run);
        g = h.xcd_run ? gx : bx;
    }
    const uint32_t q0 = 2u * g;
    const bool has_a = q0 < h.n_units, has_b = q0 + 1u < h.n_units;
    if (!has_a) return;
    auto unit_of = [&](uint32_t q) {
        const uint32_t c = fdiv_apply(q, h.d_nseg.m, h.d_nseg.s);
        return c * h.nseg + (h.nseg - 1u - (q - c * h.nseg));
    };
    const uint32_t u_a = unit_of(q0), u_b = has_b ? unit_of(q0 + 1u) : u_a;
    const uint32_t expected = p.g.nbytes;
    uint4 A[K], B[K];
    Unit ua, ub;
    if (h.pred) {
        const Unit ga = predict_unit_h(h, u_a), gb = predict_unit_h(h, u_b);
        load_unit_rows(ga, true, t, A);
        load_unit_rows(gb, has_b, t, B);
        ua = resolve_unit(p, u_a, expected);
        ub = has_b ? advance_unit(p, ua, u_b, expected) : ua;
        const bool bad_a = ua.mode == ZHIP_ST_OK && ua.cp != ga.cp;
        const bool bad_b = has_b && ub.mode == ZHIP_ST_OK && ub.cp != gb.cp;
        if (bad_a || bad_b) {  // a wrong guess reloads from the live index; the full drain keeps later waits exact
            if (bad_a) load_unit_rows(ua, true, t, A);
            if (bad_b) load_unit_rows(ub, true, t, B);
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        }
    } else {
        ua = resolve_unit(p, u_a, expected);
        ub = has_b ? advance_unit(p, ua, u_b, expected) : ua;
        load_unit_rows(ua, true, t, A);
        load_unit_rows(ub, has_b, t, B);
    }
    const RowSteps ma = load_row_steps(p, ua), mb = load_row_steps(p, ub);
    uint8_t* sink = reinterpret_cast<uint8_t*>(g_rows_sink);
    const uint32_t lane_row = (16u * (uint32_t)t) >> p.row_shift;
    const uint32_t lane_col = (16u * (uint32_t)t) & ((1u << p.row_shift) - 1u);
    const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
    store_unit_rows<ITEM, SWAP, K>(p, ua, ma, true, lane_row, lane_off, sink, A);
    store_unit_rows<ITEM, SWAP, K>(p, ub, mb, has_b, lane_row, lane_off, sink, B);
    unit_status_pair(p, ua, false, t);
    if (has_b) unit_status_pair(p, ub, false, t);
}

// k_decode_lead4: k_decode_lead for chunks of at most 16 KiB (one unit per
// chunk; the reference's example array has 64 x 64 float32 inner chunks).  Such
// a unit's first four 4 KiB steps lie before the chunk start (seg_lo =
// E - 32 KiB <= -16 KiB), so the pair kernel spends half its loads on the zero
// line and half its stores on the sink.  Here a workgroup decodes four chunks
// with only the last four steps of each: 16 loads and 16 stores per lane, all
// live except the whole empty head steps of a chunk under 16 KiB.  The row map
// is zhip_rows_map's, unchanged (entries 4..7 of each unit); no XCD remap (four
// consecutive chunks per workgroup already keep a shard's chunks together).
// CRC: inner chunks with a crc32c trailer.  A workgroup owns its four chunks
// whole, so each one's Horner state (four accumulators through the 11/11/10
// tables, as k_decode_pair) folds, takes unit 0's lane constant, reduces in
// LDS and is compared with the trailer by lane i of wave 0: no publication.
// NQ = 8 (launched as "k_decode_lead8"): chunks of <= 8 KiB, eight per
// workgroup over their last two steps.
template <int KS>
struct RowTail {
    zhip_rowblk e[KS];
};

template <int ITEM, bool SWAP, bool CRC = false, int NQ = 4>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_decode_lead4(const DecodeParams p) {
    static_assert(NQ == 4 || NQ == 8, "four or eight chunks per workgroup");
    constexpr int KS = 16 / NQ, K0 = kDefaultBlocks - KS;  // 16 blocks per lane either way
    __shared__ uint32_t s_tab[kPairTabWords];
    __shared__ uint32_t s_red[kThreads / 64];
    __shared__ uint32_t s_crc[CRC ? NQ : 1][kThreads / 64];
    const int t = threadIdx.x;
    PairHot h = p.h;
    pair_hot(h);
    uint32_t bx = blockIdx.x;
    const uint32_t lead = (h.n_idx + 7u) & ~7u;
    if (bx < lead) {
        if (bx < h.n_idx) index_lead(p, bx, t, s_tab, s_red);
        return;
    }
    const uint32_t q0 = (uint32_t)NQ * (bx - lead);  // nseg == 1: unit = chunk
    if (q0 >= h.n_units) return;
    const uint32_t expected = p.g.nbytes + (CRC ? 4u : 0u);
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_rows_zero);
    // CRC: the pair tables and unit 0's lane constants first (L2 hits, back
    // before the chunk data)
    uint4 tv0, tv1, tv2, tv3, tv4, tv5;
    uint32_t kl = 0;
    if constexpr (CRC) {
        const uint4* gt = reinterpret_cast<const uint4*>(p.pair_tab);
        tv0 = gt[t];
        tv1 = gt[t + kThreads];
        tv2 = gt[t + 2 * kThreads];
        tv3 = gt[t + 3 * kThreads];
        tv4 = gt[t + 4 * kThreads];
        tv5 = gt[t + 5 * kThreads];
        kl = load_u32_any(reinterpret_cast<const uint8_t*>(p.kpair11 + t));
    }
    auto load_tail = [&](const Unit& u, bool live, uint4 (&b)[KS]) {
        const bool ok = live && u.mode == ZHIP_ST_OK;
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            const int32_t base = u.seg_lo + kWgStride * (K0 + k);
            b[k] = load_stream16_any(ok && base >= 0 ? u.cp + base + 16 * t : zero);
        }
    };
    bool live[NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i) live[i] = q0 + (uint32_t)i < h.n_units;
    Unit U[NQ];
    uint4 blk[NQ][KS];
    if (h.pred) {
        Unit gs[NQ];
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
            gs[i] = predict_unit_h(h, live[i] ? q0 + i : q0);
            load_tail(gs[i], live[i], blk[i]);
        }
        bool bad = false;
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
            U[i] = live[i] ? resolve_unit(p, q0 + i, expected) : U[0];
            const bool b = live[i] && U[i].mode == ZHIP_ST_OK && U[i].cp != gs[i].cp;
            if (b) load_tail(U[i], true, blk[i]);
            bad = bad || b;
        }
        if (bad) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): later waits stay exact
    } else {
#pragma unroll
        for (int i = 0; i < NQ; ++i) U[i] = live[i] ? resolve_unit(p, q0 + i, expected) : U[0];
#pragma unroll
        for (int i = 0; i < NQ; ++i) load_tail(U[i], live[i], blk[i]);
    }
    RowTail<KS> m[NQ];  // the live row-map entries K0..7 of each unit
#pragma unroll
    for (int i = 0; i < NQ; ++i)
        m[i] = load_uniform<RowTail<KS>>(p.rowmap + ((size_t)U[i].sel * p.nseg + U[i].sidx) * kDefaultBlocks + K0);
    uint32_t stored[NQ];
    if constexpr (CRC) {
#pragma unroll
        for (int i = 0; i < NQ; ++i)
            stored[i] = (live[i] && U[i].mode == ZHIP_ST_OK) ? load_trailer_uniform(U[i].cp, p.g.nbytes) : 0u;
        uint4* st = reinterpret_cast<uint4*>(s_tab);
        st[t] = tv0;
        st[t + kThreads] = tv1;
        st[t + 2 * kThreads] = tv2;
        st[t + 3 * kThreads] = tv3;
        st[t + 4 * kThreads] = tv4;
        st[t + 5 * kThreads] = tv5;
        __syncthreads();
    }
    uint8_t* sink = reinterpret_cast<uint8_t*>(g_rows_sink);
    const uint32_t lane_row = (16u * (uint32_t)t) >> p.row_shift;
    const uint32_t lane_col = (16u * (uint32_t)t) & ((1u << p.row_shift) - 1u);
    const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        const bool present = live[i] && U[i].mode == ZHIP_ST_OK;
        const bool writes = live[i] && (U[i].mode == ZHIP_ST_OK || U[i].mode == ZHIP_ST_MISSING);
        uint8_t* const base = p.out + U[i].out_off;
        Acc4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            const zhip_rowblk& e = m[i].e[k];
            const uint32_t lo = e.lo, hi = e.hi;
            const bool wr = writes && lane_row - lo < hi - lo;  // unsigned: lo <= lane_row < hi
            store_nt16(wr ? base + e.rel + lane_off : sink, present ? swap_block<ITEM, SWAP>(blk[i][k]) : f);
            // (zero head blocks of a chunk under 16 KiB leave the state at 0)
            if constexpr (CRC) crc_block4(s_tab, acc, blk[i][k]);
        }
        if constexpr (CRC) {
            const uint32_t v = wave_xor(present ? lanemul_reg(kl, fold4(s_tab, acc)) : 0u);
            if ((t & 63) == 0) s_crc[i][t >> 6] = v;
        }
    }
    if constexpr (CRC) {
        __syncthreads();
        if (t < 64) {  // wave 0: one verdict per chunk against its trailer
#pragma unroll
            for (int i = 0; i < NQ; ++i)
                if (live[i] && U[i].mode == ZHIP_ST_OK)
                    finalize_uniform(p, U[i].c, __builtin_amdgcn_readfirstlane(stored[i]),
                                     __builtin_amdgcn_readfirstlane(s_crc[i][0] ^ s_crc[i][1] ^ s_crc[i][2] ^
                                                                    s_crc[i][3]),
                                     t, true);
        }
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i)
        if (live[i]) unit_status_pair(p, U[i], CRC, t);
}int debug_stamps(uint64_t* host_out, uint32_t n_wg) {
    if (n_wg > kStampWG) n_wg = kStampWG;
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamps), (size_t)n_wg * kStampSlots * sizeof(uint64_t), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

using KernelFn = void (*)(const DecodeParams);

template <int NU>
KernelFn select_pair_nu(bool crc, int item, bool swap) {
    switch (item) {
        case 1: return crc ? k_decode_pair<true, 1, false, NU> : k_decode_pair<false, 1, false, NU>;
        case 2: return crc ? (swap ? k_decode_pair<true, 2, true, NU> : k_decode_pair<true, 2, false, NU>)
                           : (swap ? k_decode_pair<false, 2, true, NU> : k_decode_pair<false, 2, false, NU>);
        case 4: return crc ? (swap ? k_decode_pair<true, 4, true, NU> : k_decode_pair<true, 4, false, NU>)
                           : (swap ? k_decode_pair<false, 4, true, NU> : k_decode_pair<false, 4, false, NU>);
        case 8: return crc ? (swap ? k_decode_pair<true, 8, true, NU> : k_decode_pair<true, 8, false, NU>)
                           : (swap ? k_decode_pair<false, 8, true, NU> : k_decode_pair<false, 8, false, NU>);
        default: return nullptr;
    }
}

KernelFn select_pair_kernel(bool crc, int item, bool swap, int nu) {
    if (nu == 9) {  // no data CRC, leading index-check workgroups (k_decode_lead)
        if (crc) return nullptr;
        switch (item) {
            case 1: return k_decode_lead<1, false>;
            case 2: return swap ? k_decode_lead<2, true> : k_decode_lead<2, false>;
            case 4: return swap ? k_decode_lead<4, true> : k_decode_lead<4, false>;
            case 8: return swap ? k_decode_lead<8, true> : k_decode_lead<8, false>;
            default: return nullptr;
        }
    }
    if (nu == 10 || nu == 11) {  // chunks of <= 16 / 8 KiB: four / eight per workgroup (k_decode_lead4)
        const bool e8 = nu == 11;
        switch (item) {
            case 1: return crc ? (e8 ? k_decode_lead4<1, false, true, 8> : k_decode_lead4<1, false, true>)
                               : (e8 ? k_decode_lead4<1, false, false, 8> : k_decode_lead4<1, false>);
            case 2: return crc ? (swap ? (e8 ? k_decode_lead4<2, true, true, 8> : k_decode_lead4<2, true, true>)
                                       : (e8 ? k_decode_lead4<2, false, true, 8> : k_decode_lead4<2, false, true>))
                               : (swap ? (e8 ? k_decode_lead4<2, true, false, 8> : k_decode_lead4<2, true>)
                                       : (e8 ? k_decode_lead4<2, false, false, 8> : k_decode_lead4<2, false>));
            case 4: return crc ? (swap ? (e8 ? k_decode_lead4<4, true, true, 8> : k_decode_lead4<4, true, true>)
                                       : (e8 ? k_decode_lead4<4, false, true, 8> : k_decode_lead4<4, false, true>))
                               : (swap ? (e8 ? k_decode_lead4<4, true, false, 8> : k_decode_lead4<4, true>)
                                       : (e8 ? k_decode_lead4<4, false, false, 8> : k_decode_lead4<4, false>));
            case 8: return crc ? (swap ? (e8 ? k_decode_lead4<8, true, true, 8> : k_decode_lead4<8, true, true>)
                                       : (e8 ? k_decode_lead4<8, false, true, 8> : k_decode_lead4<8, false, true>))
                               : (swap ? (e8 ? k_decode_lead4<8, true, false, 8> : k_decode_lead4<8, true>)
                                       : (e8 ? k_decode_lead4<8, false, false, 8> : k_decode_lead4<8, false>));
            default: return nullptr;
        }
    }
#if ZHIP_TUNING
    if (nu == 5)  // tuning arm (headline item type only): VARIANT 3, no lookups
        return !(crc && item == 4 && !swap) ? nullptr : k_decode_pair<true, 4, false, 2, 8, 3>;
    if (nu >= 6 && nu <= 8) {  // tuning arms (headline item type only): VARIANT 6 / 7 / 8
        if (!(crc && item == 4 && !swap)) return nullptr;
        return nu == 6 ? k_decode_pair<true, 4, false, 2, 8, 6>
               : nu == 7 ? k_decode_pair<true, 4, false, 2, 8, 7> : k_decode_pair<true, 4, false, 2, 8, 8>;
    }
    if (nu == 1) return select_pair_nu<1>(crc, item, swap);  // kTuneSingle
#endif
    if (nu != 2) return nullptr;
    return select_pair_nu<2>(crc, item, swap);
}

// ---------------------------------------------------------------------------
// k_decode_duo: k_decode_pair's decode with one unit per 256-thread half of a
// 512-thread workgroup, so the 24 KiB of CRC tables in LDS serve two units
// while every unit keeps its own waves: 8 waves per workgroup, 4 workgroups
// (32 waves) per CU, the whole headline batch resident at once.  Each half
// runs the NU == 1 arm of k_decode_pair (own Horner chain, VALU lane multiply
// by kpair11, own publication); barriers are workgroup-wide, so both halves
// pass every one of them whatever their unit's state.
template <bool CRC, int ITEM, bool SWAP, int K = 8>
__global__ __launch_bounds__(2 * kThreads) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_decode_duo(
    const DecodeParams p) {
    __shared__ uint32_t s_tab[CRC ? kPairTabWords : 1];
    __shared__ uint32_t s_red[3][kThreads / 64];
    const int t = threadIdx.x, h = t >> 8, tl = t & (kThreads - 1);
    const uint32_t G = gridDim.x, g = blockIdx.x;
    const uint32_t q = 2u * g + (uint32_t)h;
    if (2u * g >= p.n_units && g >= p.n_idx) return;  // workgroup-uniform
    const bool has = q < p.n_units;
    const uint32_t expected = p.g.nbytes + (CRC ? 4u : 0u);
    const uint32_t u = has ? (q / p.nseg) * p.nseg + (p.nseg - 1u - q % p.nseg) : 0u;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_rows_zero);
    // 1. vector loads in a path-independent order and count: [CRC: tables (3),
    //    lane constants (2), first shard-index block], the unit (K)
    uint4 tv0, tv1, tv2;
    uint32_t kth = 0, ku = 0;
    if constexpr (CRC) {
        const uint4* gt = reinterpret_cast<const uint4*>(p.pair_tab);
        tv0 = gt[t];
        tv1 = gt[t + 2 * kThreads];
        tv2 = gt[t + 4 * kThreads];
        kth = load_u32_any(reinterpret_cast<const uint8_t*>(p.kthread11 + tl));
        ku = load_u32_any(reinterpret_cast<const uint8_t*>(p.kpair11 + (size_t)(u % p.nseg) * kThreads + tl));
    }
    uint4 A[K];
    Unit ua;
    uint4 ipre = make_uint4(0, 0, 0, 0);
    if (p.pred) {
        const Unit ga = predict_unit(p, u);
        load_unit_rows(ga, has, tl, A);
        ua = resolve_unit(p, u, expected);
        if (has && ua.mode == ZHIP_ST_OK && ua.cp != ga.cp) {  // wrong guess: reload, full drain
            load_unit_rows(ua, true, tl, A);
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        }
        if constexpr (CRC) ipre = index_prefetch(p, g, g < p.n_idx && h == 0, tl, zero);
    } else {
        ua = resolve_unit(p, u, expected);
        if constexpr (CRC) ipre = index_prefetch(p, g, g < p.n_idx && h == 0, tl, zero);
        load_unit_rows(ua, has, tl, A);
    }
    const RowSteps ma = load_row_steps(p, ua);
    const bool crc_on = CRC && has && ua.mode == ZHIP_ST_OK;
    uint32_t stored = 0;
    if (crc_on) stored = load_trailer_uniform(ua.cp, p.g.nbytes);
    // 2. tables into LDS
    if constexpr (CRC) {
        uint4* st = reinterpret_cast<uint4*>(s_tab);
        st[t] = tv0;
        st[t + 2 * kThreads] = tv1;
        st[t + 4 * kThreads] = tv2;
        __syncthreads();
    }
    // 3. stores, each block's Horner step after its store
    uint8_t* sink = reinterpret_cast<uint8_t*>(g_rows_sink);
    const uint32_t lane_row = (16u * (uint32_t)tl) >> p.row_shift;
    const uint32_t lane_col = (16u * (uint32_t)tl) & ((1u << p.row_shift) - 1u);
    const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
    Acc4 acc = {0u, 0u, 0u, 0u};
    store_unit_rows<ITEM, SWAP, K>(p, ua, ma, has, lane_row, lane_off, sink, A, crc_on, s_tab, &acc);
    // 4. run end: every half reaches the barrier; only a valid one publishes
    if constexpr (CRC) {
        uint32_t v = crc_on ? gf_mul(fold4(s_tab, acc), ku) : 0u;
        v = wave_xor(v);
        if ((tl & 63) == 0) s_red[h][tl >> 6] = v;
        __syncthreads();
        if (crc_on && tl < 64) {
            const uint32_t V = __builtin_amdgcn_readfirstlane(s_red[h][0] ^ s_red[h][1] ^ s_red[h][2] ^ s_red[h][3]);
            publish_run(p, ua, V, 1u << (ua.sidx & 31u), __builtin_amdgcn_readfirstlane(stored), tl);
        }
    }
    if (has) unit_status_pair(p, ua, CRC, tl);
    // 5. fused shard-index checks by half 0 (half 1 joins the barriers)
    if constexpr (CRC)
        for (uint32_t j = g; j < p.n_idx; j += G)
            verify_index_pair(p, j, tl, kth, s_tab, s_red[2], j == g, ipre, h == 0);
}

// ---------------------------------------------------------------------------
// k_decode_il: the whole-row decode with interleaved steps, for batches far
// larger than one resident wave of workgroups (C4, C5).  A chunk's 4 KiB steps
// form groups of S x 8; workgroup r of the chunk (group r / S, offset
// j = r % S) takes steps j, j + S, ..., j + 7S of its group, so the S
// workgroups of a group -- consecutive in dispatch order -- sweep S x 32 KiB
// together, 4 KiB each at a time, instead of each streaming its own 64 KiB.
// At 4 GiB that access order copies at 0.75 of HBM peak where 32 KiB spans
// reach 0.61-0.67 (profiles/r03/copy_*.jsonl, graphbench arms).  Per lane the
// eight blocks are D = 4096 S bytes apart: one Horner chain through the
// A_D 11/11/10 tables (four word accumulators, A4 fold), one windowed lane
// multiply by the workgroup's host-built constant, one publication per
// workgroup (arrival bit r; > 32 workgroups per chunk: xor + count).  Same
// statuses, stores (row map, sink for unselected rows), fused index checks
// (one step per lane; the constants carry the A_D frame) as k_decode_pair.
// (CPU emulation: zhip_emulate_chunk_crc_il.)
//
// wstride: 64-bit words between chunks' publication words; default 2 (16 B
// per chunk, eight chunks per 128-byte line).  k_decode_il / k_decode_tile4
// pass kPubLine / 2 instead, one line per chunk (zhip_plan_info reports
// >= kPubLine workspace words per chunk for CRC layouts).
__device__ __forceinline__ void publish_il(const DecodeParams& p, uint32_t c, uint32_t r, uint32_t wpc, uint32_t V,
                                           uint32_t stored, int t, uint32_t wstride = 2u) {
    if (wpc <= 32u) {
        const uint64_t full = wpc >= 32u ? 0xFFFFFFFFull : ((1ull << wpc) - 1ull);
        const uint64_t bits = 1ull << r;
        uint64_t prev = 0;
        uint64_t* const w = reinterpret_cast<uint64_t*>(p.ws) + (uint64_t)wstride * c;
        if (t == 0) prev = __hip_atomic_fetch_xor(w, (bits << 32) | V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)prev);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(prev >> 32));
        if ((uint64_t)(hi ^ (uint32_t)bits) == full) {
            if (t == 0) __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            finalize_uniform(p, c, stored, lo ^ V, t, true);
        }
    } else {  // more than 32 workgroups per chunk: xor, then count arrivals
        uint32_t raw = 0, last = 0;
        if (t == 0) {
            uint32_t* accw = p.ws + 4ull * c;
            const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
            const uint32_t tk = __hip_atomic_fetch_add(accw + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tk + 1u == wpc) {
                raw = __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::"v"(raw) : "memory");
                __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = 1;
            }
        }
        if (__builtin_amdgcn_readfirstlane(last))
            finalize_uniform(p, c, stored, __builtin_amdgcn_readfirstlane(raw), t, true);
    }
}

// publish_il through two subwords of 16 arrivals on lines of their own and a
// second level on the chunk's line (tileg_arrive SPR; 17..32 workgroups per
// chunk; tuning arm 49): 16 returning atomics per line instead of 32 on one
// word, one more round trip for the two subwords' last arrivals.
__device__ __forceinline__ void publish_il_split(const DecodeParams& p, uint32_t c, uint32_t r, uint32_t wpc,
                                                 uint32_t V, uint32_t stored, int t) {
    uint32_t raw = 0, last = 0;
    if (t == 0) {
        bool any_ne;
        last = tileg_arrive<true>(p.ws, p.n_chunks, c, r, wpc, (wpc + 15u) / 16u, V, false, raw, any_ne) ? 1u : 0u;
    }
    if (__builtin_amdgcn_readfirstlane(last)) finalize_uniform(p, c, stored, __builtin_amdgcn_readfirstlane(raw), t, true);
}

// publish_lb: the look-back finalizer (round 6; PUB = 5, at most 64
// workgroups per chunk).  Workgroups r < wpc - 1 publish (bit r << 32) | V
// with a NON-returning agent-scope xor into word r / 32 of the chunk's line
// and retire at once; the chunk's highest-index workgroup r = wpc - 1 polls
// the words (one lane, relaxed agent loads, s_sleep between polls) until every
// other arrival bit is set, resets them and finalizes.  Forward progress: the
// only waiting workgroups are the finalizers, one per chunk, and they wait
// only on workgroups that never wait; the host takes this form only when
// n_chunks < CUs (launch_decode), so the finalizers can never hold every
// resident slot whatever the dispatch order.  (CPU-side protocol checks:
// tests/test_gpu_decode.py, a corrupted unit in every position.)
__device__ __forceinline__ void publish_lb(const DecodeParams& p, uint32_t c, uint32_t r, uint32_t wpc, uint32_t V,
                                           uint32_t stored, int t, uint32_t wstride) {
    uint64_t* const w = reinterpret_cast<uint64_t*>(p.ws) + (uint64_t)wstride * c;
    if (r + 1u < wpc) {
        if (t == 0)
            (void)__hip_atomic_fetch_xor(w + (r >> 5), ((1ull << (r & 31u)) << 32) | V, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    // arrival bits expected in word 0 / word 1 (the finalizer's own excluded)
    const uint32_t n0 = wpc < 32u ? wpc : 32u, n1 = wpc - n0;
    const uint32_t e0 = n1 ? 0xFFFFFFFFu : (uint32_t)((1ull << (n0 - 1u)) - 1ull);
    const uint32_t e1 = n1 ? (uint32_t)((1ull << (n1 - 1u)) - 1ull) : 0u;
    uint32_t lo = 0;
    if (t == 0) {
        uint64_t a = 0, b = 0;
        for (;;) {
            a = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)(a >> 32) == e0) break;
            __builtin_amdgcn_s_sleep(1);
        }
        if (n1) {
            for (;;) {
                b = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)(b >> 32) == e1) break;
                __builtin_amdgcn_s_sleep(1);
            }
            __hip_atomic_store(w + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lo = (uint32_t)a ^ (uint32_t)b;
    }
    finalize_uniform(p, c, stored, __builtin_amdgcn_readfirstlane(lo) ^ V, t, true);
}

// LEAN (tuning arm kTuneIlLean): the PairHot batch, then tables, constants
// and -- at the addresses the default shard packing predicts (zhip_predict) --
// the data loads, all before the header chain (chunk record -> index entry)
// resolves; a wrong prediction reloads.  Measured 1.5 us SLOWER on the
// headline than the production order (data loads after the resolved header:
// the tables, L2 hits, are in LDS before the data flood;
// profiles/r03/lean/).
// LM (arms kTuneIlRegMul / kTuneIlOcc6): 0 = lane multiply from the LDS
// column (production); 1 = in registers (lanemul_reg), 4 workgroups per CU;
// 2 = in registers with 24 KiB of LDS and 6 workgroups per CU.
// TUNE: the timing arms that read p.tune at run time (kTuneNoTables,
// kTuneNoRunEnd, kTuneNoPub) are compiled in; the production instantiation has
// TUNE = false and no such branch.
// PUB: how a workgroup's CRC contribution reaches the chunk's verdict.
//   3 (production, round 4): the returning 64-bit publication with arrival
//     bits (publish_il), the chunk's word alone in its 128-byte line
//     (p.ws + kPubLine c); the last arriver compares with the trailer.
//   0 (arm ZHIP_TUNE_ARM = 1): the same at p.ws + 4 c (round 3: eight
//     chunks' words share a line).
//   2 (arm ZHIP_TUNE_ARM = 2): deferred verdicts (zarrhip.h) -- a
//     NON-returning atomic xor into the chunk's word of this launch's bank
//     (the chunk's first workgroup also folds in c3 ^ ~stored and records the
//     trailer); the first workgroup of each chunk checks the other bank (the
//     previous launch's verdict) and clears it.
//   Graph-timed on one box (profiles/r04/c/arms_*.jsonl), headline / N = 8
//   share: 3: 26.01 / 9.45 us, 0: 26.22 / 9.62, 2: 26.38 / 10.14, no
//   publication at all 25.48 / 9.17.
// AFF (production for ZHIP_DF_WHOLE launches of plans with aff_ok): the K
//   destinations from the plan's two-level affine form of the whole-chunk row
//   map (aff_rowblk) in scalar registers instead of K scalar loads of the map:
//   graph-timed 26.06 vs 26.38 us on the headline, SALU instructions 3.61 M ->
//   2.80 M per launch (profiles/r05/w/).
// PRIO (tuning arms 51-53): wave issue priority (s_setprio 3) -- bit 0: from
//   the run end on (a finishing workgroup frees its CU slot sooner), bit 1:
//   until the data loads are issued (a starting workgroup's loads go out ahead
//   of its neighbours' Horner steps), bit 2: until the tables are in LDS
//   (production for the AFF launches: graph-timed 25.78-25.98 vs 25.97-26.09
//   us median in four interleaved pairs, profiles/r05/ag/; arm 56 keeps 0);
//   0 = the other instantiations.
// STW (tuning arms 64 / 65, outs below 2 GiB): the stores through a buffer
//   descriptor on the chunk's out base, unselected rows dropped by the range
//   check instead of written to the sink; 1 = write-through (sc1: no dirty
//   lines left in L2 at the kernel's end), 2 = nontemporal (the production
//   policy, isolating the store form)
template <bool CRC, int ITEM, bool SWAP, bool LEAN = false, bool CF = false, int LM = 0, bool TUNE = false,
          int PUB = 3, bool AFF = false, int PRIO = 0, int STW = 0>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(LM == 2 ? 6 : 4, LM == 2 ? 6 : 4)))
void k_decode_il(const DecodeParams p) {
    constexpr int K = kDefaultBlocks;
    if constexpr ((PRIO & 6) != 0) __builtin_amdgcn_s_setprio(3);
    __shared__ uint32_t s_tab[CRC ? kPairTabWords : 1];
    __shared__ uint32_t s_mul[CRC && LM == 0 ? 12 * kThreads : 1];
    __shared__ uint32_t s_red[2][kThreads / 64];
    const int t = threadIdx.x;
    const uint32_t G = gridDim.x;
    // (PRIO bit 3, tuning arm 57: XCD-contiguous eighths of the grid -- the
    // dispatcher's XCD blockIdx % 8 takes workgroups [x G/8, (x + 1) G/8);
    // -0.14 to -0.56 us on one box, +0.4 to +0.8 us on another in four
    // interleaved pairs, profiles/r05/ai/: not adopted)
    const uint32_t g = ((PRIO & 8) != 0 && (G & 7u) == 0u) ? (blockIdx.x & 7u) * (G >> 3) + (blockIdx.x >> 3)
                                                           : blockIdx.x;
    const uint32_t expected = p.g.nbytes + (CRC ? 4u : 0u);
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_rows_zero);
    uint32_t c, r, st0;
    bool has, ok;
    Unit U;
    int32_t lo_frame;
    uint4 ipre = make_uint4(0, 0, 0, 0);
    uint4 tv0, tv1, tv2, tv3, tv4, tv5;
    uint32_t kl = 0, kix = 0;
    uint64_t dvprev = 0;  // PUB == 2: {word, stored} of the other bank (first workgroup of a chunk)
    uint4 A[K];
    if constexpr (LEAN) {
        PairHot h = p.h;
        pair_hot(h);
        il_hot(h);
        const uint32_t wpc = h.nseg, S = h.il_S;  // S in {2, 4, 8}
        const uint32_t ls = (uint32_t)__builtin_ctz(S);
        c = fdiv_apply(g, h.d_nseg.m, h.d_nseg.s);
        r = g - c * wpc;
        has = c < h.n_chunks;
        if (!has && g >= h.n_idx) return;
        if constexpr (CRC) {
            const uint4* gt = reinterpret_cast<const uint4*>(h.il_tab);
            tv0 = gt[t];
            tv1 = gt[t + kThreads];
            tv2 = gt[t + 2 * kThreads];
            tv3 = gt[t + 3 * kThreads];
            tv4 = gt[t + 4 * kThreads];
            tv5 = gt[t + 5 * kThreads];
            kl = load_u32_any(reinterpret_cast<const uint8_t*>(reinterpret_cast<const uint32_t*>(h.il_klane) +
                                                               (size_t)(has ? r : 0u) * kThreads + t));
            kix = load_u32_any(reinterpret_cast<const uint8_t*>(reinterpret_cast<const uint32_t*>(h.il_kidx) + t));
        }
        st0 = ((r >> ls) << ls) * (uint32_t)K + (r & (S - 1u));
        lo_frame = (int32_t)h.E - (int32_t)(h.nseg * h.seg);
        if (h.pred) {
            const uint32_t grp = fdiv_apply(c, h.d_per.m, h.d_per.s);
            const uint8_t* cpp = reinterpret_cast<const uint8_t*>(h.src) + h.pred_base + (uint64_t)grp * h.pred_outer +
                                 (uint64_t)(c - grp * h.pred_per) * h.pred_inner;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int32_t base = lo_frame + kWgStride * (int32_t)(st0 + S * (uint32_t)k);
                A[k] = load_stream16_any(has && base >= 0 ? cpp + base + 16 * t : zero);
            }
            if (has) U = resolve_unit(p, c * h.nseg, expected);
            ok = has && U.mode == ZHIP_ST_OK;
            if (ok && U.cp != cpp) {  // a wrong guess: reload from the live index, full drain
                // (diagnostics: counted in the last stamp slot, zhip_debug_stamps)
                if (t == 0) atomicAdd(reinterpret_cast<unsigned long long*>(&g_stamps[kStampWG * kStampSlots - 1]), 1ull);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int32_t base = lo_frame + kWgStride * (int32_t)(st0 + S * (uint32_t)k);
                    A[k] = load_stream16_any(base >= 0 ? U.cp + base + 16 * t : zero);
                }
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            }
            if constexpr (CRC) ipre = index_prefetch(p, g, g < h.n_idx, t, zero);
        } else {
            if (has) U = resolve_unit(p, c * h.nseg, expected);
            ok = has && U.mode == ZHIP_ST_OK;
            if constexpr (CRC) ipre = index_prefetch(p, g, g < h.n_idx, t, zero);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int32_t base = lo_frame + kWgStride * (int32_t)(st0 + S * (uint32_t)k);
                A[k] = load_stream16_any(ok && base >= 0 ? U.cp + base + 16 * t : zero);
            }
        }
        if (!has) {
            U.c = 0;
            U.sidx = 0;
            U.mode = ZHIP_ST_MISSING;
            U.cp = zero;
            U.seg_lo = 0;
            U.sel = 0;
            U.out_off = 0;
        }
    } else {
    const uint32_t wpc = p.nseg, S = p.il_S;  // workgroups per chunk = its 32 KiB units
    c = g / wpc;
    r = g - c * wpc;
    has = c < p.n_chunks;
    if (!has && g >= p.n_idx) return;
    if constexpr (TUNE) stamp(p, g, t, 0);
    // 1. vector loads in a path-independent order and count: [CRC: tables (6),
    //    the lane constant, the index lane constant, the first index block],
    //    the K data blocks; headers, row-map entries and the trailer are scalar
    if constexpr (CRC) {
        // (timing arm kTuneNoTables: every lane reads one zero line instead of
        // the 24 KiB of tables; results invalid)
        const bool ntab = TUNE && (p.tune & kTuneNoTables) != 0;
        const uint4* gt = ntab ? reinterpret_cast<const uint4*>(g_rows_zero)
                               : reinterpret_cast<const uint4*>(p.il_tab);
        const int ti = ntab ? 0 : t, ts = ntab ? 0 : kThreads;
        tv0 = gt[ti];
        tv1 = gt[ti + ts];
        tv2 = gt[ti + 2 * ts];
        tv3 = gt[ti + 3 * ts];
        tv4 = gt[ti + 4 * ts];
        tv5 = gt[ti + 5 * ts];
        kl = load_u32_any(reinterpret_cast<const uint8_t*>(p.il_klane + (size_t)(has ? r : 0u) * kThreads + t));
        kix = load_u32_any(reinterpret_cast<const uint8_t*>(p.il_kidx + t));
        // the previous launch's verdict of this chunk (deferred verdicts)
        if constexpr (PUB == 2) dvprev = dv_prev(p, c, has && r == 0, g_rows_zero);
    }
    if (has) U = resolve_unit(p, c * p.nseg, expected);
    else {
        U.c = 0;
        U.sidx = 0;
        U.mode = ZHIP_ST_MISSING;
        U.cp = zero;
        U.seg_lo = 0;
        U.sel = 0;
        U.out_off = 0;
    }
    ok = has && U.mode == ZHIP_ST_OK;
    st0 = (r / S) * S * (uint32_t)K + (r % S);
    lo_frame = (int32_t)p.E - (int32_t)(p.nseg * p.seg);
    if constexpr (CRC) ipre = index_prefetch(p, g, g < p.n_idx, t, zero);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int32_t base = lo_frame + kWgStride * (int32_t)(st0 + p.il_S * (uint32_t)k);
        A[k] = load_stream16_any(ok && base >= 0 ? U.cp + base + 16 * t : zero);
    }
    if constexpr (TUNE) stamp(p, g, t, 1);
    }
    if constexpr ((PRIO & 2) != 0) __builtin_amdgcn_s_setprio(0);
    const uint32_t S = p.il_S, wpc = p.nseg;
    // destinations of the K steps (scalar loads, consumed at the stores)
    zhip_rowblk m[K];
    // (AFF: only for a chunk whose selection record is whole, sel_whole)
    if (AFF && (!has || sel_whole(p, U.sel))) {
#pragma unroll
        for (int k = 0; k < K; ++k) m[k] = aff_rowblk(p, st0 + S * (uint32_t)k);
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t st = st0 + S * (uint32_t)k;
            const uint32_t sidx = p.nseg - 1u - st / (uint32_t)K;
            m[k] = load_uniform<zhip_rowblk>(p.rowmap + ((size_t)U.sel * p.nseg + sidx) * K + (st % (uint32_t)K));
        }
    }
    uint32_t stored = 0;
    if (CRC && ok) stored = load_trailer_uniform(U.cp, p.g.nbytes);
    // 2. tables into LDS, the lane-multiply column
    if constexpr (CRC) {
        uint4* stt = reinterpret_cast<uint4*>(s_tab);
        stt[t] = tv0;
        stt[t + kThreads] = tv1;
        stt[t + 2 * kThreads] = tv2;
        stt[t + 3 * kThreads] = tv3;
        stt[t + 4 * kThreads] = tv4;
        stt[t + 5 * kThreads] = tv5;
        if constexpr (LM == 0) lanemul3_init(s_mul, t, kl);
        __syncthreads();
        if constexpr ((PRIO & 4) != 0) __builtin_amdgcn_s_setprio(0);
        if constexpr (TUNE) stamp(p, g, t, 2);
    }
    if (has) {
        // 3. stores, each block's Horner step after its store
        uint8_t* sink = reinterpret_cast<uint8_t*>(g_rows_sink);
        const uint32_t lane_row = (16u * (uint32_t)t) >> p.row_shift;
        const uint32_t lane_col = (16u * (uint32_t)t) & ((1u << p.row_shift) - 1u);
        const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
        const bool writes = ok || U.mode == ZHIP_ST_MISSING;
        uint8_t* const obase = p.out + U.out_off;
        const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
        Acc4 acc = {0u, 0u, 0u, 0u};
#if ZHIP_TUNING
        __amdgpu_buffer_rsrc_t ors;
        if constexpr (STW != 0) ors = __builtin_amdgcn_make_buffer_rsrc(obase, (short)0, 0x7FFFFFF0, 0x00020000);
#endif
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t lo = m[k].lo, hi = m[k].hi;
            const bool wr = writes && lane_row - lo < hi - lo;
#if ZHIP_TUNING
            if constexpr (STW != 0) {
                const uint4 v = ok ? swap_block<ITEM, SWAP>(A[k]) : f;
                zhip_v4u w = {v.x, v.y, v.z, v.w};
                __builtin_amdgcn_raw_buffer_store_b128(w, ors, wr ? (int)(m[k].rel + lane_off) : 0x7FFFFFF0, 0,
                                                       STW == 1 ? 16 : 2);
            } else
#endif
            store_nt16(wr ? obase + m[k].rel + lane_off : sink, ok ? swap_block<ITEM, SWAP>(A[k]) : f);
            if constexpr (CF) {  // timing arm: the lookups at lane-owned banks (results invalid)
                if (CRC && ok) crc_block4_cf(s_tab, acc, A[k], (uint32_t)t & 31u);
            } else {
                if (CRC && ok) crc_block4(s_tab, acc, A[k]);
            }
        }
        // 4. run end: one chain per workgroup, one publication
        if constexpr ((PRIO & 1) != 0) __builtin_amdgcn_s_setprio(3);
        if constexpr (TUNE) stamp(p, g, t, 3);
        if constexpr (CRC) {
            uint32_t v = ok ? ((TUNE && (p.tune & kTuneNoRunEnd)) ? acc.a0 ^ acc.a1 ^ acc.a2 ^ acc.a3  // timing arm
                               : LM == 0 ? lanemul3(s_mul, t, fold4(s_tab, acc))
                                         : lanemul_reg(kl, fold4(s_tab, acc)))
                            : 0u;
            v = wave_xor(v);
            if ((t & 63) == 0) s_red[0][t >> 6] = v;
            __syncthreads();
            if (ok && t < 64 && !(TUNE && (p.tune & kTuneNoPub))) {
                const uint32_t V = __builtin_amdgcn_readfirstlane(s_red[0][0] ^ s_red[0][1] ^ s_red[0][2] ^ s_red[0][3]);
                if constexpr (TUNE) stamp(p, g, t, 4);
                if constexpr (PUB == 2) {
                    if (t == 0) dv_publish(p, c, r == 0, V, __builtin_amdgcn_readfirstlane(stored));
                } else if constexpr (PUB == 3) {  // the chunk's word alone in its line
                    publish_il(p, c, r, wpc, V, __builtin_amdgcn_readfirstlane(stored), t, kPubLine / 2u);
                } else if constexpr (PUB == 5) {  // look-back finalizer (arm 58)
                    publish_lb(p, c, r, wpc, V, __builtin_amdgcn_readfirstlane(stored), t, kPubLine / 2u);
                } else if constexpr (PUB == 4) {  // two subwords of 16 (tuning arm 49)
                    if (wpc > 16u && wpc <= 32u)
                        publish_il_split(p, c, r, wpc, V, __builtin_amdgcn_readfirstlane(stored), t);
                    else
                        publish_il(p, c, r, wpc, V, __builtin_amdgcn_readfirstlane(stored), t, kPubLine / 2u);
                } else {
                    publish_il(p, c, r, wpc, V, __builtin_amdgcn_readfirstlane(stored), t);
                }
            }
        }
        // (deferred verdicts: the status of a present chunk is OK here; a
        // mismatch is reported from its bank word)
        if (r == 0) unit_status_pair(p, U, CRC && PUB != 2, t);
        if constexpr (CRC && PUB == 2)
            if (r == 0 && t == 0) dv_settle(p, c, dvprev);  // the previous launch's mismatch: sticky
    }
    if constexpr (TUNE) stamp(p, g, t, 7);
    // 5. fused shard-index checks (one step per lane: launch_decode admits
    //    this kernel only then), the first block prefetched with the data
    if constexpr (CRC)
        for (uint32_t j = g; j < p.n_idx; j += G) verify_index_pair(p, j, t, kix, s_tab, s_red[1], j == g, ipre);
}

#if ZHIP_TUNING
KernelFn select_il_kernel_tuned(bool crc, int item, bool swap) {  // runtime timing arms (p.tune)
    return (crc && item == 4 && !swap) ? k_decode_il<true, 4, false, false, false, 0, true> : nullptr;
}

KernelFn select_il_kernel_arm(bool crc, int item, bool swap, int arm) {  // ZHIP_TUNE_ARM experiments
    if (!(crc && item == 4 && !swap)) return nullptr;
    switch (arm) {
        case 1: return k_decode_il<true, 4, false, false, false, 0, false, 0>;  // round 3: words 16 B apart
        case 2: return k_decode_il<true, 4, false, false, false, 0, false, 2>;  // deferred verdicts
        case 49: return k_decode_il<true, 4, false, false, false, 0, false, 4, true>;  // split publication (AFF)
        case 51: return k_decode_il<true, 4, false, false, false, 0, false, 3, true, 1>;  // priority: run end (AFF)
        case 52: return k_decode_il<true, 4, false, false, false, 0, false, 3, true, 2>;  // priority: load issue (AFF)
        case 53: return k_decode_il<true, 4, false, false, false, 0, false, 3, true, 3>;  // priority: both (AFF)
        case 54: return k_decode_il<true, 4, false, false, false, 0, false, 3, true, 4>;  // priority: to the tables (AFF; production)
        case 56: return k_decode_il<true, 4, false, false, false, 0, false, 3, true, 0>;  // no priority (AFF; round-5 production)
        case 57: return k_decode_il<true, 4, false, false, false, 0, false, 3, true, 12>;  // 54 + XCD eighths (AFF)
        case 55: return k_decode_il<true, 4, false, false, false, 0, false, 3, true, 5>;  // 54 + run end (AFF)
        case 58: return k_decode_il<true, 4, false, false, false, 0, false, 5, true, 4>;  // 54 + look-back finalizer (AFF)
        case 64: return k_decode_il<true, 4, false, false, false, 0, false, 3, true, 4, 1>;  // 54 + write-through stores
        case 65: return k_decode_il<true, 4, false, false, false, 0, false, 3, true, 4, 2>;  // 54 + buffer nt stores
        default: return k_decode_il<true, 4, false>;  // arms of other kernels: production
    }
}

#endif

// Deferred verdicts of whole batches (zhip_dv_check): both banks' words of
// every chunk of every referenced launch folded into its statuses + errflag
// and cleared (blockIdx.y = the launch).
__global__ void k_dv_check(const zhip_dv_ref* refs) {
    const zhip_dv_ref R = refs[blockIdx.y];
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < R.n_chunks; c += gridDim.x * blockDim.x) {
        for (uint32_t b = 0; b < 2; ++b) {
            const uint32_t w = R.workspace[4ull * c + 2u * b];
            if (w != 0u) {
                const uint32_t st = R.workspace[4ull * c + 2u * b + 1u];
                zhip_status s = {ZHIP_ST_CRC_MISMATCH, st, w ^ st, 0u};
                R.status[c] = s;
                atomicOr(R.errflag, 1u << ZHIP_ST_CRC_MISMATCH);
                R.workspace[4ull * c + 2u * b] = 0u;
            }
        }
    }
}

int launch_dv_check(const zhip_dv_ref* d_refs, uint32_t n_refs, hipStream_t stream) {
    if (n_refs == 0) return ZHIP_OK;
    hipLaunchKernelGGL(k_dv_check, dim3(16, n_refs), dim3(256), 0, stream, d_refs);
    return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
}

#if ZHIP_TUNING
KernelFn select_il_kernel_lean(bool crc, int item, bool swap) {  // kTuneIlLean (4-byte LE CRC item type only)
    return (crc && item == 4 && !swap) ? k_decode_il<true, 4, false, true> : nullptr;
}

KernelFn select_il_kernel_cf(bool crc, int item, bool swap) {  // kTuneCfLookup timing arm (results invalid)
    return (crc && item == 4 && !swap) ? k_decode_il<true, 4, false, false, true> : nullptr;
}

KernelFn select_il_kernel_regmul(bool crc, int item, bool swap, bool occ6) {  // kTuneIlRegMul / kTuneIlOcc6 arms
    if (!(crc && item == 4 && !swap)) return nullptr;
    return occ6 ? k_decode_il<true, 4, false, false, false, 2> : k_decode_il<true, 4, false, false, false, 1>;
}

#endif

KernelFn select_il_kernel(bool crc, int item, bool swap, bool aff) {  // aff: ZHIP_DF_WHOLE (CRC chains)
#define ZHIP_IL(I, W) (aff ? k_decode_il<true, I, W, false, false, 0, false, 3, true, 4> : k_decode_il<true, I, W>)
    switch (item) {
        case 1: return crc ? ZHIP_IL(1, false) : k_decode_il<false, 1, false>;
        case 2: return crc ? (swap ? ZHIP_IL(2, true) : ZHIP_IL(2, false))
                           : (swap ? k_decode_il<false, 2, true> : k_decode_il<false, 2, false>);
        case 4: return crc ? (swap ? ZHIP_IL(4, true) : ZHIP_IL(4, false))
                           : (swap ? k_decode_il<false, 4, true> : k_decode_il<false, 4, false>);
        case 8: return crc ? (swap ? ZHIP_IL(8, true) : ZHIP_IL(8, false))
                           : (swap ? k_decode_il<false, 8, true> : k_decode_il<false, 8, false>);
        default: return nullptr;
    }
#undef ZHIP_IL
}

// ---------------------------------------------------------------------------
// k_decode_ilq: k_decode_il with NQ consecutive units of one chunk per
// workgroup (NQ x 256 threads).  Quarter q = threadIdx.x / 256 runs unit
// r0 + q exactly as k_decode_il's workgroup r0 + q would (same loads, row-map
// stores, one 8-step Horner chain per lane through the A_(4096 S) tables, the
// same host-built lane constants), but the NQ units share one 24 KiB table
// fill, one workgroup reduction and one publication (arrival bits
// ((1 << NQ) - 1) << r0), so per byte decoded the table traffic, the run-end
// barrier and the returning atomics drop by NQ.  GLDS: the tables go global
// -> LDS by LDS-DMA (global_load_lds_dwordx4, issued in inline asm ahead of
// every compiler-visible data load, so the compiler's counted vmcnt waits
// stay exact; one manual vmcnt before the table barrier), which frees the
// staging VGPRs and the ds_write_b128 transfers.  CPU emulation of the CRC
// algebra: zhip_emulate_chunk_crc_il (the chains are k_decode_il's).
__device__ __forceinline__ uint32_t lds_addr32(const void* a) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)a;
}

// One LDS-DMA piece: lane i's 16 bytes at g land at LDS byte lds + 16 i (lds
// wave-uniform).  M0 is saved and restored around it.
__device__ __forceinline__ void glds16(const void* g, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds)
                 : "memory");
}

// publish_il for a workgroup carrying several arrival bits of chunk c
__device__ __forceinline__ void publish_ilq(const DecodeParams& p, uint32_t c, uint32_t r0, uint32_t nq, uint32_t wpc,
                                            uint32_t V, uint32_t stored, int t) {
    if (wpc <= 32u) {
        const uint64_t full = wpc >= 32u ? 0xFFFFFFFFull : ((1ull << wpc) - 1ull);
        const uint32_t bits = ((1u << nq) - 1u) << r0;
        uint64_t prev = 0;
        uint64_t* const w = reinterpret_cast<uint64_t*>(p.ws) + (uint64_t)(kPubLine / 2u) * c;
        if (t == 0) prev = __hip_atomic_fetch_xor(w, ((uint64_t)bits << 32) | V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)prev);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(prev >> 32));
        if ((uint64_t)(hi ^ bits) == full) {
            if (t == 0) __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            finalize_uniform(p, c, stored, lo ^ V, t, true);
        }
    } else {  // more than 32 units per chunk: xor, then count arrivals
        uint32_t raw = 0, last = 0;
        if (t == 0) {
            uint32_t* accw = p.ws + 4ull * c;
            const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
            const uint32_t tk = __hip_atomic_fetch_add(accw + 2, nq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tk + nq == wpc) {
                raw = __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::"v"(raw) : "memory");
                __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = 1;
            }
        }
        if (__builtin_amdgcn_readfirstlane(last))
            finalize_uniform(p, c, stored, __builtin_amdgcn_readfirstlane(raw), t, true);
    }
}

template <int ITEM, bool SWAP, int NQ, bool GLDS>
__global__ __launch_bounds__(NQ * kThreads) __attribute__((amdgpu_waves_per_eu(NQ == 4 ? 8 : NQ == 2 ? 6 : 4)))
void k_decode_ilq(const DecodeParams p) {
    constexpr int K = kDefaultBlocks;
    constexpr int NT = NQ * kThreads;
    constexpr int NTV = kPairTabWords / 4;  // 16-byte table pieces
    constexpr int NL = (NTV + NT - 1) / NT;
    static_assert(K == 8, "the manual table wait below counts K + 1 younger loads");
    __shared__ uint32_t s_tab[kPairTabWords];
    __shared__ uint32_t s_mul[12 * NT];
    __shared__ uint32_t s_red[NT / 64];
    __shared__ uint32_t s_ridx[4 * NQ];
    const int T = threadIdx.x;
    const int q = T >> 8, t = T & (kThreads - 1);
    const uint32_t G = gridDim.x, g = blockIdx.x;
    const uint32_t wpc = p.nseg, S = p.il_S;
    const uint32_t u0 = g * (uint32_t)NQ;
    const uint32_t c = u0 / wpc;
    const uint32_t r0 = u0 - c * wpc, r = r0 + (uint32_t)q;
    const bool has = c < p.n_chunks;
    if (!has && u0 >= p.n_idx) return;  // workgroup-uniform
    const uint32_t expected = p.g.nbytes + 4u;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_rows_zero);
    // 1. vector loads: the lane constants, [GLDS: the table pieces], the K data
    //    blocks, the first index block; headers, row map, trailer are scalar
    const uint32_t kl = load_u32_any(reinterpret_cast<const uint8_t*>(p.il_klane + (size_t)(has ? r : 0u) * kThreads + t));
    const uint32_t kix = load_u32_any(reinterpret_cast<const uint8_t*>(p.il_kidx + t));
    const uint4* gt = reinterpret_cast<const uint4*>(p.il_tab);
    uint4 tv[GLDS ? 1 : NL];
    if constexpr (GLDS) {
        const uint32_t wv = (uint32_t)T & ~63u;
        const uint32_t lb = __builtin_amdgcn_readfirstlane(lds_addr32(s_tab) + 16u * wv);
#pragma unroll
        for (int i = 0; i < NL; ++i)
            if ((uint32_t)(i * NT) + wv < (uint32_t)NTV) glds16(gt + i * NT + T, lb + 16u * (uint32_t)(i * NT));
    } else {
#pragma unroll
        for (int i = 0; i < NL; ++i) tv[i] = gt[min(i * NT + T, NTV - 1)];
    }
    Unit U;
    if (has) U = resolve_unit(p, c * wpc, expected);
    else {
        U.c = 0;
        U.sidx = 0;
        U.mode = ZHIP_ST_MISSING;
        U.cp = zero;
        U.seg_lo = 0;
        U.sel = 0;
        U.out_off = 0;
    }
    const bool ok = has && U.mode == ZHIP_ST_OK;
    const uint32_t st0 = (r / S) * S * (uint32_t)K + (r % S);
    const int32_t lo_frame = (int32_t)p.E - (int32_t)(p.nseg * p.seg);
    uint4 A[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int32_t base = lo_frame + kWgStride * (int32_t)(st0 + S * (uint32_t)k);
        A[k] = load_stream16_any(ok && base >= 0 ? U.cp + base + 16 * t : zero);
    }
    const uint32_t jq = u0 + (uint32_t)q;
    const uint4 ipre = index_prefetch(p, jq, jq < p.n_idx, t, zero);
    zhip_rowblk m[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t st = st0 + S * (uint32_t)k;
        const uint32_t sidx = p.nseg - 1u - st / (uint32_t)K;
        m[k] = load_uniform<zhip_rowblk>(p.rowmap + ((size_t)U.sel * p.nseg + sidx) * K + (st % (uint32_t)K));
    }
    uint32_t stored = 0;
    if (ok) stored = load_trailer_uniform(U.cp, p.g.nbytes);
    // 2. tables into LDS, the lane-multiply column of this quarter
    uint32_t* const smq = s_mul + q * 12 * kThreads;
    if constexpr (GLDS) {
        asm volatile("s_waitcnt vmcnt(9)" ::: "memory");  // all but the K data loads and the index block
    } else {
        uint4* stt = reinterpret_cast<uint4*>(s_tab);
#pragma unroll
        for (int i = 0; i < NL; ++i)
            if (i * NT + T < NTV) stt[i * NT + T] = tv[i];
    }
    lanemul3_init(smq, t, kl);
    __syncthreads();
    if (has) {
        // 3. stores, each block's Horner step after its store
        uint8_t* sink = reinterpret_cast<uint8_t*>(g_rows_sink);
        const uint32_t lane_row = (16u * (uint32_t)t) >> p.row_shift;
        const uint32_t lane_col = (16u * (uint32_t)t) & ((1u << p.row_shift) - 1u);
        const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
        const bool writes = ok || U.mode == ZHIP_ST_MISSING;
        uint8_t* const obase = p.out + U.out_off;
        const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
        Acc4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t lo = m[k].lo, hi = m[k].hi;
            const bool wr = writes && lane_row - lo < hi - lo;
            store_nt16(wr ? obase + m[k].rel + lane_off : sink, ok ? swap_block<ITEM, SWAP>(A[k]) : f);
            if (ok) crc_block4(s_tab, acc, A[k]);
        }
        // 4. run end: one reduction and one publication for the NQ units
        uint32_t v = ok ? lanemul3(smq, t, fold4(s_tab, acc)) : 0u;
        v = wave_xor(v);
        if ((T & 63) == 0) s_red[T >> 6] = v;
        __syncthreads();
        if (ok && T < 64) {
            uint32_t V = 0;
#pragma unroll
            for (int w = 0; w < NT / 64; ++w) V ^= s_red[w];
            publish_ilq(p, c, r0, (uint32_t)NQ, wpc, __builtin_amdgcn_readfirstlane(V),
                        __builtin_amdgcn_readfirstlane(stored), T);
        }
        if (r == 0) unit_status_pair(p, U, true, t);
    }
    // 5. fused shard-index checks: quarter q checks index jj NQ + q (one step
    //    per lane), every quarter joins every barrier
    for (uint32_t jj = g; jj * (uint32_t)NQ < p.n_idx; jj += G) {
        const uint32_t j = jj * (uint32_t)NQ + (uint32_t)q;
        const bool act = j < p.n_idx;
        verify_index_pair(p, act ? j : 0u, t, kix, s_tab, s_ridx + 4 * q, act && jj == g, ipre, act);
    }
}

// ---------------------------------------------------------------------------
// k_decode_ilc: k_decode_il without a table load and without the header chain
// in front of its data loads.  The workgroup timeline of k_decode_il
// (scripts/stamps.py, profiles/r05/b/): start -> data loads issued 1.8 us
// median (2.7 us for the slowest 5 %: kernel arguments, then the chunk
// record, then the shard-index entry, dependent scalar round trips under a
// saturated memory system), -> tables in LDS 1.3 us (24 KiB of L2 reads per
// workgroup), -> stores and Horner steps 3.1 us, -> run end 0.9 us, -> exit
// 0.5 us.  Here the data loads go out right after the kernel arguments, at
// the addresses the default shard packing predicts (zhip_predict; a wrong
// guess reloads once the index entry arrives, as k_decode_lead), behind only
// the lane constant (the oldest load, an L2 hit), and the A_(4096 S)
// 11/11/10 tables and the A4 fold tables are BUILT in LDS while the data is
// in flight: every table is linear in its index, so entry i is the XOR of the
// single-bit entries of i's set bits (64 host-built words, scalar loads);
// thread t writes T1 / T2 entries 4t..4t+3 (+1024), T3 entries 4t..4t+3 and
// A4 entry t of each byte table: 8 lane masks, ~60 VALU, 5 ds_write_b128 +
// 4 ds_write_b32 per thread, no vector memory.  The rest -- stores, chains,
// run end, publication, fused index checks -- is k_decode_il's.
__device__ __forceinline__ void build_il_tables_lds(uint32_t* s, int t, const uint32_t* gbasis) {
    struct B64 {
        uint32_t w[kIlBasisWords];
    };
    const B64 B = load_uniform<B64>(gbasis);
    uint32_t m[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) m[b] = 0u - (((uint32_t)t >> b) & 1u);
    auto lane_part = [&](int off) {
        uint32_t L = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b) L ^= m[b] & B.w[off + b];
        return L;
    };
    {  // T1 (index bits 0..10 of a word): entry 4t + q + 1024 h
        const uint32_t L = lane_part(2), q1 = B.w[0], q2 = B.w[1], hb = B.w[10];
        const uint4 lo = make_uint4(L, L ^ q1, L ^ q2, L ^ q1 ^ q2);
        *reinterpret_cast<uint4*>(s + kPairT1 + 4 * t) = lo;
        *reinterpret_cast<uint4*>(s + kPairT1 + 1024 + 4 * t) =
            make_uint4(lo.x ^ hb, lo.y ^ hb, lo.z ^ hb, lo.w ^ hb);
    }
    {  // T2 (bits 11..21)
        const uint32_t L = lane_part(13), q1 = B.w[11], q2 = B.w[12], hb = B.w[21];
        const uint4 lo = make_uint4(L, L ^ q1, L ^ q2, L ^ q1 ^ q2);
        *reinterpret_cast<uint4*>(s + kPairT2 + 4 * t) = lo;
        *reinterpret_cast<uint4*>(s + kPairT2 + 1024 + 4 * t) =
            make_uint4(lo.x ^ hb, lo.y ^ hb, lo.z ^ hb, lo.w ^ hb);
    }
    {  // T3 (bits 22..31): entry 4t + q
        const uint32_t L = lane_part(24), q1 = B.w[22], q2 = B.w[23];
        *reinterpret_cast<uint4*>(s + kPairT3 + 4 * t) = make_uint4(L, L ^ q1, L ^ q2, L ^ q1 ^ q2);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) s[kPairA4 + 256 * j + t] = lane_part(32 + 8 * j);  // A4 byte tables
}

template <int ITEM, bool SWAP>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_decode_ilc(
    const DecodeParams p) {
    constexpr int K = kDefaultBlocks;
    __shared__ uint32_t s_tab[kPairTabWords];
    __shared__ uint32_t s_mul[12 * kThreads];
    __shared__ uint32_t s_red[2][kThreads / 64];
    const int t = threadIdx.x;
    PairHot h = p.h;
    pair_hot(h);
    il_hot(h);
    const uint32_t G = gridDim.x, g = blockIdx.x;
    const uint32_t wpc = h.nseg, S = h.il_S;
    const uint32_t c = fdiv_apply(g, h.d_nseg.m, h.d_nseg.s);
    const uint32_t r = g - c * wpc;
    const bool has = c < h.n_chunks;
    if (!has && g >= h.n_idx) return;
    const uint32_t expected = p.g.nbytes + 4u;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_rows_zero);
    // 1. the lane constants (the oldest loads: waited for alone), then the data
    const uint32_t kl = load_u32_any(reinterpret_cast<const uint8_t*>(
        reinterpret_cast<const uint32_t*>(h.il_klane) + (size_t)(has ? r : 0u) * kThreads + t));
    const uint32_t kix = load_u32_any(reinterpret_cast<const uint8_t*>(reinterpret_cast<const uint32_t*>(h.il_kidx) + t));
    const uint32_t ls = (uint32_t)__builtin_ctz(S);
    const uint32_t st0 = ((r >> ls) << ls) * (uint32_t)K + (r & (S - 1u));
    const int32_t lo_frame = (int32_t)h.E - (int32_t)(h.nseg * h.seg);
    uint4 A[K];
    const uint8_t* cpp = zero;
    if (h.pred) {
        const uint32_t grp = fdiv_apply(c, h.d_per.m, h.d_per.s);
        cpp = reinterpret_cast<const uint8_t*>(h.src) + h.pred_base + (uint64_t)grp * h.pred_outer +
              (uint64_t)(c - grp * h.pred_per) * h.pred_inner;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int32_t base = lo_frame + kWgStride * (int32_t)(st0 + S * (uint32_t)k);
            A[k] = load_stream16_any(has && base >= 0 ? cpp + base + 16 * t : zero);
        }
    }
    // 2. the tables built in LDS (no memory reads but 64 scalar words), the lane-multiply column
    build_il_tables_lds(s_tab, t, p.il_basis);
    lanemul3_init(s_mul, t, kl);
    // 3. the header chain: verifies the guess (or, unpredicted, addresses the loads)
    Unit U;
    if (has) U = resolve_unit(p, c * h.nseg, expected);
    else {
        U.c = 0;
        U.sidx = 0;
        U.mode = ZHIP_ST_MISSING;
        U.cp = zero;
        U.seg_lo = 0;
        U.sel = 0;
        U.out_off = 0;
    }
    const bool ok = has && U.mode == ZHIP_ST_OK;
    if (h.pred) {
        if (ok && U.cp != cpp) {  // a wrong guess: reload from the live index, full drain
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int32_t base = lo_frame + kWgStride * (int32_t)(st0 + S * (uint32_t)k);
                A[k] = load_stream16_any(base >= 0 ? U.cp + base + 16 * t : zero);
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        }
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int32_t base = lo_frame + kWgStride * (int32_t)(st0 + S * (uint32_t)k);
            A[k] = load_stream16_any(ok && base >= 0 ? U.cp + base + 16 * t : zero);
        }
    }
    const uint4 ipre = index_prefetch(p, g, g < h.n_idx, t, zero);
    zhip_rowblk m[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t st = st0 + S * (uint32_t)k;
        const uint32_t sidx = h.nseg - 1u - st / (uint32_t)K;
        m[k] = load_uniform<zhip_rowblk>(p.rowmap + ((size_t)U.sel * h.nseg + sidx) * K + (st % (uint32_t)K));
    }
    uint32_t stored = 0;
    if (ok) stored = load_trailer_uniform(U.cp, p.g.nbytes);
    __syncthreads();
    if (has) {
        // 4. stores, each block's Horner step after its store
        uint8_t* sink = reinterpret_cast<uint8_t*>(g_rows_sink);
        const uint32_t lane_row = (16u * (uint32_t)t) >> p.row_shift;
        const uint32_t lane_col = (16u * (uint32_t)t) & ((1u << p.row_shift) - 1u);
        const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
        const bool writes = ok || U.mode == ZHIP_ST_MISSING;
        uint8_t* const obase = p.out + U.out_off;
        const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
        Acc4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t lo = m[k].lo, hi = m[k].hi;
            const bool wr = writes && lane_row - lo < hi - lo;
            store_nt16(wr ? obase + m[k].rel + lane_off : sink, ok ? swap_block<ITEM, SWAP>(A[k]) : f);
            if (ok) crc_block4(s_tab, acc, A[k]);
        }
        // 5. run end: one chain per workgroup, one publication
        uint32_t v = ok ? lanemul3(s_mul, t, fold4(s_tab, acc)) : 0u;
        v = wave_xor(v);
        if ((t & 63) == 0) s_red[0][t >> 6] = v;
        __syncthreads();
        if (ok && t < 64) {
            const uint32_t V = __builtin_amdgcn_readfirstlane(s_red[0][0] ^ s_red[0][1] ^ s_red[0][2] ^ s_red[0][3]);
            publish_il(p, c, r, wpc, V, __builtin_amdgcn_readfirstlane(stored), t, kPubLine / 2u);
        }
        if (r == 0) unit_status_pair(p, U, true, t);
    }
    // 6. fused shard-index checks (one step per lane), the first block prefetched
    for (uint32_t j = g; j < h.n_idx; j += G) verify_index_pair(p, j, t, kix, s_tab, s_red[1], j == g, ipre);
}

// ---------------------------------------------------------------------------
// k_decode_ilp: k_decode_ilc with the shard-index entry OFF the stores' path.
// k_decode_ilc / the lean prologue issue the data at the predicted address
// first but still resolve the unit (chunk record -> index entry, a cold HBM
// read behind the data flood) before storing.  Here the stores need only the
// chunk record and the row map (small hot tables); the index entry and the
// predicted trailer are VECTOR loads issued after the data (so waiting for the
// data never waits for them), checked after the Horner steps: a wrong guess,
// an index-missing or failing inner chunk redoes the unit on a slow path
// (drain, reload or fill, restore, re-hash).  launch_decode admits it only
// with a prediction (zhip_predict).
template <int ITEM, bool SWAP>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_decode_ilp(
    const DecodeParams p) {
    constexpr int K = kDefaultBlocks;
    __shared__ uint32_t s_tab[kPairTabWords];
    __shared__ uint32_t s_mul[12 * kThreads];
    __shared__ uint32_t s_red[2][kThreads / 64];
    const int t = threadIdx.x;
    PairHot h = p.h;
    pair_hot(h);
    il_hot(h);
    const uint32_t G = gridDim.x, g = blockIdx.x;
    const uint32_t wpc = h.nseg, S = h.il_S;
    const uint32_t c = fdiv_apply(g, h.d_nseg.m, h.d_nseg.s);
    const uint32_t r = g - c * wpc;
    const bool has = c < h.n_chunks;
    if (!has && g >= h.n_idx) return;
    stamp(p, g, t, 0);
    const uint32_t expected = p.g.nbytes + 4u;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_rows_zero);
    const uint32_t ls = (uint32_t)__builtin_ctz(S);
    const uint32_t st0 = ((r >> ls) << ls) * (uint32_t)K + (r & (S - 1u));
    const int32_t lo_frame = (int32_t)h.E - (int32_t)(h.nseg * h.seg);
    // 1. the data at the predicted address, first
    const uint32_t grp = fdiv_apply(c, h.d_per.m, h.d_per.s);
    const uint8_t* const cpp = reinterpret_cast<const uint8_t*>(h.src) + h.pred_base + (uint64_t)grp * h.pred_outer +
                               (uint64_t)(c - grp * h.pred_per) * h.pred_inner;
    uint4 A[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int32_t base = lo_frame + kWgStride * (int32_t)(st0 + S * (uint32_t)k);
        A[k] = load_stream16_any(has && base >= 0 ? cpp + base + 16 * t : zero);
    }
    stamp(p, g, t, 1);
    // 2. the chunk record and the row map (scalar, hot), the lane constants,
    //    the index entry and the predicted trailer (vector, after the data)
    zhip_chunk ch = {};
    if (has) ch = load_uniform<zhip_chunk>(p.chunks + c);
    const uint32_t kl = load_u32_any(reinterpret_cast<const uint8_t*>(
        reinterpret_cast<const uint32_t*>(h.il_klane) + (size_t)(has ? r : 0u) * kThreads + t));
    const uint32_t kix = load_u32_any(reinterpret_cast<const uint8_t*>(reinterpret_cast<const uint32_t*>(h.il_kidx) + t));
    const bool sharded = (p.lflags & ZHIP_LF_SHARDED) != 0;
    const bool ch_missing = (ch.flags & ZHIP_CF_MISSING) != 0;
    const uint64_t ipos = (p.lflags & ZHIP_LF_INDEX_START) ? 0ull : ch.src_len - p.index_size;
    const uint4 ie = load16_any(has && sharded && !ch_missing ? p.src + ch.src + ipos + 16ull * ch.slot : zero);
    const uint32_t trp = load_u32_any(has ? cpp + p.g.nbytes : zero);
    const uint4 ipre = index_prefetch(p, g, g < h.n_idx, t, zero);
    zhip_rowblk m[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t st = st0 + S * (uint32_t)k;
        const uint32_t sidx = h.nseg - 1u - st / (uint32_t)K;
        m[k] = load_uniform<zhip_rowblk>(p.rowmap + ((size_t)ch.sel * h.nseg + sidx) * K + (st % (uint32_t)K));
    }
    // 3. tables built in LDS, the lane-multiply column
    build_il_tables_lds(s_tab, t, p.il_basis);
    lanemul3_init(s_mul, t, kl);
    __syncthreads();
    stamp(p, g, t, 2);
    uint8_t* sink = reinterpret_cast<uint8_t*>(g_rows_sink);
    const uint32_t lane_row = (16u * (uint32_t)t) >> p.row_shift;
    const uint32_t lane_col = (16u * (uint32_t)t) & ((1u << p.row_shift) - 1u);
    const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
    uint8_t* const obase = p.out + ch.out_off;
    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
    Acc4 acc = {0u, 0u, 0u, 0u};
    if (has) {
        // 4. stores and Horner steps of the predicted data (a chunk the chunk
        //    record marks missing: fill)
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t lo = m[k].lo, hi = m[k].hi;
            const bool wr = lane_row - lo < hi - lo;
            store_nt16(wr ? obase + m[k].rel + lane_off : sink, ch_missing ? f : swap_block<ITEM, SWAP>(A[k]));
            if (!ch_missing) crc_block4(s_tab, acc, A[k]);
        }
    }
    stamp(p, g, t, 3);
    // 5. the unit as resolve_unit sees it (zhip_decode_common.h), from the
    //    vector-loaded entry
    uint32_t mode = ch_missing ? (uint32_t)ZHIP_ST_MISSING : (uint32_t)ZHIP_ST_OK;
    uint64_t base = ch.src;
    if (has && !ch_missing) {
        if (sharded) {
            const uint64_t off = ((uint64_t)__builtin_amdgcn_readfirstlane(ie.y) << 32) |
                                 __builtin_amdgcn_readfirstlane(ie.x);
            const uint64_t len = ((uint64_t)__builtin_amdgcn_readfirstlane(ie.w) << 32) |
                                 __builtin_amdgcn_readfirstlane(ie.z);
            if (off == ~0ull && len == ~0ull) mode = ZHIP_ST_MISSING;
            else if (u64_gt(off, ch.src_len) || u64_gt(len, ch.src_len - off)) mode = ZHIP_ST_INDEX_OOB;
            else if (len != expected) mode = ZHIP_ST_LENGTH_MISMATCH;
            else base = ch.src + off;
        } else if (ch.src_len != expected) {
            mode = ZHIP_ST_LENGTH_MISMATCH;
        }
    }
    const uint8_t* const cp = p.src + base;
    const bool ok = has && mode == ZHIP_ST_OK;
    uint32_t stored = __builtin_amdgcn_readfirstlane(trp);
    if (has && !ch_missing && !(ok && cp == cpp)) {
        // a wrong guess, or the index says missing / fails: redo the unit
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the predicted stores are out
        acc = {0u, 0u, 0u, 0u};
        if (ok) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int32_t b2 = lo_frame + kWgStride * (int32_t)(st0 + S * (uint32_t)k);
                A[k] = load_stream16_any(b2 >= 0 ? cp + b2 + 16 * t : zero);
            }
            stored = load_trailer_uniform(cp, p.g.nbytes);
        }
        const bool fill = mode == ZHIP_ST_MISSING;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t lo = m[k].lo, hi = m[k].hi;
            const bool wr = (ok || fill) && lane_row - lo < hi - lo;
            store_nt16(wr ? obase + m[k].rel + lane_off : sink, ok ? swap_block<ITEM, SWAP>(A[k]) : f);
            if (ok) crc_block4(s_tab, acc, A[k]);
        }
    }
    if (has) {
        // 6. run end: one chain per workgroup, one publication
        uint32_t v = ok ? lanemul3(s_mul, t, fold4(s_tab, acc)) : 0u;
        v = wave_xor(v);
        if ((t & 63) == 0) s_red[0][t >> 6] = v;
        __syncthreads();
        if (ok && t < 64) {
            const uint32_t V = __builtin_amdgcn_readfirstlane(s_red[0][0] ^ s_red[0][1] ^ s_red[0][2] ^ s_red[0][3]);
            stamp(p, g, t, 4);
            publish_il(p, c, r, wpc, V, stored, t, kPubLine / 2u);
        }
        if (r == 0) {
            Unit U;
            U.c = c;
            U.sidx = 0;
            U.mode = mode;
            U.cp = cp;
            U.seg_lo = 0;
            U.sel = ch.sel;
            U.out_off = ch.out_off;
            unit_status_pair(p, U, true, t);
        }
    }
    stamp(p, g, t, 7);
    // 7. fused shard-index checks (one step per lane), the first block prefetched
    for (uint32_t j = g; j < h.n_idx; j += G) verify_index_pair(p, j, t, kix, s_tab, s_red[1], j == g, ipre);
}

// ---------------------------------------------------------------------------
// k_decode_ilh (production for small launches since round 6, with LB; tuning
// arm 41 without it): half units -- 16 KiB per workgroup (4 096 on
// the headline: four residency rounds instead of two, the change that gave
// the transposes 1.6 us), lane t taking the four 4 KiB sub-steps 8 r + 4 h + k
// of its segment's half h at 16 t: one chain through the pair kernel's
// A_4096 tables, lane constants per (half unit, lane) from capi.cpp; up to
// 64 workgroups per chunk publish per 32-workgroup word with a second level.
template <int ITEM, bool SWAP, bool LB = false, bool AFF = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_decode_ilh(
    const DecodeParams p) {
    constexpr int KW = 4;
    __shared__ uint32_t s_tab[kPairTabWords];
    __shared__ uint32_t s_mul[12 * kThreads];
    __shared__ uint32_t s_red[2][kThreads / 64];
    const int t = threadIdx.x;
    const uint32_t G = gridDim.x, g = blockIdx.x;
    const uint32_t wpc = 2u * p.nseg;
    const uint32_t c = g / wpc, u = g - c * wpc, r = u >> 1, hh = u & 1u;
    const bool has = c < p.n_chunks;
    if (!has && g >= p.n_idx) return;
    const uint32_t expected = p.g.nbytes + 4u;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_rows_zero);
    const uint4* gt = reinterpret_cast<const uint4*>(p.pair_tab);
    const uint4 tv0 = gt[t], tv1 = gt[t + kThreads], tv2 = gt[t + 2 * kThreads], tv3 = gt[t + 3 * kThreads],
                tv4 = gt[t + 4 * kThreads], tv5 = gt[t + 5 * kThreads];
    const uint32_t kl = load_u32_any(reinterpret_cast<const uint8_t*>(p.ilh_klane + (size_t)(has ? u : 0u) * kThreads + t));
    const uint32_t kix = load_u32_any(reinterpret_cast<const uint8_t*>(p.kthread11 + t));
    Unit U;
    if (has) U = resolve_unit(p, c * p.nseg, expected);
    else {
        U.c = 0;
        U.sidx = 0;
        U.mode = ZHIP_ST_MISSING;
        U.cp = zero;
        U.seg_lo = 0;
        U.sel = 0;
        U.out_off = 0;
    }
    const bool ok = has && U.mode == ZHIP_ST_OK;
    const int32_t lo_frame = (int32_t)p.E - (int32_t)(p.nseg * p.seg);
    const uint4 ipre = index_prefetch(p, g, g < p.n_idx, t, zero);
    uint4 A[KW];
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        const int32_t base = lo_frame + kWgStride * (int32_t)(8u * r + 4u * hh + (uint32_t)k);
        A[k] = load_stream16_any(ok && base >= 0 ? U.cp + base + 16 * t : zero);
    }
    zhip_rowblk m[KW];
    const uint32_t sidx = p.nseg - 1u - r;
    if (AFF && (!has || sel_whole(p, U.sel))) {  // (k_decode_il's AFF, checked by sel_whole)
#pragma unroll
        for (int k = 0; k < KW; ++k) m[k] = aff_rowblk(p, 8u * r + 4u * hh + (uint32_t)k);
    } else {
#pragma unroll
        for (int k = 0; k < KW; ++k)
            m[k] = load_uniform<zhip_rowblk>(p.rowmap + ((size_t)U.sel * p.nseg + sidx) * kDefaultBlocks +
                                             4u * hh + (uint32_t)k);
    }
    uint32_t stored = 0;
    if (ok) stored = load_trailer_uniform(U.cp, p.g.nbytes);
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
    if (has) {
        uint8_t* sink = reinterpret_cast<uint8_t*>(g_rows_sink);
        const uint32_t lane_row = (16u * (uint32_t)t) >> p.row_shift;
        const uint32_t lane_col = (16u * (uint32_t)t) & ((1u << p.row_shift) - 1u);
        const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
        const bool writes = ok || U.mode == ZHIP_ST_MISSING;
        uint8_t* const obase = p.out + U.out_off;
        const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
        Acc4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            const uint32_t lo = m[k].lo, hi = m[k].hi;
            const bool wr = writes && lane_row - lo < hi - lo;
            store_nt16(wr ? obase + m[k].rel + lane_off : sink, ok ? swap_block<ITEM, SWAP>(A[k]) : f);
            if (ok) crc_block4(s_tab, acc, A[k]);
        }
        uint32_t v = ok ? lanemul3(s_mul, t, fold4(s_tab, acc)) : 0u;
        v = wave_xor(v);
        if ((t & 63) == 0) s_red[0][t >> 6] = v;
        __syncthreads();
        if (ok && t < 64) {
            const uint32_t V = __builtin_amdgcn_readfirstlane(s_red[0][0] ^ s_red[0][1] ^ s_red[0][2] ^ s_red[0][3]);
            const uint32_t st = __builtin_amdgcn_readfirstlane(stored);
            if (LB && wpc <= 64u) {  // look-back finalizer (tuning arm 59)
                publish_lb(p, c, u, wpc, V, st, t, kPubLine / 2u);
            } else if (wpc <= 32u) {
                publish_il(p, c, u, wpc, V, st, t, kPubLine / 2u);
            } else {  // words of 32 arrivals, then the line's third word
                uint64_t* const w = reinterpret_cast<uint64_t*>(p.ws) + (uint64_t)(kPubLine / 2u) * c;
                const uint32_t h2 = u >> 5;
                const uint32_t n_h = h2 ? wpc - 32u : 32u;
                const uint64_t bit = 1ull << (u & 31u);
                uint64_t prev = 0;
                if (t == 0) prev = __hip_atomic_fetch_xor(w + h2, (bit << 32) | V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)prev);
                const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(prev >> 32));
                const uint64_t fullh = n_h >= 32u ? 0xFFFFFFFFull : ((1ull << n_h) - 1ull);
                if ((uint64_t)(hi ^ (uint32_t)bit) == fullh) {
                    if (t == 0) __hip_atomic_store(w + h2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint32_t Vh = lo ^ V;
                    const uint64_t hb = 1ull << h2;
                    uint64_t p2 = 0;
                    if (t == 0) p2 = __hip_atomic_fetch_xor(w + 2, (hb << 32) | Vh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint32_t lo2 = __builtin_amdgcn_readfirstlane((uint32_t)p2);
                    const uint32_t hi2 = __builtin_amdgcn_readfirstlane((uint32_t)(p2 >> 32));
                    if ((hi2 ^ (uint32_t)hb) == 3u) {
                        if (t == 0) __hip_atomic_store(w + 2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        finalize_uniform(p, c, st, lo2 ^ Vh, t, true);
                    }
                }
            }
        }
        if (u == 0) unit_status_pair(p, U, true, t);
    }
    // fused shard-index checks under the pair tables (A_4096: the pair kernel's kthread11)
    for (uint32_t j = g; j < p.n_idx; j += G) verify_index_pair(p, j, t, kix, s_tab, s_red[1], j == g, ipre);
}

// production (round 6) for launches of at most kIlwMaxUnits units while
// fewer chunks than CUs are in flight: LB (the look-back finalizer) with the
// AFF form for ZHIP_DF_WHOLE launches; the tuning build adds the returning
// publication (arm 41) and LB without AFF (arm 59)
KernelFn select_ilh_kernel(int item, bool swap, bool lb, bool aff) {  // CRC chains only
#if ZHIP_TUNING
#define ZHIP_ILH(I, W) (!lb ? k_decode_ilh<I, W> : aff ? k_decode_ilh<I, W, true, true> : k_decode_ilh<I, W, true>)
#else
    if (!lb) return nullptr;
#define ZHIP_ILH(I, W) (aff ? k_decode_ilh<I, W, true, true> : k_decode_ilh<I, W, true>)
#endif
    switch (item) {
        case 1: return ZHIP_ILH(1, false);
        case 2: return swap ? ZHIP_ILH(2, true) : ZHIP_ILH(2, false);
        case 4: return swap ? ZHIP_ILH(4, true) : ZHIP_ILH(4, false);
        case 8: return swap ? ZHIP_ILH(8, true) : ZHIP_ILH(8, false);
        default: return nullptr;
    }
#undef ZHIP_ILH
}

// ---------------------------------------------------------------------------
// k_decode_ilw: small shares (below ~2 workgroups per CU: the N = 4 / 8 shares
// of the strong-scaled headline).  k_decode_il there runs ONE 4-wave
// workgroup per CU, each lane's eight Horner steps in series with nothing to
// interleave (stamps at the N = 8 share, profiles/r05/d/: 2.0 us from tables
// to the last stored block, 0.7 us run end).  Here a 32 KiB unit is taken by
// NT = 512 or 1024 lanes, 2048 / NT blocks each (lane t: the blocks at 16 t +
// 16 NT k of the unit), so a CU holds 8 or 16 waves whose chains interleave,
// under the tables of A_(16 NT); the 4 KiB sub-step of block k is 8 r + t /
// 256 + (NT / 256) k, so stores, row map and lane offsets are k_decode_il's
// per sub-step.  Lane constants F(r) G(t) from capi.cpp (off_ilw).
template <int NT>
__device__ __forceinline__ void lanemul3_init_w(uint32_t* s_mul, int t, uint32_t k) {
    const uint32_t k1 = mulx1(k), k2 = mulx1(k1);
#pragma unroll
    for (uint32_t v = 0; v < 8; ++v)
        s_mul[v * NT + t] = ((v & 4u) ? k : 0u) ^ ((v & 2u) ? k1 : 0u) ^ ((v & 1u) ? k2 : 0u);
#pragma unroll
    for (uint32_t v = 0; v < 4; ++v) s_mul[(8u + v) * NT + t] = ((v & 2u) ? k : 0u) ^ ((v & 1u) ? k1 : 0u);
}

template <int NT>
__device__ __forceinline__ uint32_t lanemul3_w(const uint32_t* s_mul, int t, uint32_t a) {
    uint32_t m[11];
#pragma unroll
    for (int j = 0; j < 10; ++j) m[j] = s_mul[((a >> (3 * j)) & 7u) * NT + t];
    m[10] = s_mul[(8u + (a >> 30)) * NT + t];
    uint32_t q = m[0];
#pragma unroll
    for (int j = 1; j < 10; ++j) q = (q >> 3) ^ r3(q & 7u) ^ m[j];
    return (q >> 2) ^ r2(q & 3u) ^ m[10];
}

// LMR: the lane multiply in registers (lanemul_reg, VALU) instead of the LDS
// column: the run end's LDS reads halve.  MIX (tuning arm 42): the waves of
// the second 256 lanes multiply in registers, the first through the LDS
// column, so the run end's lookups and VALU work overlap.
template <int ITEM, bool SWAP, int NT, bool LMR = false, bool MIX = false, bool AFF = false, bool SPL = false,
          bool LB = false>
__global__ __launch_bounds__(NT) void k_decode_ilw(const DecodeParams p) {
    constexpr int KW = 2048 / NT;  // blocks per lane
    constexpr int QW = NT / 256;   // 4 KiB sub-steps per row of lanes
    constexpr int TV = (kPairTabWords / 4 + NT - 1) / NT;
    __shared__ uint32_t s_tab[kPairTabWords];
    __shared__ uint32_t s_mul[LMR ? 1 : 12 * NT];
    __shared__ uint32_t s_red[2][NT / 64];
    const int t = threadIdx.x;
    const uint32_t G = gridDim.x, g = blockIdx.x;
    const uint32_t wpc = p.nseg;
    const uint32_t c = g / wpc, r = g - c * wpc;
    const bool has = c < p.n_chunks;
    if (!has && g >= p.n_idx) return;
    stamp(p, g, t, 0);
    const uint32_t expected = p.g.nbytes + 4u;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_rows_zero);
    // 1. tables, lane constants, then (header chain) the data
    uint4 tv[TV];
    const uint4* gt = reinterpret_cast<const uint4*>(p.ilw_tab);
#pragma unroll
    for (int i = 0; i < TV; ++i) {
        const int ix = t + i * NT;
        tv[i] = ix < kPairTabWords / 4 ? gt[ix] : make_uint4(0, 0, 0, 0);
    }
    const uint32_t kl = load_u32_any(reinterpret_cast<const uint8_t*>(p.ilw_klane + (size_t)(has ? r : 0u) * NT + t));
    const uint32_t kix = load_u32_any(reinterpret_cast<const uint8_t*>(p.ilw_kidx + (t & (kThreads - 1))));
    Unit U;
    if (has) U = resolve_unit(p, c * p.nseg, expected);
    else {
        U.c = 0;
        U.sidx = 0;
        U.mode = ZHIP_ST_MISSING;
        U.cp = zero;
        U.seg_lo = 0;
        U.sel = 0;
        U.out_off = 0;
    }
    const bool ok = has && U.mode == ZHIP_ST_OK;
    const int32_t lo_frame = (int32_t)p.E - (int32_t)(p.nseg * p.seg);
    const uint32_t q = __builtin_amdgcn_readfirstlane((uint32_t)t >> 8);  // wave-uniform
    const uint32_t l = (uint32_t)t & 255u;
    const uint4 ipre = index_prefetch(p, g, g < p.n_idx && t < kThreads, t, zero);
    uint4 A[KW];
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        const int32_t base = lo_frame + kWgStride * (int32_t)(8u * r + q + (uint32_t)(QW * k));
        A[k] = load_stream16_any(ok && base >= 0 ? U.cp + base + 16 * l : zero);
    }
    stamp(p, g, t, 1);
    zhip_rowblk m[KW];
    const uint32_t sidx = p.nseg - 1u - r;
    if (AFF && (!has || sel_whole(p, U.sel))) {  // (k_decode_il's AFF, checked by sel_whole)
#pragma unroll
        for (int k = 0; k < KW; ++k) m[k] = aff_rowblk(p, 8u * r + q + (uint32_t)(QW * k));
    } else {
#pragma unroll
        for (int k = 0; k < KW; ++k)
            m[k] = load_uniform<zhip_rowblk>(p.rowmap + ((size_t)U.sel * p.nseg + sidx) * kDefaultBlocks + q +
                                             (uint32_t)(QW * k));
    }
    uint32_t stored = 0;
    if (ok) stored = load_trailer_uniform(U.cp, p.g.nbytes);
    // 2. tables into LDS, the lane-multiply column
    {
        uint4* stt = reinterpret_cast<uint4*>(s_tab);
#pragma unroll
        for (int i = 0; i < TV; ++i) {
            const int ix = t + i * NT;
            if (ix < kPairTabWords / 4) stt[ix] = tv[i];
        }
        if constexpr (!LMR) {
            if (!MIX || t < kThreads) lanemul3_init_w<NT>(s_mul, t, kl);
        }
    }
    __syncthreads();
    stamp(p, g, t, 2);
    if (has) {
        // 3. stores, each block's Horner step after its store
        uint8_t* sink = reinterpret_cast<uint8_t*>(g_rows_sink);
        const uint32_t lane_row = (16u * l) >> p.row_shift;
        const uint32_t lane_col = (16u * l) & ((1u << p.row_shift) - 1u);
        const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)lane_col;
        const bool writes = ok || U.mode == ZHIP_ST_MISSING;
        uint8_t* const obase = p.out + U.out_off;
        const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
        Acc4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            const uint32_t lo = m[k].lo, hi = m[k].hi;
            const bool wr = writes && lane_row - lo < hi - lo;
            store_nt16(wr ? obase + m[k].rel + lane_off : sink, ok ? swap_block<ITEM, SWAP>(A[k]) : f);
            if (ok) crc_block4(s_tab, acc, A[k]);
        }
        stamp(p, g, t, 3);
        // 4. run end: one chain per workgroup, one publication
        uint32_t v = 0;
        if (ok) {
            const uint32_t fo = fold4(s_tab, acc);
            if (LMR || (MIX && t >= kThreads)) v = lanemul_reg(kl, fo);  // (wave-uniform choice)
            else v = lanemul3_w<NT>(s_mul, t, fo);
        }
        v = wave_xor(v);
        if ((t & 63) == 0) s_red[0][t >> 6] = v;
        __syncthreads();
        if (ok && t < 64) {
            uint32_t x = 0;
#pragma unroll
            for (int w = 0; w < NT / 64; ++w) x ^= s_red[0][w];
            const uint32_t V = __builtin_amdgcn_readfirstlane(x);
            stamp(p, g, t, 4);
            if (SPL && wpc > 16u && wpc <= 32u)  // (tuning arm 49)
                publish_il_split(p, c, r, wpc, V, __builtin_amdgcn_readfirstlane(stored), t);
            else if (LB && wpc <= 64u)  // look-back finalizer (tuning arm 58)
                publish_lb(p, c, r, wpc, V, __builtin_amdgcn_readfirstlane(stored), t, kPubLine / 2u);
            else
                publish_il(p, c, r, wpc, V, __builtin_amdgcn_readfirstlane(stored), t, kPubLine / 2u);
        }
        if (r == 0) unit_status_pair(p, U, true, t);
    }
    stamp(p, g, t, 7);
    // 5. fused shard-index checks (one step per lane, the first 256 lanes)
    for (uint32_t j = g; j < p.n_idx; j += G)
        verify_index_pair(p, j, t, kix, s_tab, s_red[1], j == g, ipre, t < kThreads);
}

// production: 512 lanes, the LDS lane multiply (small grids, launch_decode),
// the AFF form for ZHIP_DF_WHOLE launches; the tuning build adds 1024 lanes
// and the register multiply (513: half the waves, arm 42)
KernelFn select_ilw_kernel(int item, bool swap, int nt, bool lmr, bool aff) {  // CRC chains only
#if ZHIP_TUNING
#define ZHIP_ILW(I, W)                                                                         \
    (nt == 1024 ? (lmr ? k_decode_ilw<I, W, 1024, true> : k_decode_ilw<I, W, 1024>)            \
     : nt == 513 ? k_decode_ilw<I, W, 512, false, true>                                         \
     : nt == 515 ? k_decode_ilw<I, W, 512, false, false, true, true>                            \
     : nt == 516 ? k_decode_ilw<I, W, 512, false, false, true, false, true>                     \
     : lmr       ? k_decode_ilw<I, W, 512, true>                                                \
     : aff       ? k_decode_ilw<I, W, 512, false, false, true>                                  \
                 : k_decode_ilw<I, W, 512>)
#else
    if (nt != 512 || lmr) return nullptr;
#define ZHIP_ILW(I, W) (aff ? k_decode_ilw<I, W, 512, false, false, true> : k_decode_ilw<I, W, 512>)
#endif
    switch (item) {
        case 1: return ZHIP_ILW(1, false);
        case 2: return swap ? ZHIP_ILW(2, true) : ZHIP_ILW(2, false);
        case 4: return swap ? ZHIP_ILW(4, true) : ZHIP_ILW(4, false);
        case 8: return swap ? ZHIP_ILW(8, true) : ZHIP_ILW(8, false);
        default: return nullptr;
    }
#undef ZHIP_ILW
}

#if ZHIP_TUNING
KernelFn select_ilp_kernel(int item, bool swap) {  // CRC chains only
    switch (item) {
        case 1: return k_decode_ilp<1, false>;
        case 2: return swap ? k_decode_ilp<2, true> : k_decode_ilp<2, false>;
        case 4: return swap ? k_decode_ilp<4, true> : k_decode_ilp<4, false>;
        case 8: return swap ? k_decode_ilp<8, true> : k_decode_ilp<8, false>;
        default: return nullptr;
    }
}

KernelFn select_ilc_kernel(int item, bool swap) {  // CRC chains only
    switch (item) {
        case 1: return k_decode_ilc<1, false>;
        case 2: return swap ? k_decode_ilc<2, true> : k_decode_ilc<2, false>;
        case 4: return swap ? k_decode_ilc<4, true> : k_decode_ilc<4, false>;
        case 8: return swap ? k_decode_ilc<8, true> : k_decode_ilc<8, false>;
        default: return nullptr;
    }
}
#endif

#if ZHIP_TUNING
KernelFn select_ilq_kernel(int item, bool swap, int nq, bool glds) {  // CRC chains only
#define ZHIP_ILQ(I, W) \
    (nq == 4 ? (glds ? k_decode_ilq<I, W, 4, true> : k_decode_ilq<I, W, 4, false>) \
             : nq == 2 ? (glds ? k_decode_ilq<I, W, 2, true> : k_decode_ilq<I, W, 2, false>) \
                       : (glds ? k_decode_ilq<I, W, 1, true> : k_decode_ilq<I, W, 1, false>))
    switch (item) {
        case 4: return swap ? ZHIP_ILQ(4, true) : ZHIP_ILQ(4, false);
        default: return nullptr;
    }
#undef ZHIP_ILQ
}
#endif

// ---------------------------------------------------------------------------
// k_decode_xw: the whole-row decode with the four waves of a workgroup on four
// consecutive chunks of the batch (a shard's x-adjacent inner chunks), each
// wave on the same 8 KiB span (r of P = chunk / 8 KiB) of its own chunk: lane
// l's eight blocks at 1 KiB apart, so one wave streams 8 KiB contiguously and
// the workgroup's stores are the four chunks' rows side by side in the out
// (512-byte runs for C4's 128-byte rows).  That access order copies at 0.80 of
// HBM peak on the headline and 0.68-0.69 at C4, where the pair kernel's 32 KiB
// per-lane-strided spans reach 0.75 / 0.63 (scripts/copybench k_scatter_g,
// profiles/r03/xw/).  Per lane one Horner chain through the A_1024 11/11/10
// tables (four word accumulators, A4 fold), one windowed lane multiply by the
// host-built constant of (r, l), one publication per WAVE (no workgroup
// reduction): arrival bit r, two-level for P > 32 (32-bit subwords in the
// workspace tail), xor + count above 1024.  Statuses, row-map stores and the
// fused index checks as k_decode_il.  (CPU emulation: zhip_emulate_chunk_crc_xw.)
__device__ __forceinline__ void publish_xw(const DecodeParams& p, uint32_t c, uint32_t r, uint32_t V,
                                           uint32_t stored, uint32_t l) {
    const uint32_t P = p.xw, ns = p.xw_nsub;
    if (P <= 32u || ns == 0u) {
        publish_il(p, c, r, P, V, stored, (int)l);
        return;
    }
    const uint32_t sg = r >> 5, in_sg = min(32u, P - (sg << 5));
    const uint64_t bit = 1ull << (r & 31u);
    uint64_t* sw = reinterpret_cast<uint64_t*>(p.ws + 4ull * p.n_chunks) + (uint64_t)c * ns + sg;
    uint64_t prev = 0;
    if (l == 0) prev = __hip_atomic_fetch_xor(sw, (bit << 32) | V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)prev);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(prev >> 32));
    const uint64_t full = in_sg >= 32u ? 0xFFFFFFFFull : ((1ull << in_sg) - 1ull);
    if ((uint64_t)(hi ^ (uint32_t)bit) != full) return;
    if (l == 0) __hip_atomic_store(sw, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    publish_il(p, c, sg, ns, V ^ lo, stored, (int)l);
}

template <bool CRC, int ITEM, bool SWAP>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_decode_xw(const DecodeParams p) {
    constexpr int K = kDefaultBlocks;
    __shared__ uint32_t s_tab[CRC ? kPairTabWords : 1];
    __shared__ uint32_t s_mul[CRC ? 12 * kThreads : 1];
    __shared__ uint32_t s_red[kThreads / 64];
    const int t = threadIdx.x;
    const uint32_t l = (uint32_t)t & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane((uint32_t)t >> 6);
    const uint32_t G = gridDim.x, g = blockIdx.x;
    const uint32_t P = p.xw;  // 8 KiB spans per chunk
    const uint32_t quad = g / P, r = g - quad * P;
    if (quad * 4u >= p.n_chunks && g >= p.n_idx) return;  // workgroup-uniform
    const uint32_t c = quad * 4u + wv;
    const bool has = c < p.n_chunks;
    const uint32_t expected = p.g.nbytes + (CRC ? 4u : 0u);
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_rows_zero);
    // 1. vector loads in a path-independent order: [CRC: tables (6), the lane
    //    constant, the index lane constant, the first index block], the K data
    //    blocks; headers, row-map entries and the trailer are scalar (per wave)
    uint4 tv0, tv1, tv2, tv3, tv4, tv5;
    uint32_t kl = 0, kix = 0;
    if constexpr (CRC) {
        const uint4* gt = reinterpret_cast<const uint4*>(p.xw_tab);
        tv0 = gt[t];
        tv1 = gt[t + kThreads];
        tv2 = gt[t + 2 * kThreads];
        tv3 = gt[t + 3 * kThreads];
        tv4 = gt[t + 4 * kThreads];
        tv5 = gt[t + 5 * kThreads];
        kl = load_u32_any(reinterpret_cast<const uint8_t*>(p.xw_klane + (size_t)r * 64u + l));
        kix = load_u32_any(reinterpret_cast<const uint8_t*>(p.xw_kidx + t));
    }
    Unit U;
    if (has) U = resolve_unit(p, c * p.nseg, expected);
    else {
        U.c = 0;
        U.sidx = 0;
        U.mode = ZHIP_ST_MISSING;
        U.cp = zero;
        U.seg_lo = 0;
        U.sel = 0;
        U.out_off = 0;
    }
    const bool ok = has && U.mode == ZHIP_ST_OK;
    const int32_t lo_frame = (int32_t)p.E - (int32_t)(p.nseg * p.seg);  // a multiple of 4096 (whole rows)
    uint4 ipre = make_uint4(0, 0, 0, 0);
    if constexpr (CRC) ipre = index_prefetch(p, g, g < p.n_idx, t, zero);
    uint4 A[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int32_t base = lo_frame + 8192 * (int32_t)r + 1024 * k;
        A[k] = load_stream16_any(ok && base >= 0 ? U.cp + base + 16 * l : zero);
    }
    // destinations of the span's two 4 KiB steps (scalar loads)
    zhip_rowblk m[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t st = 2u * r + (uint32_t)h;
        const uint32_t sidx = p.nseg - 1u - st / (uint32_t)K;
        m[h] = load_uniform<zhip_rowblk>(p.rowmap + ((size_t)U.sel * p.nseg + sidx) * K + (st % (uint32_t)K));
    }
    uint32_t stored = 0;
    if (CRC && ok) stored = load_trailer_uniform(U.cp, p.g.nbytes);
    // 2. tables into LDS, the lane-multiply column
    if constexpr (CRC) {
        uint4* stt = reinterpret_cast<uint4*>(s_tab);
        stt[t] = tv0;
        stt[t + kThreads] = tv1;
        stt[t + 2 * kThreads] = tv2;
        stt[t + 3 * kThreads] = tv3;
        stt[t + 4 * kThreads] = tv4;
        stt[t + 5 * kThreads] = tv5;
        lanemul3_init(s_mul, t, kl);
        __syncthreads();
    }
    if (has) {
        // 3. stores, each block's Horner step after its store
        uint8_t* sink = reinterpret_cast<uint8_t*>(g_rows_sink);
        const bool writes = ok || U.mode == ZHIP_ST_MISSING;
        uint8_t* const obase = p.out + U.out_off;
        const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
        const uint32_t rmask = (1u << p.row_shift) - 1u;
        Acc4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const zhip_rowblk& mk = m[k >> 2];
            const uint32_t o = 1024u * (uint32_t)(k & 3) + 16u * l;  // byte in the 4 KiB step
            const uint32_t lane_row = o >> p.row_shift;
            const bool wr = writes && lane_row - mk.lo < mk.hi - mk.lo;
            const int64_t lane_off = (int64_t)lane_row * p.r_oy + (int64_t)(o & rmask);
            store_nt16(wr ? obase + mk.rel + lane_off : sink, ok ? swap_block<ITEM, SWAP>(A[k]) : f);
            if (CRC && ok) crc_block4(s_tab, acc, A[k]);
        }
        // 4. run end: one chain per lane, one publication per wave
        if constexpr (CRC) {
            uint32_t v = ok ? lanemul3(s_mul, t, fold4(s_tab, acc)) : 0u;
            v = wave_xor(v);
            if (ok && !(p.tune & kTuneNoPub))
                publish_xw(p, c, r, __builtin_amdgcn_readfirstlane(v), __builtin_amdgcn_readfirstlane(stored), l);
        }
        if (r == 0) unit_status_pair(p, U, CRC, (int)l);
    }
    // 5. fused shard-index checks (one step per lane), the first block prefetched
    if constexpr (CRC)
        for (uint32_t j = g; j < p.n_idx; j += G) verify_index_pair(p, j, t, kix, s_tab, s_red, j == g, ipre);
}

#if ZHIP_TUNING
KernelFn select_xw_kernel(bool crc, int item, bool swap) {
    if (!crc) return nullptr;
    switch (item) {
        case 1: return k_decode_xw<true, 1, false>;
        case 2: return swap ? k_decode_xw<true, 2, true> : k_decode_xw<true, 2, false>;
        case 4: return swap ? k_decode_xw<true, 4, true> : k_decode_xw<true, 4, false>;
        case 8: return swap ? k_decode_xw<true, 8, true> : k_decode_xw<true, 8, false>;
        default: return nullptr;
    }
}
#endif

KernelFn select_duo_kernel(bool crc, int item, bool swap) {
    switch (item) {
        case 1: return crc ? k_decode_duo<true, 1, false> : k_decode_duo<false, 1, false>;
        case 2: return crc ? (swap ? k_decode_duo<true, 2, true> : k_decode_duo<true, 2, false>)
                           : (swap ? k_decode_duo<false, 2, true> : k_decode_duo<false, 2, false>);
        case 4: return crc ? (swap ? k_decode_duo<true, 4, true> : k_decode_duo<true, 4, false>)
                           : (swap ? k_decode_duo<false, 4, true> : k_decode_duo<false, 4, false>);
        case 8: return crc ? (swap ? k_decode_duo<true, 8, true> : k_decode_duo<true, 8, false>)
                           : (swap ? k_decode_duo<false, 8, true> : k_decode_duo<false, 8, false>);
        default: return nullptr;
    }
}

KernelFn select_rows_kernel(bool crc, int item, bool swap, int k) {
#if ZHIP_TUNING
    if (k == 4) {  // 16 KiB units (tuning arm)
        if (crc && item == 4 && !swap) return k_decode_rows<true, 4, false, 4>;
        return nullptr;
    }
#endif
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
