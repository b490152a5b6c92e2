// Fused zarr v3 decode for MI355X (gfx950): shard sub-chunk resolution,
// CRC-32C verify, bytes-codec byteswap and scatter into the selection of a
// device-resident N-d output — one read of every encoded byte, one write of
// every selected decoded byte.
//
// Reference behaviour restated (file:line under /root/reference):
//   Crc32cCodec._decode_sync        src/zarr/codecs/crc32c_.py:34-50
//   BytesCodec._decode_sync         src/zarr/codecs/bytes.py:97-131
//   TransposeCodec._decode_sync     src/zarr/codecs/transpose.py:98-104 (folded into
//                                   the stored-dim -> out-stride map by the planner)
//   decode_and_scatter_chunk        src/zarr/core/chunk_utils.py:193-214
//   scatter_chunk (missing -> fill) src/zarr/core/chunk_utils.py:88-112
//   _ShardIndex.get_chunk_slice     src/zarr/codecs/sharding.py:248-254 (MAX_UINT_64 -> missing)
//
// Work decomposition.  A chunk's decoded payload [0, N) is cut into "units" of
// seg = 4 KiB * K (K = 8 by default: 32 KiB), aligned to E = align16(N) from the END
// (unit s covers [E-(s+1)seg, E-s*seg)); bytes outside [0, N) are zero.  One 256-thread
// workgroup handles one unit: thread t owns the 16-byte blocks at
// lo + 16t + 4096k, k < 8 (each wave instruction reads 1 KiB contiguous).
//
// CRC.  Each thread keeps a Horner accumulator positioned at the start of its
// next block: acc' = A4096(acc ^ w0) ^ A4092(w1) ^ A4088(w2) ^ A4084(w3), each
// A_k a 32x32 GF(2) operator applied as 4 byte-indexed lookups in LDS
// (16 KiB of tables, host-built).  At the end thread t's value is shifted by a
// per-thread constant to a common point, xor-reduced over the workgroup,
// shifted to the chunk reference R = E + 4096 by a per-unit constant and
// atomically xor-ed into a per-chunk word.  The last unit of a chunk to arrive
// (agent-scope ticket) converts the accumulator into the CRC-32C value, compares
// it with the stored little-endian trailer and writes the chunk status.  Zero
// bytes before the chunk contribute nothing, so no unit needs to know another's
// data: the combine is pure XOR, order-independent and bitwise reproducible.
#include <hip/hip_runtime.h>

#include "../../include/zarrhip.h"
#include "zhip_gf2.h"
#include "zhip_internal.h"
#include "zhip_device.h"
#include "zhip_decode_common.h"

namespace zhip {

#if ZHIP_TUNING
int g_tune_max_grid = 0;
#endif

// Work assignment: unit "positions" q are numbered chunk-major in INCREASING
// address order (q = c*nseg + nseg-1-sidx) and every workgroup takes one
// contiguous, balanced range of them.  Consecutive units of one chunk then
// continue the same per-thread Horner chain (stride 4096 B), so a workgroup
// reduces, shifts and publishes once per (chunk, run), not once per unit.
template <bool CRC, bool WRITE, bool FAST, int ITEM, bool SWAP, int K = 8>
__global__ __launch_bounds__(kThreads) void k_decode(const DecodeParams p) {
    __shared__ uint32_t s_tab[CRC ? 16 * 256 : 1];
    __shared__ uint32_t s_red[2][kThreads / 64];
    const int t = threadIdx.x;
    uint32_t kth = 0;
    const bool crc_on = CRC && !(p.tune & kTuneSkipCrc);
    if constexpr (CRC) {
        const uint4* g = reinterpret_cast<const uint4*>(p.horner);
        uint4* sv = reinterpret_cast<uint4*>(s_tab);
        for (int i = t; i < 1024; i += kThreads) sv[i] = g[i];
        kth = p.kthread[t];
    }
    const uint32_t expected = p.g.nbytes + (CRC ? 4u : 0u);
    // one 64-bit arrival word per chunk: high half = bitmask of arrived units, low = xor
    const bool one_atomic = p.nseg <= 32 && !(p.tune & (kTuneAcqRel | kTuneNoTicket));
    const uint64_t full = p.nseg >= 32 ? 0xFFFFFFFFull : ((1ull << p.nseg) - 1ull);
    Pending pend;
    pend.valid = 0;

    const uint32_t G = gridDim.x, g = blockIdx.x;
    const uint32_t per = p.n_units / G, rem = p.n_units % G;
    const uint32_t q0 = g * per + (g < rem ? g : rem);
    const uint32_t q1 = q0 + per + (g < rem ? 1u : 0u);
    if (q0 >= q1 && g >= p.n_idx) return;
    uint4 A[K], B[K];
    auto unit_of = [&](uint32_t q) {
        const uint32_t c = q / p.nseg;
        return c * p.nseg + (p.nseg - 1u - (q - c * p.nseg));
    };
    Unit ua;
    uint32_t stored = 0;
    if (q0 < q1) {
        ua = resolve_unit(p, unit_of(q0), expected);
        load_unit<K>(p, ua, t, A);
        if (CRC && t == 0 && ua.mode == ZHIP_ST_OK) stored = load_trailer(ua.cp, p.g.nbytes);
    }
    if constexpr (CRC) {
        __syncthreads();  // tables in LDS
        // fused shard-index checks (_decode_shard_index_sync, sharding.py:624-631):
        // workgroup g verifies indexes g, g+G, ... while its first unit's loads fly
        for (uint32_t j = g; j < p.n_idx; j += G) verify_index(p, j, t, kth, s_tab, s_red[1]);
    }
    if (q0 >= q1) return;
    uint32_t acc = 0, run_bits = 0, run_len = 0, parity = 0;
    for (uint32_t q = q0;;) {
        // software pipeline: issue the next unit's loads before working on this one
        const uint32_t qn = q + 1;
        const bool more = qn < q1;
        Unit ub;
        if (more) {
            ub = resolve_unit(p, unit_of(qn), expected);
            load_unit<K>(p, ub, t, B);
        }
        const bool run_end = !more || ub.c != ua.c;
        const zhip_sel& sel = p.sels[ua.sel];
        if (ua.mode == ZHIP_ST_OK) {
            // stores first: they do not depend on the CRC, and starting the write
            // stream early interleaves it with the read stream of later units
            if constexpr (WRITE) {
                if (FAST && (p.tune & kTuneNT)) {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const int32_t o = ua.seg_lo + kWgStride * k + 16 * t;
                        if (o < 0 || (uint32_t)o >= p.g.nbytes) continue;
                        scatter_block_rows<ITEM, SWAP, true>(p.g, p.out, sel, ua.out_off, o, A[k]);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const int32_t o = ua.seg_lo + kWgStride * k + 16 * t;
                        if (o < 0 || (uint32_t)o >= p.g.nbytes) continue;
                        if constexpr (FAST) scatter_block_rows<ITEM, SWAP>(p.g, p.out, sel, ua.out_off, o, A[k]);
                        else scatter_block_generic<ITEM, SWAP>(p.g, p.out, sel, ua.out_off, o, A[k]);
                    }
                }
            }
            if (crc_on) {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const uint4 v = A[k];
                    acc = tab_apply(s_tab, acc ^ v.x) ^ tab_apply(s_tab + 1024, v.y) ^
                          tab_apply(s_tab + 2048, v.z) ^ tab_apply(s_tab + 3072, v.w);
                }
            } else if constexpr (CRC) {
#pragma unroll
                for (int k = 0; k < K; ++k) acc ^= A[k].x ^ A[k].y ^ A[k].z ^ A[k].w;
            }
            run_bits |= 1u << (ua.sidx & 31u);
            ++run_len;
            if constexpr (CRC) {
                if (run_end) {
                    uint32_t v = crc_on ? gf_mul(acc, kth) : acc;
                    v = wave_xor(v);
                    if ((t & 63) == 0) s_red[parity][t >> 6] = v;
                    __syncthreads();
                    if (t == 0) {
                        uint32_t V = s_red[parity][0] ^ s_red[parity][1] ^ s_red[parity][2] ^
                                     s_red[parity][3];
                        V = gf_mul(V, p.kunit[ua.sidx]);
                        if (one_atomic) {
                            retire(p, pend, full);  // the previous run's arrival has returned by now
                            uint64_t* w = reinterpret_cast<uint64_t*>(p.ws) + 2ull * ua.c;
                            pend.prev = __hip_atomic_fetch_xor(w, ((uint64_t)run_bits << 32) | V,
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            pend.stored = stored;
                            pend.c = ua.c;
                            pend.bits = run_bits;
                            pend.V = V;
                            pend.valid = 1;
                        } else {
                            uint32_t* accw = p.ws + 4ull * ua.c;
                            uint32_t tk;
                            if (p.tune & kTuneAcqRel) {
                                __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                tk = __hip_atomic_fetch_add(accw + 2, run_len, __ATOMIC_ACQ_REL,
                                                            __HIP_MEMORY_SCOPE_AGENT);
                            } else {
                                // the xor must be performed at the device-coherent point
                                // before the count is drawn: wait for its return first
                                const uint32_t prev = __hip_atomic_fetch_xor(accw, V, __ATOMIC_RELAXED,
                                                                             __HIP_MEMORY_SCOPE_AGENT);
                                asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
                                tk = (p.tune & kTuneNoTicket)
                                         ? 0u
                                         : __hip_atomic_fetch_add(accw + 2, run_len, __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT);
                            }
                            if (tk + run_len == p.nseg && !(p.tune & kTuneNoTicket)) {
                                const uint32_t raw =
                                    __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                finalize_chunk(p, ua.c, stored, raw);
                            }
                        }
                    }
                    parity ^= 1u;
                    acc = 0;
                    run_bits = 0;
                    run_len = 0;
                }
            } else {
                if (ua.sidx == 0 && t == 0) {
                    zhip_status st = {ZHIP_ST_OK, 0u, 0u, 0u};
                    p.status[ua.c] = st;
                }
            }
        } else {
            if constexpr (WRITE) {
                if (ua.mode == ZHIP_ST_MISSING) {
                    const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const int32_t o = ua.seg_lo + kWgStride * k + 16 * t;
                        if (o < 0 || (uint32_t)o >= p.g.nbytes) continue;
                        if constexpr (FAST) scatter_block_rows<ITEM, false>(p.g, p.out, sel, ua.out_off, o, f);
                        else scatter_block_generic<ITEM, false>(p.g, p.out, sel, ua.out_off, o, f);
                    }
                }
            }
            if (ua.sidx == 0 && t == 0) {
                zhip_status st = {ua.mode, 0u, 0u, 0u};
                p.status[ua.c] = st;
                if (ua.mode != ZHIP_ST_MISSING) atomicOr(p.errflag, 1u << ua.mode);
            }
        }
        if (!more) break;
        if (CRC && t == 0 && ub.c != ua.c && ub.mode == ZHIP_ST_OK) stored = load_trailer(ub.cp, p.g.nbytes);
        q = qn;
        ua = ub;
#pragma unroll
        for (int k = 0; k < K; ++k) A[k] = B[k];
    }
    if (t == 0) retire(p, pend, full);
}


// ---------------------------------------------------------------------------
// Tiled transpose decode (TransposeCodec._decode_sync, transpose.py:98-104, for
// orders whose out-contiguous dim is not the innermost stored dim).  A tile =
// kTileRows rows of the stored dim tq (contiguous in out) x kTileCols bytes of
// the innermost stored row, other dims fixed.  Loads: 16 rows x 256 B per pass
// (every wave reads whole 256-byte row pieces); the tile is transposed through
// LDS and stored as whole out rows (256 B contiguous per column element).
// CRC: thread t's blocks sit at a constant stride 16*sstride[tq], so it keeps
// a Horner chain with stride-specific tables; per-thread / per-tile shift
// constants (host-built) bring every tile's contribution to the chunk reference.
// ---------------------------------------------------------------------------
template <bool CRC, int ITEM, bool SWAP>
__global__ __launch_bounds__(kThreads) void k_decode_tile(const DecodeParams p) {
    constexpr int kPitch = ITEM == 8 ? 264 : 260;  // bytes per LDS tile row (2-way read conflicts)
    constexpr int kPasses = kTileRows / 16;
    __shared__ uint32_t s_tab[CRC ? 16 * 256 : 1];
    __shared__ __attribute__((aligned(16))) uint8_t s_tile[kTileRows * kPitch];
    __shared__ uint32_t s_red[kThreads / 64];
    const int t = threadIdx.x;
    uint32_t kth = 0;
    if constexpr (CRC) {
        const uint4* g = reinterpret_cast<const uint4*>(p.horner);
        uint4* sv = reinterpret_cast<uint4*>(s_tab);
        for (int i = t; i < 1024; i += kThreads) sv[i] = g[i];
        kth = p.kthread[t];
        __syncthreads();
    }
    const uint32_t expected = p.g.nbytes + (CRC ? 4u : 0u);
    const int32_t last = p.g.ndim - 1;
    const uint32_t rows_q = (uint32_t)p.g.shape[p.tq];
    const uint32_t sq = p.sstride[p.tq];
    const int64_t oq = p.g.ostride[p.tq];      // == ITEM
    const int64_t ocol = p.g.ostride[last];    // out stride of the innermost stored dim
    const uint32_t G = gridDim.x, gi = blockIdx.x;
    const uint32_t per = p.n_units / G, rem = p.n_units % G;
    const uint32_t q0 = gi * per + (gi < rem ? gi : rem);
    const uint32_t q1 = q0 + per + (gi < rem ? 1u : 0u);
    uint32_t runV = 0, run_len = 0;
    for (uint32_t q = q0; q < q1; ++q) {
        const uint32_t c = q / p.t_per_chunk;
        const uint32_t ti = q - c * p.t_per_chunk;
        // chunk source (as resolve_unit)
        const zhip_chunk ch = p.chunks[c];
        uint32_t mode = ZHIP_ST_OK;
        uint64_t base = ch.src;
        if (ch.flags & ZHIP_CF_MISSING) {
            mode = ZHIP_ST_MISSING;
        } else if (p.lflags & ZHIP_LF_SHARDED) {
            const uint64_t ipos = (p.lflags & ZHIP_LF_INDEX_START) ? 0ull : ch.src_len - p.index_size;
            const uint8_t* e = p.src + ch.src + ipos + 16ull * ch.slot;
            const uint64_t off = load_u64_le_bytes(e);
            const uint64_t len = load_u64_le_bytes(e + 8);
            if (off == ~0ull && len == ~0ull) mode = ZHIP_ST_MISSING;
            else if (off > ch.src_len || len > ch.src_len - off) mode = ZHIP_ST_INDEX_OOB;
            else if (len != expected) mode = ZHIP_ST_LENGTH_MISMATCH;
            else base = ch.src + off;
        } else if (ch.src_len != expected) {
            mode = ZHIP_ST_LENGTH_MISMATCH;
        }
        mode = __builtin_amdgcn_readfirstlane(mode);
        const uint8_t* cp = p.src + base;
        // tile coordinates
        uint32_t r = ti;
        const uint32_t rq = fdiv_apply(r, p.d_cb.m, p.d_cb.s);
        const uint32_t cb = r - rq * p.n_cb;
        r = rq;
        const uint32_t rr = fdiv_apply(r, p.d_qb.m, p.d_qb.s);
        const uint32_t qb = r - rr * p.n_qb;
        r = rr;
        uint32_t tbase = qb * (uint32_t)kTileRows * sq + cb * (uint32_t)kTileCols;
        int64_t obase = ch.out_off + (int64_t)qb * kTileRows * oq + (int64_t)(cb * (kTileCols / ITEM)) * ocol;
#pragma unroll
        for (int d = ZHIP_MAX_DIMS - 1; d >= 0; --d) {
            if (d >= last || d == p.tq) continue;
            const uint32_t qd = fdiv_apply(r, p.g.dshape[d].m, p.g.dshape[d].s);
            const uint32_t sd = r - qd * (uint32_t)p.g.shape[d];
            r = qd;
            tbase += sd * p.sstride[d];
            obase += (int64_t)sd * p.g.ostride[d];
        }
        const uint32_t rows_here = min((uint32_t)kTileRows, rows_q - qb * kTileRows);
        const uint32_t cols_here = min((uint32_t)kTileCols, p.g.row_bytes - cb * kTileCols);
        if (mode == ZHIP_ST_OK) {
            const int row0 = t >> 4;
            const uint32_t col = 16u * (uint32_t)(t & 15);
            uint4 blk[kPasses];
            const uint32_t al4 =
                __builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<uintptr_t>(cp) & 3u) == 0u ? 1u : 0u);
            if (al4) {
#pragma unroll
                for (int k = 0; k < kPasses; ++k) {
                    const uint32_t row = 16u * k + row0;
                    blk[k] = (row < rows_here && col < cols_here)
                                 ? *reinterpret_cast<const uint4*>(cp + tbase + row * sq + col)
                                 : make_uint4(0, 0, 0, 0);
                }
            } else {
#pragma unroll
                for (int k = 0; k < kPasses; ++k) {
                    const uint32_t row = 16u * k + row0;
                    blk[k] = (row < rows_here && col < cols_here)
                                 ? load_block<false>(cp, (int32_t)(tbase + row * sq + col), p.g.nbytes)
                                 : make_uint4(0, 0, 0, 0);
                }
            }
            uint32_t acc = 0;
            if constexpr (CRC) {
#pragma unroll
                for (int k = 0; k < kPasses; ++k) {
                    const uint4 v = blk[k];
                    acc = tab_apply(s_tab, acc ^ v.x) ^ tab_apply(s_tab + 1024, v.y) ^
                          tab_apply(s_tab + 2048, v.z) ^ tab_apply(s_tab + 3072, v.w);
                }
            }
#pragma unroll
            for (int k = 0; k < kPasses; ++k) {
                const uint4 v = swap_block<ITEM, SWAP>(blk[k]);
                uint32_t* d = reinterpret_cast<uint32_t*>(s_tile + (16 * k + row0) * kPitch + col);
                d[0] = v.x;
                d[1] = v.y;
                d[2] = v.z;
                d[3] = v.w;
            }
            __syncthreads();
            // out pieces: column element j, 16/ITEM consecutive rows from q0
            constexpr int kPer = 16 / ITEM;                  // rows per 16-byte piece
            constexpr int kPiecesPerCol = kTileRows / kPer;  // pieces per out row
#pragma unroll
            for (int k = 0; k < kPasses; ++k) {
                const uint32_t pc = (uint32_t)(k * kThreads + t);
                const uint32_t j = pc / kPiecesPerCol;
                const uint32_t r0 = (pc % kPiecesPerCol) * kPer;
                if (j * ITEM >= cols_here || r0 >= rows_here) continue;
                uint32_t w[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) w[e] = 0;
#pragma unroll
                for (int e = 0; e < kPer; ++e) {
                    const uint8_t* src = s_tile + (r0 + e) * kPitch + j * ITEM;
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
                uint8_t* dst = p.out + obase + (int64_t)j * ocol + (int64_t)r0 * oq;
                if (r0 + kPer <= rows_here) {
                    *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
                } else {
                    for (uint32_t e = 0; e < rows_here - r0; ++e)
                        for (int b = 0; b < ITEM; ++b)
                            dst[e * ITEM + b] = (uint8_t)(w[(e * ITEM + b) / 4] >> (8 * ((e * ITEM + b) % 4)));
                }
            }
            if constexpr (CRC) {
                uint32_t v = gf_mul(acc, kth);
                v = wave_xor(v);
                if ((t & 63) == 0) s_red[t >> 6] = v;
            }
            __syncthreads();  // LDS tile and s_red reads done before the next tile
            if constexpr (CRC) {
                if (t == 0) {
                    const uint32_t V = s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3];
                    runV ^= gf_mul(V, p.kunit[ti]);
                    ++run_len;
                    const bool run_end = (q + 1 >= q1) || ((q + 1) / p.t_per_chunk != c);
                    if (run_end) {
                        uint32_t* accw = p.ws + 4ull * c;
                        const uint32_t prev =
                            __hip_atomic_fetch_xor(accw, runV, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        asm volatile("s_waitcnt vmcnt(0)" ::"v"(prev) : "memory");
                        const uint32_t tk =
                            __hip_atomic_fetch_add(accw + 2, run_len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (tk + run_len == p.t_per_chunk) {
                            const uint32_t raw =
                                __hip_atomic_exchange(accw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            __hip_atomic_store(accw + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            finalize_chunk(p, c, load_trailer(cp, p.g.nbytes), raw);
                        }
                        runV = 0;
                        run_len = 0;
                    }
                }
            } else if (t == 0 && ti == 0) {
                zhip_status st = {ZHIP_ST_OK, 0u, 0u, 0u};
                p.status[c] = st;
            }
        } else {
            // missing chunk: fill this tile's region of out
            const uint4 f = make_uint4(p.fill[0], p.fill[1], p.fill[2], p.fill[3]);
            constexpr int kPer = 16 / ITEM;
            constexpr int kPiecesPerCol = kTileRows / kPer;
            if (mode == ZHIP_ST_MISSING) {
#pragma unroll
                for (int k = 0; k < kPasses; ++k) {
                    const uint32_t pc = (uint32_t)(k * kThreads + t);
                    const uint32_t j = pc / kPiecesPerCol;
                    const uint32_t r0 = (pc % kPiecesPerCol) * kPer;
                    if (j * ITEM >= cols_here || r0 >= rows_here) continue;
                    uint8_t* dst = p.out + obase + (int64_t)j * ocol + (int64_t)r0 * oq;
                    if (r0 + kPer <= rows_here) {
                        *reinterpret_cast<uint4*>(dst) = f;
                    } else {
                        const uint32_t fw[4] = {f.x, f.y, f.z, f.w};
                        for (uint32_t e = 0; e < (rows_here - r0) * ITEM; ++e)
                            dst[e] = (uint8_t)(fw[e / 4] >> (8 * (e % 4)));
                    }
                }
            }
            if (t == 0 && ti == 0) {
                zhip_status st = {mode, 0u, 0u, 0u};
                p.status[c] = st;
                if (mode != ZHIP_ST_MISSING) atomicOr(p.errflag, 1u << mode);
            }
        }
    }
}

using KernelFn = void (*)(const DecodeParams);

template <bool CRC, bool WRITE, bool FAST, int K>
static KernelFn pick_item(int item, bool swap) {
    switch (item) {
        case 1: return k_decode<CRC, WRITE, FAST, 1, false, K>;
        case 2: return swap ? k_decode<CRC, WRITE, FAST, 2, true, K> : k_decode<CRC, WRITE, FAST, 2, false, K>;
        case 4: return swap ? k_decode<CRC, WRITE, FAST, 4, true, K> : k_decode<CRC, WRITE, FAST, 4, false, K>;
        case 8: return swap ? k_decode<CRC, WRITE, FAST, 8, true, K> : k_decode<CRC, WRITE, FAST, 8, false, K>;
        default: return nullptr;
    }
}

KernelFn select_decode_kernel(bool crc, bool write, bool fast, int item, bool swap, int k) {
    if (!write) {
        if (!crc) return nullptr;
        return k == 4 ? k_decode<true, false, false, 1, false, 4>
             : k == 16 ? k_decode<true, false, false, 1, false, 16> : k_decode<true, false, false, 1, false, 8>;
    }
    if (crc && fast) {
        return k == 4 ? pick_item<true, true, true, 4>(item, swap)
             : k == 16 ? pick_item<true, true, true, 16>(item, swap) : pick_item<true, true, true, 8>(item, swap);
    }
    if (k != 8) return nullptr;
    if (crc) return pick_item<true, true, false, 8>(item, swap);
    return fast ? pick_item<false, true, true, 8>(item, swap) : pick_item<false, true, false, 8>(item, swap);
}

static KernelFn select_tile_kernel(bool crc, int item, bool swap) {
    switch (item) {
        case 1: return crc ? k_decode_tile<true, 1, false> : k_decode_tile<false, 1, false>;
        case 2: return crc ? (swap ? k_decode_tile<true, 2, true> : k_decode_tile<true, 2, false>)
                           : (swap ? k_decode_tile<false, 2, true> : k_decode_tile<false, 2, false>);
        case 4: return crc ? (swap ? k_decode_tile<true, 4, true> : k_decode_tile<true, 4, false>)
                           : (swap ? k_decode_tile<false, 4, true> : k_decode_tile<false, 4, false>);
        case 8: return crc ? (swap ? k_decode_tile<true, 8, true> : k_decode_tile<true, 8, false>)
                           : (swap ? k_decode_tile<false, 8, true> : k_decode_tile<false, 8, false>);
        default: return nullptr;
    }
}

KernelFn select_rows_kernel(bool crc, int item, bool swap, int k);  // decode_rows.hip
KernelFn select_pair_kernel(bool crc, int item, bool swap, int nu);  // decode_rows.hip
KernelFn select_duo_kernel(bool crc, int item, bool swap);           // decode_rows.hip
KernelFn select_il_kernel(bool crc, int item, bool swap, bool aff);  // decode_rows.hip
KernelFn select_ilw_kernel(int item, bool swap, int nt, bool lmr, bool aff);  // decode_rows.hip
KernelFn select_ilh_kernel(int item, bool swap, bool lb, bool aff);  // decode_rows.hip
#if ZHIP_TUNING
KernelFn select_il_kernel_lean(bool crc, int item, bool swap);       // decode_rows.hip
KernelFn select_il_kernel_tuned(bool crc, int item, bool swap);      // decode_rows.hip
KernelFn select_il_kernel_arm(bool crc, int item, bool swap, int arm);  // decode_rows.hip
KernelFn select_il_kernel_cf(bool crc, int item, bool swap);         // decode_rows.hip
KernelFn select_il_kernel_regmul(bool crc, int item, bool swap, bool occ6);  // decode_rows.hip
KernelFn select_xw_kernel(bool crc, int item, bool swap);            // decode_rows.hip
KernelFn select_ilq_kernel(int item, bool swap, int nq, bool glds);  // decode_rows.hip
KernelFn select_ilc_kernel(int item, bool swap);                     // decode_rows.hip
KernelFn select_ilp_kernel(int item, bool swap);                     // decode_rows.hip
KernelFn select_tile4f_kernel(int item, bool swap);                  // decode_tile.hip
#endif
KernelFn select_tile4_kernel(bool crc, int item, bool swap);         // decode_tile.hip
KernelFn select_tile4w_kernel(int item, bool swap);                  // decode_tile.hip
KernelFn select_tile2w_kernel(int item, bool swap, int nt);          // decode_tile.hip
KernelFn select_tilegw_kernel(int item, bool swap, bool defer, int nt);  // decode_tile.hip
KernelFn select_tileg_kernel(bool crc, int item, bool swap, bool defer);  // decode_tile.hip

// name of the kernel the last launch_decode chose (zhip_last_kernel: bench
// labels and tests; the selection depends on layout, plan and tuning bits)
const char* g_last_kernel = "";
#if ZHIP_TUNING
// Overhead probes (arms 28-30; results invalid): the launch of a decode-shaped
// grid with the decode's kernel arguments and nothing else (28), plus the
// k_decode_il LDS footprint (29), plus the header chain (resolve_unit) of
// each workgroup's chunk (30).
template <int MODE>
__global__ __launch_bounds__(kThreads) void k_probe(const DecodeParams p) {
    __shared__ uint32_t s_big[MODE >= 1 ? 9216 : 1];
    const uint32_t g = blockIdx.x;
    const int t = threadIdx.x;
    uint32_t v = g;
    if constexpr (MODE >= 1) {
        s_big[(t * 37u + g) % 9216u] = g;
        __syncthreads();
        v ^= s_big[(t * 41u) % 9216u];
    }
    if constexpr (MODE == 2) {
        const uint32_t c = g / p.nseg;
        if (c < p.n_chunks) {
            const Unit U = resolve_unit(p, c * p.nseg, p.g.nbytes + 4u);
            v ^= (uint32_t)U.out_off ^ (uint32_t)(uintptr_t)U.cp ^ U.mode;
        }
    }
    if (v == 0xFFFFFFFFu && t == 1000) p.errflag[0] = v;  // never: keeps the work live
}
#endif


int launch_decode(const DecodeParams& p, hipStream_t stream, int max_grid) {
    // the look-back finalizer (publish_lb) waits only while fewer chunks than
    // CUs are in the launch (max_grid arrives as CUs * 8)
    const bool lb_ok = p.n_chunks < (uint32_t)(max_grid / 8);
    (void)lb_ok;
    if (g_tune_max_grid > 0) max_grid = g_tune_max_grid;
    // the ablation bits: a compile-time 0 outside the tuning build
    const uint32_t tune = ZHIP_TUNING ? p.tune : 0u;
    // (the kTunePersist arm never applies to a launch carrying fused index
    // checks of CRC-free inner chunks: only k_decode_lead carries those)
    const bool lead_launch = !(p.lflags & ZHIP_LF_CRC) && p.n_idx != 0;
    if (p.rows && p.rowmap && p.seg == (uint32_t)kWgStride * kDefaultBlocks &&
        (!(tune & kTunePersist) || lead_launch)) {
        // one workgroup per pair of units, non-persistent (k_decode_pair)
        const int nu = (tune & kTuneSingle) ? 1 : 2;
        const bool crc = (p.lflags & ZHIP_LF_CRC) != 0, swap = (p.lflags & ZHIP_LF_SWAP) != 0;
        if (p.nseg == 1u && p.E <= 4u * kWgStride && g_tune_arm != 11) {
            // chunks of <= 16 KiB (sharded or not, with a CRC or not): four per
            // workgroup over their live steps, after the leading index-check
            // workgroups if any (k_decode_lead4; arm 11 keeps the pair kernels)
            // (chunks of 4-8 KiB: eight per workgroup over their last two steps;
            // graph-timed on the example array unsharded, profiles/r04/lead8/:
            // 8 KiB chunks 25.3-25.6 us vs 37.1 with four per workgroup and 30.8
            // with the pair kernel; 4 KiB chunks 37.2 with four, 52.4 with eight,
            // 41.4 with the pair kernel.  Arms 12 / 13 force four / eight.)
            // (k_decode_lead8 covers at most two steps: arm 13 cannot force it
            // onto chunks of more than 8 KiB)
            const bool e8 = p.E <= 2u * kWgStride &&
                            (g_tune_arm == 13 || (g_tune_arm != 12 && p.E > (uint32_t)kWgStride));
            KernelFn qfn = select_pair_kernel(crc, p.g.itemsize, swap, e8 ? 11 : 10);
            if (!qfn) return ZHIP_E_UNSUPPORTED;
            const uint32_t per = e8 ? 8u : 4u;
            const uint32_t quads = (uint32_t)(((uint64_t)p.n_units + per - 1u) / per);
            const uint32_t lead = (p.n_idx + 7u) & ~7u;
            if ((uint64_t)quads + lead > 0x7FFFFFFFull) return ZHIP_E_UNSUPPORTED;
            g_last_kernel = e8 ? "k_decode_lead8" : "k_decode_lead4";
            hipLaunchKernelGGL(qfn, dim3(quads + lead), dim3(kThreads), 0, stream, p);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
        if (!crc && p.n_idx) {
            // inner chunks without a CRC, shard indexes with one (zarr's default
            // sharding codecs): leading index-check workgroups, then the pairs
            // (k_decode_lead); > 32 units per chunk is not fused
            if (p.nseg > 32u) return ZHIP_E_UNSUPPORTED;
            KernelFn lfn = select_pair_kernel(false, p.g.itemsize, swap, 9);
            if (!lfn) return ZHIP_E_UNSUPPORTED;
            const uint32_t pairs = (uint32_t)(((uint64_t)p.n_units + 1u) / 2u);
            const uint32_t lead = (p.n_idx + 7u) & ~7u;
            if ((uint64_t)pairs + lead > 0x7FFFFFFFull) return ZHIP_E_UNSUPPORTED;
            DecodeParams q = p;
            q.xcd_run = (!(tune & kTuneNoXcd) && pairs % 8u == 0u && pairs <= (uint32_t)(max_grid / 8) * 4u)
                            ? pairs / 8u : 0u;
            q.h.xcd_run = q.xcd_run;
            q.h.d_xcd = make_fdiv(q.xcd_run ? q.xcd_run : 1u);
            g_last_kernel = "k_decode_lead";
            hipLaunchKernelGGL(lfn, dim3(pairs + lead), dim3(kThreads), 0, stream, q);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
        // chunks of a multiple of 8 x 32 KiB: interleaved steps in groups of
        // eight workgroups (k_decode_il, see decode_rows.hip) -- graph-timed
        // 26.4 vs 27.8 us on the headline; groups of four lose to the pair
        // kernel at C4 (profiles/r03/il/).  kTuneIl / kTuneNoIl force.
        const bool il = p.il_S != 0 && crc && !(tune & (kTuneNoIl | kTuneSkipCrc | kTuneSingle | kTuneDuo)) &&
                        ((tune & kTuneIl) || p.il_S >= 8u);
#if ZHIP_TUNING
        const bool xw = p.xw != 0 && crc && (tune & kTuneXw) &&
                        !(tune & (kTuneNoXw | kTuneSkipCrc | kTuneSingle | kTuneDuo | kTuneIl));
        if (xw) {
            KernelFn xfn = select_xw_kernel(crc, p.g.itemsize, swap);
            if (!xfn) return ZHIP_E_UNSUPPORTED;
            const uint64_t xg = (uint64_t)((p.n_chunks + 3u) / 4u) * p.xw;
            const uint64_t grid = xg > p.n_idx ? xg : p.n_idx;
            if (grid == 0) return ZHIP_OK;
            if (grid > 0x7FFFFFFFull) return ZHIP_E_UNSUPPORTED;
            g_last_kernel = "k_decode_xw";
            hipLaunchKernelGGL(xfn, dim3((uint32_t)grid), dim3(kThreads), 0, stream, p);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
        if (g_tune_arm >= 28 && g_tune_arm <= 30) {  // overhead probes
            const uint32_t pgrid = p.n_units > p.n_idx ? p.n_units : p.n_idx;
            if (pgrid == 0) return ZHIP_OK;
            KernelFn pf = g_tune_arm == 28 ? k_probe<0> : g_tune_arm == 29 ? k_probe<1> : k_probe<2>;
            g_last_kernel = g_tune_arm == 28 ? "k_probe_args" : g_tune_arm == 29 ? "k_probe_lds" : "k_probe_header";
            hipLaunchKernelGGL(pf, dim3(pgrid), dim3(kThreads), 0, stream, p);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
        if (crc && p.ilw_nt && (g_tune_arm == 26 || g_tune_arm == 27 || g_tune_arm == 31 || g_tune_arm == 32 ||
                                g_tune_arm == 42)) {
            // k_decode_ilw: one 32 KiB unit per workgroup of 1024 / 512 lanes
            // (31 / 32: the lane multiply in registers; 42: half in registers)
            KernelFn wfn = g_tune_arm == 42
                               ? select_ilw_kernel(p.g.itemsize, swap, 513, false, false)
                               : select_ilw_kernel(p.g.itemsize, swap, (int)p.ilw_nt, g_tune_arm >= 31, p.aff_ok != 0);
            if (!wfn) return ZHIP_E_UNSUPPORTED;
            const uint32_t wgrid = p.n_units > p.n_idx ? p.n_units : p.n_idx;
            if (wgrid == 0) return ZHIP_OK;
            g_last_kernel = g_tune_arm == 42 ? "k_decode_ilw512m"
                            : p.ilw_nt == 1024u ? (g_tune_arm >= 31 ? "k_decode_ilw1024r" : "k_decode_ilw1024")
                                                : (g_tune_arm >= 31 ? "k_decode_ilw512r" : "k_decode_ilw512");
            hipLaunchKernelGGL(wfn, dim3(wgrid), dim3(p.ilw_nt), 0, stream, p);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
        if (il && (g_tune_arm == 41 || g_tune_arm == 59) && p.ilh_klane) {  // k_decode_ilh: 16 KiB per workgroup
            // (59: with the look-back finalizer, at most 64 half units per chunk)
            KernelFn hfn = select_ilh_kernel(p.g.itemsize, swap, g_tune_arm == 59 && lb_ok && p.nseg <= 32u, false);
            if (!hfn) return ZHIP_E_UNSUPPORTED;
            const uint32_t hunits = 2u * p.n_units;
            const uint32_t hgrid = hunits > p.n_idx ? hunits : p.n_idx;
            if (hgrid == 0) return ZHIP_OK;
            g_last_kernel = "k_decode_ilh";
            hipLaunchKernelGGL(hfn, dim3(hgrid), dim3(kThreads), 0, stream, p);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
        if (il && g_tune_arm == 35 && p.pred) {  // k_decode_ilp: index entry off the stores' path
            KernelFn pfn = select_ilp_kernel(p.g.itemsize, swap);
            if (!pfn) return ZHIP_E_UNSUPPORTED;
            const uint32_t igrid = p.n_units > p.n_idx ? p.n_units : p.n_idx;
            if (igrid == 0) return ZHIP_OK;
            g_last_kernel = "k_decode_ilp";
            hipLaunchKernelGGL(pfn, dim3(igrid), dim3(kThreads), 0, stream, p);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
        if (il && g_tune_arm == 25) {  // k_decode_ilc: tables built in LDS, predicted loads first
            KernelFn cfn = select_ilc_kernel(p.g.itemsize, swap);
            if (!cfn) return ZHIP_E_UNSUPPORTED;
            const uint32_t igrid = p.n_units > p.n_idx ? p.n_units : p.n_idx;
            if (igrid == 0) return ZHIP_OK;
            g_last_kernel = "k_decode_ilc";
            hipLaunchKernelGGL(cfn, dim3(igrid), dim3(kThreads), 0, stream, p);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
        if (il && g_tune_arm >= 20 && g_tune_arm <= 24) {
            // k_decode_ilq arms: NQ units per workgroup, tables by registers or LDS-DMA
            static const char* names[] = {"k_decode_ilq2", "k_decode_ilq4", "k_decode_ilq1_glds",
                                          "k_decode_ilq2_glds", "k_decode_ilq4_glds"};
            const int a = g_tune_arm - 20;
            const int nq = (a == 0 || a == 3) ? 2 : (a == 1 || a == 4) ? 4 : 1;
            if (p.nseg % (uint32_t)nq) return ZHIP_E_UNSUPPORTED;
            KernelFn qfn = select_ilq_kernel(p.g.itemsize, swap, nq, a >= 2);
            if (!qfn) return ZHIP_E_UNSUPPORTED;
            const uint32_t ug = (uint32_t)(((uint64_t)p.n_units + nq - 1u) / nq);
            const uint32_t xg = (p.n_idx + (uint32_t)nq - 1u) / (uint32_t)nq;
            const uint32_t qgrid = ug > xg ? ug : xg;
            if (qgrid == 0) return ZHIP_OK;
            g_last_kernel = names[a];
            hipLaunchKernelGGL(qfn, dim3(qgrid), dim3(nq * kThreads), 0, stream, p);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
#endif
        // grids of at most kIlwMaxUnits units (2 per CU: the N = 4 / 8 shares of
        // the strong-scaled headline) with fewer chunks than CUs: half units of
        // 16 KiB (k_decode_ilh, two workgroups per unit) publishing through the
        // look-back finalizer -- graph-timed 8.39 vs 9.77 us (k_decode_ilw512)
        // at the N = 8 share, 10.73 vs 11.03 at N = 4 (profiles/r06/a/).
        // (Tuning build: arm 0 only; arm 58 / 49 keep k_decode_ilw512.)
        if (il && p.ilh_klane && p.n_units <= kIlwMaxUnits && lb_ok && p.nseg <= 32u &&
            (g_tune_arm == 0 || g_tune_arm == 60) && (tune & ~kTuneStamp) == 0) {
            KernelFn hfn = select_ilh_kernel(p.g.itemsize, swap, true, p.aff_ok != 0);
            if (!hfn) return ZHIP_E_UNSUPPORTED;
            const uint32_t hunits = 2u * p.n_units;
            const uint32_t hgrid = hunits > p.n_idx ? hunits : p.n_idx;
            if (hgrid == 0) return ZHIP_OK;
            g_last_kernel = "k_decode_ilh";
            hipLaunchKernelGGL(hfn, dim3(hgrid), dim3(kThreads), 0, stream, p);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
        // otherwise 512 lanes per unit, four blocks per lane (k_decode_ilw,
        // decode_rows.hip) -- graph-timed 8.8 vs 9.4 us at the N = 8 share, 10.3
        // vs 11.0 at N = 4; 14.6 vs 16.5 for k_decode_il at N = 2
        // (profiles/r05/f/).  (Tuning build: any arm keeps k_decode_il.)
        if (il && p.ilw_nt == 512u && p.n_units <= kIlwMaxUnits &&
            (g_tune_arm == 0 || g_tune_arm == 45 || g_tune_arm == 61 || ((g_tune_arm == 49 || g_tune_arm == 58) && p.aff_ok)) &&
            (tune & ~kTuneStamp) == 0) {
            // (tuning arms, whole-chunk reads: 49 the split publication, 58 the
            // look-back finalizer)
            const int nt = g_tune_arm == 49 ? 515 : (g_tune_arm == 58 && lb_ok && p.nseg <= 64u) ? 516 : 512;
            KernelFn wfn = select_ilw_kernel(p.g.itemsize, swap, nt, false, p.aff_ok != 0);
            if (!wfn) return ZHIP_E_UNSUPPORTED;
            const uint32_t wgrid = p.n_units > p.n_idx ? p.n_units : p.n_idx;
            if (wgrid == 0) return ZHIP_OK;
            g_last_kernel = "k_decode_ilw512";
            hipLaunchKernelGGL(wfn, dim3(wgrid), dim3(512), 0, stream, p);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
        if (il) {
#if ZHIP_TUNING
            // (arms 1 / 2 are k_decode_il's own; every other arm keeps production here)
            // (58: the look-back finalizer, while fewer chunks than CUs)
            KernelFn ifn = (g_tune_arm == 1 || g_tune_arm == 2 ||
                            ((g_tune_arm == 49 || (g_tune_arm >= 51 && g_tune_arm <= 57) ||
                              (g_tune_arm == 58 && lb_ok && p.nseg <= 32u) ||
                              g_tune_arm == 64 || g_tune_arm == 65) && p.aff_ok))
                               ? select_il_kernel_arm(crc, p.g.itemsize, swap, g_tune_arm)
                           : (tune & kTuneCfLookup) ? select_il_kernel_cf(crc, p.g.itemsize, swap)
                           : (tune & kTuneIlLean) ? select_il_kernel_lean(crc, p.g.itemsize, swap)
                           : (tune & (kTuneIlRegMul | kTuneIlOcc6))
                               ? select_il_kernel_regmul(crc, p.g.itemsize, swap, (tune & kTuneIlOcc6) != 0)
                               : (tune & (kTuneNoTables | kTuneNoRunEnd | kTuneNoPub | kTuneStamp))
                                   ? select_il_kernel_tuned(crc, p.g.itemsize, swap)
                                   : select_il_kernel(crc, p.g.itemsize, swap, p.aff_ok != 0);
#else
            KernelFn ifn = select_il_kernel(crc, p.g.itemsize, swap, p.aff_ok != 0);
#endif
            if (!ifn) return ZHIP_E_UNSUPPORTED;
            const uint32_t igrid = p.n_units > p.n_idx ? p.n_units : p.n_idx;
            if (igrid == 0) return ZHIP_OK;
            g_last_kernel = "k_decode_il";
            hipLaunchKernelGGL(ifn, dim3(igrid), dim3(kThreads), 0, stream, p);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
#if ZHIP_TUNING
        KernelFn fn = nu != 2 ? nullptr
                      : (tune & kTuneTrailingCrc) ? select_pair_kernel(crc, p.g.itemsize, swap, 3)
                      : (tune & kTuneSplitChain) ? select_pair_kernel(crc, p.g.itemsize, swap, 4)
                      : (tune & kTuneSkipCrc) ? select_pair_kernel(crc, p.g.itemsize, swap, 5)
                      : (tune & (kTunePrio | kTuneDeferB))
                          ? select_pair_kernel(crc, p.g.itemsize, swap,
                                               (tune & kTunePrio) && (tune & kTuneDeferB) ? 8
                                               : (tune & kTunePrio) ? 6 : 7)
                          : nullptr;
#else
        KernelFn fn = nullptr;
#endif
        if (!fn) fn = select_pair_kernel(crc, p.g.itemsize, swap, nu);
        if (!fn) return ZHIP_E_UNSUPPORTED;
        // chunks of more than 32 units (> 1 MiB): one unit per 256-thread half of
        // a 512-thread workgroup (k_decode_duo; C1 0.55 -> 0.62 of HBM peak,
        // profiles/r02/kernel_arms_ab.jsonl); kTuneDuo forces it
        if ((tune & kTuneDuo) || (p.nseg > 32 && !(tune & (kTuneSingle | kTuneSkipCrc)))) {
            KernelFn dfn = select_duo_kernel(crc, p.g.itemsize, swap);
            if (!dfn) return ZHIP_E_UNSUPPORTED;
            const uint32_t duos = (uint32_t)(((uint64_t)p.n_units + 1u) / 2u);
            const uint32_t dgrid = duos > p.n_idx ? duos : p.n_idx;
            if (dgrid == 0) return ZHIP_OK;
            g_last_kernel = "k_decode_duo";
            hipLaunchKernelGGL(dfn, dim3(dgrid), dim3(2 * kThreads), 0, stream, p);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
        const uint32_t pairs = (uint32_t)(((uint64_t)p.n_units + nu - 1u) / nu);
        const uint32_t grid = pairs > p.n_idx ? pairs : p.n_idx;
        if (grid == 0) return ZHIP_OK;
        // one resident wave of workgroups (4 per CU; max_grid = 8 per CU): the
        // workgroups of one XCD take a contiguous eighth of the batch
        DecodeParams q = p;
        q.xcd_run = (nu == 2 && !(tune & kTuneNoXcd) && grid % 8u == 0u &&
                     grid <= (uint32_t)(max_grid / 8) * 4u) ? grid / 8u : 0u;
        q.h.xcd_run = q.xcd_run;
        q.h.d_xcd = make_fdiv(q.xcd_run ? q.xcd_run : 1u);
        g_last_kernel = "k_decode_pair";
            hipLaunchKernelGGL(fn, dim3(grid), dim3(kThreads), 0, stream, q);
        return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
    }
    if (p.rows) {
        KernelFn fn = select_rows_kernel((p.lflags & ZHIP_LF_CRC) != 0, p.g.itemsize, (p.lflags & ZHIP_LF_SWAP) != 0,
                                         (int)(p.seg / kWgStride));
        if (!fn) return ZHIP_E_UNSUPPORTED;
        if (p.n_units == 0) return ZHIP_OK;
        if (g_tune_max_grid <= 0) {
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(fn), kThreads,
                                                             0) == hipSuccess && per_cu > 0)
                max_grid = (max_grid / 8) * per_cu;
        }
        const uint32_t grid = p.n_units < (uint32_t)max_grid ? p.n_units : (uint32_t)max_grid;
        g_last_kernel = "k_decode_rows";
        hipLaunchKernelGGL(fn, dim3(grid), dim3(kThreads), 0, stream, p);
        return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
    }
    if (p.tq >= 0 && p.tile4) {
        // four tiles per workgroup, non-persistent (k_decode_tile4, decode_tile.hip)
        // (arm kTuneTile4F: one A_64 chain per thread when the layout's tile step is
        // 256 B, k_decode_tile4f -- exact, measured 0.3-0.4 us slower on C3)
        const bool f4 = ZHIP_TUNING && p.t4f_tab != nullptr && (p.lflags & ZHIP_LF_CRC) != 0;
        const bool w4 = !f4 && p.t4w_tab != nullptr && (p.lflags & ZHIP_LF_CRC) != 0;
        const bool swp = (p.lflags & ZHIP_LF_SWAP) != 0;
        // two tiles per workgroup (2 048 workgroups on C3: two residency rounds
        // instead of one) -- graph-timed 27.8-27.9 vs 28.4-30.0 us on C3
        // (profiles/r05/l/); tuning arm 38 keeps four, 37 takes one (46 us)
        if (w4 && ((p.t2w_kq && g_tune_arm != 38 && g_tune_arm != 37) || (g_tune_arm == 37 && p.t1w_kq))) {
            const int nt = g_tune_arm == 37 ? 1 : 2;
            // (tuning arm 49: the split publication of 17..32 workgroups per chunk)
            // (tuning arm 67: the byte-table chains, where the plan built them)
            KernelFn fn2 = select_tile2w_kernel(p.g.itemsize, swp,
                                                (nt == 2 && g_tune_arm == 49) ? 3
                                                : (nt == 2 && g_tune_arm == 67 && p.tbt_tab) ? 4 : nt);
            if (!fn2) return ZHIP_E_UNSUPPORTED;
            if (p.n_units == 0) return ZHIP_OK;
            DecodeParams q = p;
            q.t4w_kq = nt == 1 ? p.t1w_kq : p.t2w_kq;
            g_last_kernel = nt == 1 ? "k_decode_tile1w" : g_tune_arm == 49 ? "k_decode_tile2ws"
                            : (g_tune_arm == 67 && p.tbt_tab) ? "k_decode_tile2w_bt" : "k_decode_tile2w";
            hipLaunchKernelGGL(fn2, dim3(p.n_units / (uint32_t)nt), dim3(kThreads), 0, stream, q);
            return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
        }
#if ZHIP_TUNING
        KernelFn fn = f4 ? select_tile4f_kernel(p.g.itemsize, swp)
                      : w4 ? select_tile4w_kernel(p.g.itemsize, swp)
                           : select_tile4_kernel((p.lflags & ZHIP_LF_CRC) != 0, p.g.itemsize, swp);
#else
        KernelFn fn = w4 ? select_tile4w_kernel(p.g.itemsize, swp)
                         : select_tile4_kernel((p.lflags & ZHIP_LF_CRC) != 0, p.g.itemsize, swp);
#endif
        if (!fn) return ZHIP_E_UNSUPPORTED;
        if (p.n_units == 0) return ZHIP_OK;
        g_last_kernel = f4 ? "k_decode_tile4f" : w4 ? "k_decode_tile4w" : "k_decode_tile4";
        hipLaunchKernelGGL(fn, dim3(p.n_units / 4u), dim3(kThreads), 0, stream, p);
        return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
    }
    if (p.tq >= 0 && p.tile2) {
        // consecutive tile pairs (k_decode_tile4w<2>, decode_tile.hip): 128^3
        // chunks' two 256-byte column blocks of one row band per workgroup
        KernelFn fn = select_tile2w_kernel(p.g.itemsize, (p.lflags & ZHIP_LF_SWAP) != 0, 2);
        if (!fn) return ZHIP_E_UNSUPPORTED;
        if (p.n_units == 0) return ZHIP_OK;
        if (p.n_units / 2u >= (1u << 31)) return ZHIP_E_UNSUPPORTED;
        g_last_kernel = "k_decode_tilep";
        hipLaunchKernelGGL(fn, dim3(p.n_units / 2u), dim3(kThreads), 0, stream, p);
        return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
    }
    if (p.tq >= 0 && p.tileg) {
        // tiles grouped by four along a stored dim (k_decode_tileg, decode_tile.hip)
        // (k_decode_tilegw when the plan's wave-per-tile chains are selected)
        const bool gw = p.t4w_tab != nullptr && (p.lflags & ZHIP_LF_CRC) != 0;
        // (arm 2: the returning publication whatever the flags)
        const bool defer = p.defer != 0 && g_tune_arm != 2;
        // two tiles per workgroup where the plan built their constants (as
        // k_decode_tile4w); tuning arms 38 (deferred) / 2 (returning) keep four
        int nt = (gw && p.t2w_kq && g_tune_arm != 38 && g_tune_arm != 2 && g_tune_arm != 40) ? 2 : 4;
        int nsel = nt;
#if ZHIP_TUNING
        if (gw && g_tune_arm == 40 && p.tglt_kq) nt = nsel = 5;  // four tiles, lanes pick the tile
        if (nt == 2 && g_tune_arm == 48) nsel = 6;  // the arrival words packed (round-4 layout)
        // the look-back finalizer (fewer chunks than CUs; the spread subwords)
        if (nt == 2 && g_tune_arm == 62 && lb_ok && p.n_groups <= 128u) nsel = 7;
        if (nt == 2 && g_tune_arm == 66 && p.tbt_tab) nsel = 8;  // the byte-table chains
#endif
        KernelFn fn = gw ? select_tilegw_kernel(p.g.itemsize, (p.lflags & ZHIP_LF_SWAP) != 0, defer, nsel)
                         : select_tileg_kernel((p.lflags & ZHIP_LF_CRC) != 0, p.g.itemsize,
                                               (p.lflags & ZHIP_LF_SWAP) != 0, defer);
        if (!fn) return ZHIP_E_UNSUPPORTED;
        if (p.n_chunks == 0) return ZHIP_OK;
        const uint64_t ggrid = (uint64_t)p.n_chunks * p.n_groups * (uint32_t)(nt == 2 ? 2 : 1);
        if (ggrid >= (1ull << 31)) return ZHIP_E_UNSUPPORTED;
        DecodeParams q = p;
        if (nt == 2) q.t4w_kq = p.t2w_kq;
        if (nt == 5) q.t4w_kq = p.tglt_kq;
        g_last_kernel = !gw ? "k_decode_tileg" : nsel == 6 ? "k_decode_tileg2wp" : nsel == 7 ? "k_decode_tileg2w_lb"
                                           : nsel == 8 ? "k_decode_tileg2w_bt"
                                           : nt == 2 ? "k_decode_tileg2w"
                                           : nt == 5 ? "k_decode_tileglt"
                                                                                      : "k_decode_tilegw";
        hipLaunchKernelGGL(fn, dim3((uint32_t)ggrid), dim3(kThreads), 0, stream, q);
        return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
    }
    if (p.tq >= 0) {
        KernelFn fn = select_tile_kernel((p.lflags & ZHIP_LF_CRC) != 0, p.g.itemsize, (p.lflags & ZHIP_LF_SWAP) != 0);
        if (!fn) return ZHIP_E_UNSUPPORTED;
        if (p.n_units == 0) return ZHIP_OK;
        if (g_tune_max_grid <= 0) {
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(fn), kThreads,
                                                             0) == hipSuccess && per_cu > 0)
                max_grid = (max_grid / 8) * per_cu;
        }
        const uint32_t grid = p.n_units < (uint32_t)max_grid ? p.n_units : (uint32_t)max_grid;
        g_last_kernel = "k_decode_tile";
        hipLaunchKernelGGL(fn, dim3(grid), dim3(kThreads), 0, stream, p);
        return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
    }
    KernelFn fn = select_decode_kernel((p.lflags & ZHIP_LF_CRC) != 0, (p.lflags & ZHIP_LF_NO_WRITE) == 0,
                                       p.fast != 0, p.g.itemsize, (p.lflags & ZHIP_LF_SWAP) != 0,
                                       (int)(p.seg / kWgStride));
    if (!fn) return ZHIP_E_UNSUPPORTED;
    if (p.n_units == 0) return ZHIP_OK;
    if (g_tune_max_grid <= 0) {
        // persistent grid = resident workgroups (units are software-pipelined per WG)
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(fn),
                                                         kThreads, 0) == hipSuccess && per_cu > 0)
            max_grid = (max_grid / 8) * per_cu;  // max_grid arrives as CUs * 8
    }
    const uint32_t grid = p.n_units < (uint32_t)max_grid ? p.n_units : (uint32_t)max_grid;
    g_last_kernel = "k_decode";
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kThreads), 0, stream, p);
    return hipGetLastError() == hipSuccess ? ZHIP_OK : ZHIP_E_HIP;
}

}  // namespace zhip

extern "C" const char* zhip_last_kernel(void) { return zhip::g_last_kernel; }
