// C ABI of zarr_hip (include/zarrhip.h): plan building (host GF(2) math, one
// upload), launches, error reporting, and CPU self-tests of the CRC-combine
// algebra the kernels rely on.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/zarrhip.h"
#include "zhip_gf2.h"
#include "zhip_internal.h"

using namespace zhip;

namespace {

thread_local std::string g_err;

int set_err(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return set_err(ZHIP_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_));  \
    } while (0)

uint32_t g_T[256];      // standard byte table: A_1(v) = (v >> 8) ^ T[v & 255]
uint8_t g_invtop[256];  // top byte of T[i] -> i
std::once_flag g_once;

void init_tables() {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
        g_T[i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i) g_invtop[g_T[i] >> 24] = (uint8_t)i;
}

// x^(8n) mod P
uint32_t xpow8(uint64_t n) {
    uint32_t p = kOne;
    uint32_t b = kOne >> 8;  // x^8
    while (n) {
        if (n & 1) p = gf_mul(p, b);
        b = gf_mul(b, b);
        n >>= 1;
    }
    return p;
}

// x^-8 mod P: one inverse byte step applied to 1.
uint32_t xinv8() {
    const uint32_t s = kOne;
    const uint32_t i = g_invtop[s >> 24];
    return (((s ^ g_T[i]) & 0x00FFFFFFu) << 8) | i;
}

// x^(-8n) mod P = (x^-8)^n by square-and-multiply.
uint32_t xpow8_inv(uint64_t n) {
    uint32_t p = kOne;
    uint32_t b = xinv8();
    while (n) {
        if (n & 1) p = gf_mul(p, b);
        b = gf_mul(b, b);
        n >>= 1;
    }
    return p;
}

void build_horner_stride(uint32_t* tab, uint64_t stride) {  // [op][slice][256], op k = A_(stride - 4k)
    for (int op = 0; op < 4; ++op) {
        const uint32_t x = xpow8(stride - 4u * op);
        for (int sl = 0; sl < 4; ++sl)
            for (uint32_t b = 0; b < 256; ++b) tab[op * 1024 + sl * 256 + b] = gf_mul(x, b << (8 * sl));
    }
}


uint32_t crc_bytewise(const uint8_t* p, size_t n) {
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; ++i) c = (c >> 8) ^ g_T[(c ^ p[i]) & 255u];
    return ~c;
}

// Host CRC-32C for the host stage of a chain (zhip_crc32c_host): the x86
// crc32 instruction, 8 bytes per step, as google-crc32c uses on this host;
// bytewise tables where the CPU lacks SSE4.2.
__attribute__((target("sse4.2"))) uint32_t crc_sse42(const uint8_t* p, size_t n) {
    uint64_t c = 0xFFFFFFFFu;
    while (n && (reinterpret_cast<uintptr_t>(p) & 7u)) {
        c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
        --n;
    }
    for (; n >= 8; n -= 8, p += 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        c = __builtin_ia32_crc32di(c, w);
    }
    while (n--) c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
    return ~(uint32_t)c;
}

// k_decode_pair tables (kPairTab* layout): A4096 (A_stride) over 11/11/10-bit
// slices of a word, and the byte slices of A4 that fold the four word
// accumulators
void build_pair_tables(uint32_t* tab, uint64_t stride = kWgStride) {
    const uint32_t x = xpow8(stride);
    for (uint32_t i = 0; i < 2048; ++i) {
        tab[kPairT1 + i] = gf_mul(x, i);
        tab[kPairT2 + i] = gf_mul(x, i << 11);
    }
    for (uint32_t i = 0; i < 1024; ++i) tab[kPairT3 + i] = gf_mul(x, i << 22);
    const uint32_t x4 = xpow8(4);
    for (int sl = 0; sl < 4; ++sl)
        for (uint32_t b = 0; b < 256; ++b) tab[kPairA4 + sl * 256 + b] = gf_mul(x4, b << (8 * sl));
}

void build_horner(uint32_t* tab) {  // [op][slice][256], op k = A_(4096 - 4k)
    for (int op = 0; op < 4; ++op) {
        const uint32_t x = xpow8((uint64_t)kWgStride - 4u * op);
        for (int sl = 0; sl < 4; ++sl)
            for (uint32_t b = 0; b < 256; ++b) tab[op * 1024 + sl * 256 + b] = gf_mul(x, b << (8 * sl));
    }
}

}  // namespace

namespace zhip {
// Source offset of every tile's first row in the stored chunk (tile index:
// column block fastest, then row block, then the other dims, last fastest).
std::vector<uint64_t> tile_bases(const zhip_plan& plan) {
    const zhip_layout& L = plan.layout;
    const uint64_t sq = plan.sstride[plan.tq];
    std::vector<uint64_t> base(plan.t_per_chunk);
    for (uint32_t ti = 0; ti < plan.t_per_chunk; ++ti) {
        uint32_t r = ti;
        const uint32_t cb = r % plan.n_cb;
        r /= plan.n_cb;
        const uint32_t qb = r % plan.n_qb;
        r /= plan.n_qb;
        uint64_t b = (uint64_t)qb * kTileRows * sq + (uint64_t)cb * kTileCols;
        for (int d = L.ndim - 2; d >= 0; --d) {
            if (d == plan.tq) continue;
            b += (uint64_t)(r % (uint32_t)L.shape[d]) * plan.sstride[d];
            r /= (uint32_t)L.shape[d];
        }
        base[ti] = b;
    }
    return base;
}

void fill_geom(Geom& g, const zhip_plan& plan) {
    const zhip_layout& L = plan.layout;
    g.ndim = L.ndim;
    g.itemsize = L.itemsize;
    for (int d = 0; d < ZHIP_MAX_DIMS; ++d) {
        g.shape[d] = d < L.ndim ? L.shape[d] : 1;
        g.ostride[d] = d < L.ndim ? L.out_stride[d] : 0;
        g.dshape[d] = plan.dshape[d];
    }
    g.nbytes = (uint32_t)L.nbytes;
    g.row_bytes = plan.row_bytes;
    g.drow = plan.drow;
}

#if ZHIP_TUNING
uint32_t g_tune_bits = 0;
int g_tune_blocks = 0;
int g_tune_arm = 0;
#endif
}

extern "C" {

int zhip_tuning_build(void) { return ZHIP_TUNING; }

int zhip_set_tuning(int key, int value) {
    switch (key) {
#if ZHIP_TUNING
        case ZHIP_TUNE_MAX_GRID: g_tune_max_grid = value; return ZHIP_OK;
        case ZHIP_TUNE_ABLATION: g_tune_bits = (uint32_t)value; return ZHIP_OK;
        case ZHIP_TUNE_BLOCKS: g_tune_blocks = value; return ZHIP_OK;
        case ZHIP_TUNE_ARM: g_tune_arm = value; return ZHIP_OK;
#else
        case ZHIP_TUNE_MAX_GRID:
        case ZHIP_TUNE_ABLATION:
        case ZHIP_TUNE_BLOCKS:
        case ZHIP_TUNE_ARM:
            if (value == 0) return ZHIP_OK;  // the production setting
            return set_err(ZHIP_E_UNSUPPORTED, "kernel tuning knobs exist only in the tuning build "
                                               "(libzarrhip_tune.so, make tune)");
#endif
        case ZHIP_TUNE_STAGE_STREAMS: zhip_stage_set_streams(value >= 2 ? 2u : 1u); return ZHIP_OK;
        case ZHIP_TUNE_STAGE_COPY: zhip_stage_set_copy(value ? 1u : 0u); return ZHIP_OK;
        default: return set_err(ZHIP_E_INVALID, "unknown tuning key");
    }
}

int zhip_dv_check(const zhip_dv_ref* d_refs, uint32_t n_refs, void* stream) {
    if (n_refs && !d_refs) return set_err(ZHIP_E_INVALID, "null argument");
    if (n_refs > 65535u) return set_err(ZHIP_E_INVALID, "too many launches in one check");
    if (zhip::launch_dv_check(d_refs, n_refs, static_cast<hipStream_t>(stream)) != ZHIP_OK)
        return set_err(ZHIP_E_HIP, "k_dv_check launch failed");
    return ZHIP_OK;
}

int zhip_abi_version(void) { return ZHIP_ABI_VERSION; }

int zhip_debug_stamps(uint64_t* host_out, uint32_t n_wg) {
    if (!host_out) return set_err(ZHIP_E_INVALID, "null argument");
    if (zhip::debug_stamps(host_out, n_wg) != 0) return set_err(ZHIP_E_HIP, "hipMemcpyFromSymbol failed");
    return ZHIP_OK;
}

const char* zhip_last_error(void) { return g_err.c_str(); }

int zhip_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

static void plan_affine(zhip_plan* p);

int zhip_plan_create(const zhip_layout* layout, zhip_plan** out) {
    std::call_once(g_once, init_tables);
    if (!layout || !out) return set_err(ZHIP_E_INVALID, "null argument");
    const zhip_layout& L = *layout;
    if (L.ndim < 1 || L.ndim > ZHIP_MAX_DIMS) return set_err(ZHIP_E_UNSUPPORTED, "ndim must be 1..8");
    if (!(L.itemsize == 1 || L.itemsize == 2 || L.itemsize == 4 || L.itemsize == 8))
        return set_err(ZHIP_E_UNSUPPORTED, "itemsize must be 1, 2, 4 or 8");
    uint64_t n = (uint64_t)L.itemsize;
    for (int d = 0; d < L.ndim; ++d) {
        if (L.shape[d] < 0) return set_err(ZHIP_E_INVALID, "negative shape");
        n *= (uint64_t)L.shape[d];
    }
    if (n != L.nbytes) return set_err(ZHIP_E_INVALID, "nbytes != prod(shape)*itemsize");
    if (n >= (1ull << 31) - 8192) return set_err(ZHIP_E_UNSUPPORTED, "chunk payload must be < 2 GiB");
    zhip_plan* p = new (std::nothrow) zhip_plan();
    if (!p) return set_err(ZHIP_E_INVALID, "out of memory");
    p->layout = L;
    p->E = (uint32_t)((n + 15) & ~15ull);
    p->kblocks = (g_tune_blocks == 4 || g_tune_blocks == 16) ? (uint32_t)g_tune_blocks : (uint32_t)kDefaultBlocks;
    if (L.flags & ZHIP_LF_NO_WRITE || !(L.flags & ZHIP_LF_CRC)) p->kblocks = kDefaultBlocks;
    p->seg = (uint32_t)kWgStride * p->kblocks;
    p->nseg = p->E == 0 ? 1u : (p->E + p->seg - 1) / p->seg;
    // k_decode_il: groups of S x 8 steps must tile the chunk's steps
    p->il_S = 0;
    if (p->kblocks == (uint32_t)kDefaultBlocks && (L.flags & ZHIP_LF_CRC) && !(L.flags & ZHIP_LF_NO_WRITE)) {
        const uint32_t n_steps = p->nseg * (uint32_t)kDefaultBlocks;
        for (uint32_t S = 8; S >= 2 && !p->il_S; S /= 2)
            if (n_steps % (S * (uint32_t)kDefaultBlocks) == 0) p->il_S = S;
    }
    // k_decode_xw: 8 KiB spans (whole-row layouts keep E a multiple of 4 KiB)
    p->xw_P = 0;
    p->xw_nsub = 0;
    if (p->kblocks == (uint32_t)kDefaultBlocks && (L.flags & ZHIP_LF_CRC) && !(L.flags & ZHIP_LF_NO_WRITE)) {
        p->xw_P = p->nseg * 4u;
        if (p->xw_P > 32u && p->xw_P <= 1024u) p->xw_nsub = (p->xw_P + 31u) / 32u;
    }
    p->R = (uint64_t)p->E + kWgStride;
    p->c_inv = xpow8_inv(p->R - n);
    p->c3 = gf_mul(xpow8(n), 0xFFFFFFFFu);
    for (int op = 0; op < 4; ++op) p->hx[op] = xpow8((uint64_t)kWgStride - 4u * op);
    for (int a = 0; a < 16; ++a) p->kq[a] = xpow8((uint64_t)kWgStride - 256u * a);
    for (int b = 0; b < 16; ++b) p->kq[16 + b] = xpow8_inv(16u * b);
    for (int d = 0; d < ZHIP_MAX_DIMS; ++d) p->dshape[d] = make_fdiv(d < L.ndim && L.shape[d] > 0 ? (uint32_t)L.shape[d] : 1u);
    p->row_bytes = (uint32_t)L.shape[L.ndim - 1] * (uint32_t)L.itemsize;
    p->drow = make_fdiv(p->row_bytes ? p->row_bytes : 1u);
    // fill pattern replicated to 16 bytes
    uint8_t f16[16];
    for (int i = 0; i < 16; ++i) f16[i] = L.fill[i % L.itemsize];
    std::memcpy(p->fill, f16, 16);
    p->idx_nbytes = 0;
    if (L.flags & ZHIP_LF_SHARDED) {
        const uint64_t ni = 16ull * L.n_inner;
        p->idx_nbytes = (uint32_t)ni;
        p->idx_E = (uint32_t)((ni + 15) & ~15ull);
        p->idx_c_inv = xpow8_inv((uint64_t)p->idx_E + kWgStride - ni);
        p->idx_c3 = gf_mul(xpow8(ni), 0xFFFFFFFFu);
    }
    p->device = -1;
    p->max_grid = 2048;
    p->d_tables = nullptr;
    p->d_tile_tables = nullptr;
    p->tile4 = 0;
    p->gd = -1;
    p->n_groups = 0;
    p->n_sub = 0;
    // tile mode: a stored dim (not the innermost) that is contiguous in out
    p->tq = -1;
    {
        uint64_t st = (uint64_t)L.itemsize;
        for (int d = L.ndim - 1; d >= 0; --d) {
            p->sstride[d] = (uint32_t)st;
            st *= (uint64_t)L.shape[d];
        }
        for (int d = L.ndim; d < ZHIP_MAX_DIMS; ++d) p->sstride[d] = 0;
        if (!(L.flags & ZHIP_LF_NO_WRITE) && L.ndim >= 2 && p->row_bytes % 16 == 0 && p->row_bytes > 0)
            for (int d = 0; d < L.ndim - 1; ++d)
                if (L.out_stride[d] == L.itemsize && L.shape[d] > 1) { p->tq = d; break; }
        if (p->tq >= 0) {
            p->n_qb = (uint32_t)((L.shape[p->tq] + kTileRows - 1) / kTileRows);
            p->n_cb = (p->row_bytes + kTileCols - 1) / kTileCols;
            uint64_t other = 1;
            for (int d = 0; d < L.ndim - 1; ++d)
                if (d != p->tq) other *= (uint64_t)L.shape[d];
            p->t_per_chunk = (uint32_t)(other * p->n_qb * p->n_cb);
            // k_decode_tile4 eligibility: full tiles, and every group of 4
            // consecutive tiles at one uniform base step (so one table multiply
            // carries a thread's Horner state from tile to tile)
            const uint32_t T = p->t_per_chunk;
            const std::vector<uint64_t> base = tile_bases(*p);
            const uint64_t step = T >= 2 ? base[1] - base[0] : 0;
            bool t4 = (L.shape[p->tq] % kTileRows) == 0 && (p->row_bytes % kTileCols) == 0 && T % 4 == 0 &&
                      T >= 4 && base[1] > base[0];
            for (uint32_t ti = 0; t4 && ti < T; ++ti)
                if (base[ti] != base[ti & ~3u] + (uint64_t)(ti & 3u) * step) t4 = false;
            p->tile4 = t4 ? 1u : 0u;
            p->tile4_step = step;
            // k_decode_tile4w over consecutive tile pairs where tile4 declines
            p->tile2 = (!t4 && (L.flags & ZHIP_LF_CRC) && (L.shape[p->tq] % kTileRows) == 0 &&
                        (p->row_bytes % kTileCols) == 0 && T % 2 == 0 && T >= 2 && T / 2 <= 65535u) ? 1u : 0u;
            // k_encode_tileg: the innermost other stored dim with shape % 4 == 0
            for (int d = L.ndim - 2; d >= 0 && p->gd < 0; --d)
                if (d != p->tq && L.shape[d] % 4 == 0) p->gd = d;
            if (p->gd >= 0) {
                p->n_groups = T / 4;
                // two-level arrival (subgroups of 16 workgroups) for 17..256 groups
                p->n_sub = (p->n_groups > 16u && p->n_groups <= 256u) ? (p->n_groups + 15u) / 16u : 0u;
            }
        }
    }
    plan_affine(p);
    *out = p;
    return ZHIP_OK;
}

// Upload the constant tables to the current device (done once per plan).
int zhip_plan_upload(zhip_plan* p) {
    if (!p) return set_err(ZHIP_E_INVALID, "null plan");
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    if (p->d_tables && p->device == dev) return ZHIP_OK;
    // horner (4096) | kthread (256) | kunit (nseg) | kpair (nseg x 256): the
    // per-lane constant kthread[t] * kunit[s] * c_inv of k_decode_pair, whose
    // run ends then need no uniform multiply at all
    const size_t n_old = 4096 + kThreads + p->nseg + (size_t)p->nseg * kThreads;
    const size_t n_pair = kPairTabWords + (size_t)p->nseg * kThreads + kThreads;
    const size_t n_il = p->il_S ? kPairTabWords + (size_t)p->nseg * kThreads + kThreads + kIlBasisWords : 0;
    const size_t n_xw = p->xw_P ? kPairTabWords + (size_t)p->xw_P * 64 + kThreads : 0;
    // k_decode_ilw regions (NT = 1024: tuning arms only; 512: the small-grid
    // form of k_decode_il's layouts)
    const bool ilw = (p->il_S == 8u || (ZHIP_TUNING && p->kblocks == (uint32_t)kDefaultBlocks &&
                                        (p->layout.flags & ZHIP_LF_CRC) && !(p->layout.flags & ZHIP_LF_NO_WRITE))) &&
                     p->nseg <= 256u;
    size_t n_ilw[2] = {0, 0};
    for (int i = ZHIP_TUNING ? 0 : 1; i < 2 && ilw; ++i) n_ilw[i] = kPairTabWords + (size_t)p->nseg * (1024u >> i) + kThreads;
    const size_t n_ilh = (ilw && p->il_S == 8u && 2 * p->nseg <= 64u) ? (size_t)2 * p->nseg * kThreads : 0;
    // k_decode_il's wider interleave (round 6): groups of 16 / 32 workgroups, the
    // same tables and constants for strides S = 16 / 32 where the chunk's steps
    // tile them (the decode takes the widest, il_decode_S; k_encode_il keeps
    // S = 8; tuning arms 69 / 70 / 71 force 16 / 32 / 8).  Graph-timed on the
    // headline: S = 32 25.49 / 25.33 us vs 25.76 / 25.76 for S = 8 in two
    // interleaved pairs (profiles/r06/f/)
    size_t n_ils[2] = {0, 0};
    for (int i = 0; i < 2 && p->il_S == 8u; ++i)
        if (((uint64_t)p->nseg * kDefaultBlocks) % ((16u << i) * (uint64_t)kDefaultBlocks) == 0) n_ils[i] = n_il;
    std::vector<uint32_t> h(n_old + n_pair + n_il + n_xw + n_ilw[0] + n_ilw[1] + n_ilh + n_ils[0] + n_ils[1]);
    build_horner(h.data());
    for (int t = 0; t < kThreads; ++t) h[4096 + t] = xpow8((uint64_t)kWgStride - 16u * t);
    for (uint32_t s = 0; s < p->nseg; ++s) h[4096 + kThreads + s] = xpow8((uint64_t)s * p->seg);
    for (uint32_t s = 0; s < p->nseg; ++s) {
        const uint32_t ku = gf_mul(h[4096 + kThreads + s], p->c_inv);
        for (int t = 0; t < kThreads; ++t)
            h[4096 + kThreads + p->nseg + (size_t)s * kThreads + t] = gf_mul(h[4096 + t], ku);
    }
    // pair tables; the combined four-accumulator state sits 12 bytes later than
    // the single-chain one, so the lane constants carry x^(-96)
    p->off_pair = n_old;
    build_pair_tables(h.data() + n_old);
    const uint32_t c96 = xpow8_inv(12);
    for (size_t i = 0; i < (size_t)p->nseg * kThreads; ++i)
        h[n_old + kPairTabWords + i] = gf_mul(h[4096 + kThreads + p->nseg + i], c96);
    for (int t = 0; t < kThreads; ++t)
        h[n_old + kPairTabWords + (size_t)p->nseg * kThreads + t] = gf_mul(h[4096 + t], c96);
    // k_decode_il: workgroup r of a chunk (group r / S, offset r % S) takes
    // steps st_k = (r / S) S 8 + r % S + S k; lane t's chain over them (stride
    // D = 4096 S) leaves word w of step st_0 multiplied by x^(8 D 8), so the
    // lane constant x^(8 (E - p_0 + 4096 - 8 D)) c_inv x^(-96) gives every
    // word at p the pair kernel's x^(8 (E - p + 4096)) c_inv (p_0 = E -
    // 4096 (n_steps - st_0) + 16 t); exponents may be negative
    auto build_il = [&](uint32_t* il, uint32_t il_S) {
        const uint64_t D = (uint64_t)kWgStride * il_S;
        build_pair_tables(il, D);
        const int64_t n_steps = (int64_t)p->nseg * kDefaultBlocks, K = kDefaultBlocks, S = il_S;
        for (uint32_t r = 0; r < p->nseg; ++r) {
            const int64_t st0 = (int64_t)(r / S) * S * K + (int64_t)(r % S);
            for (int t = 0; t < kThreads; ++t) {
                const int64_t e = (int64_t)kWgStride * (n_steps - st0 + 1 - S * K) - 16 * t;
                const uint32_t xe = e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)(-e));
                il[kPairTabWords + (size_t)r * kThreads + t] = gf_mul(gf_mul(xe, p->c_inv), c96);
            }
        }
        // the fused index check (one 4 KiB step per lane) under A_D: its state
        // is A_D(w) instead of A4096(w), so kthread11 times x^(-8(D - 4096))
        const uint32_t back = xpow8_inv(D - (uint64_t)kWgStride);
        for (int t = 0; t < kThreads; ++t)
            il[kPairTabWords + (size_t)p->nseg * kThreads + t] =
                gf_mul(h[n_old + kPairTabWords + (size_t)p->nseg * kThreads + t], back);
        // the tables' bases (they are linear in the index): T1 / T2 / T3 at
        // single bits, then the four A4 byte tables -- k_decode_ilc builds the
        // tables in LDS from these 64 words instead of loading 24 KiB
        uint32_t* bs = il + kPairTabWords + (size_t)p->nseg * kThreads + kThreads;
        for (int b = 0; b < 11; ++b) bs[b] = il[kPairT1 + (1u << b)];
        for (int b = 0; b < 11; ++b) bs[11 + b] = il[kPairT2 + (1u << b)];
        for (int b = 0; b < 10; ++b) bs[22 + b] = il[kPairT3 + (1u << b)];
        for (int j = 0; j < 4; ++j)
            for (int b = 0; b < 8; ++b) bs[32 + 8 * j + b] = il[kPairA4 + 256 * j + (1u << b)];
    };
    p->off_il = 0;
    if (p->il_S) {
        p->off_il = n_old + n_pair;
        build_il(h.data() + p->off_il, p->il_S);
    }
    p->off_xw = 0;
    if (p->xw_P) {
        // k_decode_xw: lane l of span r takes blocks p_k = lo + 8192 r + 1024 k
        // + 16 l (k < 8); its chain (A_1024) leaves block 0 multiplied by
        // x^(8 8192), so the constant x^(8 (E - p_0 + 4096 - 8192)) c_inv
        // x^(-96) gives every word the pair kernel's frame
        p->off_xw = n_old + n_pair + n_il;
        uint32_t* xw = h.data() + p->off_xw;
        build_pair_tables(xw, 1024);
        const int64_t n_steps = (int64_t)p->nseg * kDefaultBlocks;
        for (uint32_t r = 0; r < p->xw_P; ++r)
            for (int l = 0; l < 64; ++l) {
                const int64_t e = (int64_t)kWgStride * (n_steps - 2 * (int64_t)r - 1) - 16 * l;
                const uint32_t xe = e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)(-e));
                xw[kPairTabWords + (size_t)r * 64 + l] = gf_mul(gf_mul(xe, p->c_inv), c96);
            }
        // the fused index check under A_1024: state A_1024(w) instead of A4096(w)
        const uint32_t fwd = xpow8((uint64_t)kWgStride - 1024u);
        for (int t = 0; t < kThreads; ++t)
            xw[kPairTabWords + (size_t)p->xw_P * 64 + t] =
                gf_mul(h[n_old + kPairTabWords + (size_t)p->nseg * kThreads + t], fwd);
    }
    // k_decode_ilw: lane t of unit r (NT lanes) takes the blocks at 16 t + D k
    // (D = 16 NT, k < 2048 / NT); its A_D chain leaves every word w at p
    // multiplied by x^(8 (p_last + D - p)), so the lane constant
    // x^(8 (4096 (n_steps - 8 r - 7) - 16 t)) c_inv x^(-96) gives the pair
    // kernel's frame -- factored as F(r) G(t), G(t) = x^(-128 t)
    size_t at = n_old + n_pair + n_il + n_xw;
    for (int i = 0; i < 2; ++i) {
        p->off_ilw[i] = 0;
        if (!n_ilw[i]) continue;
        const uint32_t NT = 1024u >> i;
        const uint64_t D = 16ull * NT;
        p->off_ilw[i] = at;
        uint32_t* w = h.data() + at;
        build_pair_tables(w, D);
        const uint32_t xm128 = xpow8_inv(16);
        std::vector<uint32_t> Gt(NT);
        Gt[0] = kOne;
        for (uint32_t t = 1; t < NT; ++t) Gt[t] = gf_mul(Gt[t - 1], xm128);
        const uint64_t n_steps = (uint64_t)p->nseg * kDefaultBlocks;
        for (uint32_t r = 0; r < p->nseg; ++r) {
            const uint32_t F = gf_mul(gf_mul(xpow8(4096ull * (n_steps - 8ull * r - 7ull)), p->c_inv), c96);
            for (uint32_t t = 0; t < NT; ++t) w[kPairTabWords + (size_t)r * NT + t] = gf_mul(F, Gt[t]);
        }
        const uint32_t back = xpow8_inv(D - (uint64_t)kWgStride);
        for (int t = 0; t < kThreads; ++t)
            w[kPairTabWords + (size_t)p->nseg * NT + t] =
                gf_mul(h[n_old + kPairTabWords + (size_t)p->nseg * kThreads + t], back);
        at += n_ilw[i];
    }
    // k_decode_ilh (small launches; tuning arm 41): lane t of half unit u = 2 r + h takes the
    // sub-steps 8 r + 4 h + k (k < 4) at 16 t through A_4096; the constant
    // x^(8 (4096 (n_steps - st0 - 3) - 16 t)) c_inv x^(-96), st0 = 8 r + 4 h
    p->off_ilh = 0;
    if (n_ilh) {
        p->off_ilh = at;
        const int64_t n_steps = (int64_t)p->nseg * kDefaultBlocks;
        for (uint32_t uu = 0; uu < 2 * p->nseg; ++uu)
            for (int t = 0; t < kThreads; ++t) {
                const int64_t st0 = 8 * (int64_t)(uu >> 1) + 4 * (int64_t)(uu & 1u);
                const int64_t e = (int64_t)kWgStride * (n_steps - st0 - 3) - 16 * t;
                const uint32_t xe = e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)(-e));
                h[at + (size_t)uu * kThreads + t] = gf_mul(gf_mul(xe, p->c_inv), c96);
            }
        at += n_ilh;
    }
    for (int i = 0; i < 2; ++i) {  // S = 16 / 32
        p->off_il_s[i] = 0;
        if (!n_ils[i]) continue;
        p->off_il_s[i] = at;
        build_il(h.data() + at, 16u << i);
        at += n_ils[i];
    }
    if (p->d_tables) (void)hipFree(p->d_tables);
    p->d_tables = nullptr;
    HIP_TRY(hipMalloc(&p->d_tables, h.size() * sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(p->d_tables, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    if (p->tq >= 0) {
        // thread t's Horner state lands at rel_t = (64 + t/16)*sq + 16*(t%16) from the
        // tile base; shift every thread to REF, every tile from base+REF to R_c
        const uint64_t sq = p->sstride[p->tq];
        const uint64_t REF = (uint64_t)(kTileRows + 16) * sq + kTileCols;
        const uint32_t T = p->t_per_chunk;
        const std::vector<uint64_t> base = tile_bases(*p);
        const zhip_layout& L = p->layout;
        uint64_t maxb = 0;
        for (uint32_t ti = 0; ti < T; ++ti) maxb = std::max(maxb, base[ti]);
        const uint64_t Rc = maxb + REF;
        const bool t4 = p->tile4 != 0;
        const uint64_t step = p->tile4_step;
        const size_t n_base = 4096 + kThreads + T;
        const size_t n_t4 = t4 ? 1024 + (size_t)(T / 4) * kThreads + (size_t)T * 4 : 0;
        const size_t n_g = p->gd >= 0 ? 1024 + (size_t)p->n_groups * (sizeof(GroupEnt) / 4) : 0;
        // k_decode_tile4f: the four tiles of a group are the 256-byte pieces of
        // 1 KiB of every stored row (step 256), so thread t's blocks (row t/4,
        // 16 (t%4) + 64 n, n < 16) form one chain of stride 64 B
        const bool t4f = t4 && step == (uint64_t)kTileCols && (L.flags & ZHIP_LF_CRC);
        const size_t n_t4f = t4f ? kPairTabWords + (size_t)(T / 4) * kThreads : 0;
        // k_decode_tile4w: wave w of a workgroup owns tile w; lane l its rows
        // l/16 + 4 m (m < 16) at column block l % 16: one chain of stride 4 sq
        const bool t4w = t4 && (L.flags & ZHIP_LF_CRC);
        const size_t n_t4w = t4w ? kPairTabWords + (size_t)(T / 4) * kThreads : 0;
        // k_decode_tilegw: the same chains for the four tiles of a group
        const bool tgw = p->gd >= 0 && (L.flags & ZHIP_LF_CRC);
        const size_t n_tgw = tgw ? kPairTabWords + (size_t)p->n_groups * kThreads : 0;
        // the two-tile form of k_decode_tile4w (at most 32 workgroups per chunk:
        // the one-word publication): lane constants only
        const size_t n_t2w = (t4w && T % 2 == 0 && T / 2 <= 32) ? (size_t)(T / 2) * kThreads : 0;
        const size_t n_t1w = (ZHIP_TUNING && t4w) ? (size_t)T * kThreads : 0;  // one tile per workgroup
        // the two-tile form of k_decode_tilegw: two workgroups per group of four
        const size_t n_tg2w = tgw ? (size_t)p->n_groups * 2 * kThreads : 0;
        // the two-tile form of k_encode_tile4 (CRC, at most 32 workgroups per chunk)
        const size_t n_t2e = (t4 && (L.flags & ZHIP_LF_CRC) && T % 2 == 0 && T / 2 <= 32) ? (size_t)(T / 2) * kThreads : 0;
        // (tuning builds: the tile-pair decode, arm 39 -- 29.8-30.0 vs 29.2-29.4 us
        // for the grouped kernel on C3 in 128^3 chunks, profiles/r05/q/)
        const size_t n_t2 = (ZHIP_TUNING && p->tile2) ? kPairTabWords + (size_t)T * 4 + (size_t)(T / 2) * kThreads : 0;
        const size_t n_tgl = (ZHIP_TUNING && tgw) ? (size_t)p->n_groups * kThreads : 0;  // lane-tile form, arm 40
        // (tuning arms 66 / 67: A_(4 sq) as byte tables for the chains of the
        // two-tile forms)
        const size_t n_tbt = (ZHIP_TUNING && (t4w || tgw)) ? (size_t)kByteTabWords : 0;
        std::vector<uint32_t> ht(n_base + n_t4 + n_g + n_t4f + n_t4w + n_tgw + n_t2w + n_t1w + n_tg2w + n_t2e + n_t2 +
                                 n_tgl + n_tbt);
        build_horner_stride(ht.data(), 16ull * sq);
        for (int t = 0; t < kThreads; ++t) {
            const uint64_t rel = (uint64_t)(kTileRows + t / 16) * sq + 16u * (t % 16);
            ht[4096 + t] = xpow8(REF - rel);
        }
        for (uint32_t ti = 0; ti < T; ++ti) ht[4096 + kThreads + ti] = xpow8(Rc - base[ti] - REF);
        p->t_c_inv = xpow8_inv(Rc - L.nbytes);
        if (t4) {
            p->tile4_off_tz = n_base;
            p->tile4_off_kq = n_base + 1024;
            p->tile4_off_map = n_base + 1024 + (size_t)(T / 4) * kThreads;
            const uint32_t z = xpow8(step);
            for (int sl = 0; sl < 4; ++sl)
                for (uint32_t b = 0; b < 256; ++b) ht[p->tile4_off_tz + sl * 256 + b] = gf_mul(z, b << (8 * sl));
            for (uint32_t g4 = 0; g4 < T / 4; ++g4) {
                const uint32_t ku = gf_mul(ht[4096 + kThreads + 4 * g4 + 3], p->t_c_inv);
                for (int t = 0; t < kThreads; ++t)
                    ht[p->tile4_off_kq + (size_t)g4 * kThreads + t] = gf_mul(ht[4096 + t], ku);
            }
            // out offset of each tile relative to the chunk's out_off (full selection)
            for (uint32_t ti = 0; ti < T; ++ti) {
                uint32_t r = ti;
                const uint32_t cb = r % p->n_cb;
                r /= p->n_cb;
                const uint32_t qb = r % p->n_qb;
                r /= p->n_qb;
                int64_t o = (int64_t)qb * kTileRows * L.out_stride[p->tq] +
                            (int64_t)cb * (kTileCols / L.itemsize) * L.out_stride[L.ndim - 1];
                for (int d = L.ndim - 2; d >= 0; --d) {
                    if (d == p->tq) continue;
                    o += (int64_t)(r % (uint32_t)L.shape[d]) * L.out_stride[d];
                    r /= (uint32_t)L.shape[d];
                }
                uint32_t* e = &ht[p->tile4_off_map + 4ull * ti];
                e[0] = (uint32_t)base[ti];
                e[1] = 0;
                std::memcpy(e + 2, &o, sizeof(o));
            }
        }
        if (p->gd >= 0) {
            // groups: tiles whose gd coordinate is 4m .. 4m+3, others equal
            p->g_off_tz = n_base + n_t4;
            p->g_off_map = p->g_off_tz + 1024;
            const uint32_t z = xpow8(p->sstride[p->gd]);
            for (int sl = 0; sl < 4; ++sl)
                for (uint32_t b = 0; b < 256; ++b) ht[p->g_off_tz + sl * 256 + b] = gf_mul(z, b << (8 * sl));
            // tile-index stride of the gd coordinate (natural order: cb, qb, then
            // the other dims from ndim-2 down)
            uint64_t tstride = (uint64_t)p->n_cb * p->n_qb;
            for (int d = L.ndim - 2; d > p->gd; --d)
                if (d != p->tq) tstride *= (uint64_t)L.shape[d];
            GroupEnt* gm = reinterpret_cast<GroupEnt*>(&ht[p->g_off_map]);
            uint32_t g = 0;
            for (uint32_t ti = 0; ti < T; ++ti) {
                if ((ti / tstride) % (uint64_t)L.shape[p->gd] % 4u != 0u) continue;
                uint32_t r = ti;
                const uint32_t cb = r % p->n_cb;
                r /= p->n_cb;
                const uint32_t qb = r % p->n_qb;
                r /= p->n_qb;
                int64_t o = (int64_t)qb * kTileRows * L.out_stride[p->tq] +
                            (int64_t)cb * (kTileCols / L.itemsize) * L.out_stride[L.ndim - 1];
                for (int d = L.ndim - 2; d >= 0; --d) {
                    if (d == p->tq) continue;
                    o += (int64_t)(r % (uint32_t)L.shape[d]) * L.out_stride[d];
                    r /= (uint32_t)L.shape[d];
                }
                GroupEnt e{};
                e.tbase = (uint32_t)base[ti];
                e.rows = (uint16_t)std::min<int64_t>(kTileRows, (int64_t)L.shape[p->tq] - (int64_t)qb * kTileRows);
                e.cols = (uint16_t)std::min<int64_t>(kTileCols, (int64_t)p->row_bytes - (int64_t)cb * kTileCols);
                e.orel = o;
                e.ku = gf_mul(ht[4096 + kThreads + ti + 3 * tstride], p->t_c_inv);
                gm[g++] = e;
            }
        }
        p->tile4f = t4f ? 1u : 0u;
        p->tile4f_off = n_base + n_t4 + n_g;
        if (t4f) {
            // A_64 in the pair kernel's 11/11/10 layout; the lane constant (the
            // il kernel's frame, D = 64, 16 blocks) x^(8 (E - p_0 + 4096 - 16 * 64))
            // c_inv x^(-96) gives every word at p the pair kernel's
            // x^(8 (E - p + 4096)) c_inv (p_0: the lane's first block)
            uint32_t* f = &ht[p->tile4f_off];
            build_pair_tables(f, 64);
            const uint32_t c96 = xpow8_inv(12);
            for (uint32_t g4 = 0; g4 < T / 4; ++g4)
                for (int t = 0; t < kThreads; ++t) {
                    const int64_t p0 = (int64_t)base[4 * g4] + (int64_t)(t / 4) * (int64_t)sq + 16 * (t % 4);
                    const int64_t e = (int64_t)p->E - p0 + kWgStride - 16 * 64;
                    const uint32_t xe = e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)(-e));
                    f[kPairTabWords + (size_t)g4 * kThreads + t] = gf_mul(gf_mul(xe, p->c_inv), c96);
                }
        }
        p->tile4w = t4w ? 1u : 0u;
        p->tile4w_off = n_base + n_t4 + n_g + n_t4f;
        if (t4w) {
            // A_(4 sq); lane constant (the il frame, D = 4 sq, 16 blocks)
            // x^(8 (E - p_0 + 4096 - 16 D)) c_inv x^(-96), p_0 = base[4 g + w] +
            // (l / 16) sq + 16 (l % 16) for thread t = 64 w + l
            uint32_t* f = &ht[p->tile4w_off];
            const uint64_t D = 4ull * sq;
            build_pair_tables(f, D);
            const uint32_t c96 = xpow8_inv(12);
            for (uint32_t g4 = 0; g4 < T / 4; ++g4)
                for (int t = 0; t < kThreads; ++t) {
                    const int w = t / 64, l = t % 64;
                    const int64_t p0 = (int64_t)base[4 * g4 + w] + (int64_t)(l / 16) * (int64_t)sq + 16 * (l % 16);
                    const int64_t e = (int64_t)p->E - p0 + kWgStride - 16 * (int64_t)D;
                    const uint32_t xe = e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)(-e));
                    f[kPairTabWords + (size_t)g4 * kThreads + t] = gf_mul(gf_mul(xe, p->c_inv), c96);
                }
        }
        p->tile2w_off = 0;
        if (n_t2w) {
            // two tiles per workgroup: wave w loads rows 32 (w % 2) + l/16 + 4 m (m < 8)
            // of tile 2 g + w / 2; the same frame with 8 blocks of stride D = 4 sq
            p->tile2w_off = n_base + n_t4 + n_g + n_t4f + n_t4w + n_tgw;
            uint32_t* f = &ht[p->tile2w_off];
            const uint64_t D = 4ull * sq;
            const uint32_t c96 = xpow8_inv(12);
            for (uint32_t g2 = 0; g2 < T / 2; ++g2)
                for (int t = 0; t < kThreads; ++t) {
                    const int w = t / 64, l = t % 64;
                    const int64_t p0 = (int64_t)base[2 * g2 + w / 2] + (int64_t)(32 * (w % 2) + l / 16) * (int64_t)sq +
                                       16 * (l % 16);
                    const int64_t e = (int64_t)p->E - p0 + kWgStride - 8 * (int64_t)D;
                    const uint32_t xe = e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)(-e));
                    f[(size_t)g2 * kThreads + t] = gf_mul(gf_mul(xe, p->c_inv), c96);
                }
        }
        p->tile1w_off = 0;
        if (n_t1w) {
            // one tile per workgroup: wave w loads rows 16 w + l/16 + 4 m (m < 4)
            p->tile1w_off = n_base + n_t4 + n_g + n_t4f + n_t4w + n_tgw + n_t2w;
            uint32_t* f = &ht[p->tile1w_off];
            const uint64_t D = 4ull * sq;
            const uint32_t c96 = xpow8_inv(12);
            for (uint32_t ti = 0; ti < T; ++ti)
                for (int t = 0; t < kThreads; ++t) {
                    const int w = t / 64, l = t % 64;
                    const int64_t p0 = (int64_t)base[ti] + (int64_t)(16 * w + l / 16) * (int64_t)sq + 16 * (l % 16);
                    const int64_t e = (int64_t)p->E - p0 + kWgStride - 4 * (int64_t)D;
                    const uint32_t xe = e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)(-e));
                    f[(size_t)ti * kThreads + t] = gf_mul(gf_mul(xe, p->c_inv), c96);
                }
        }
        p->tileg2w_off = 0;
        if (n_tg2w) {
            // workgroup 2 g + h of a chunk: tiles 2 h, 2 h + 1 of group g, wave w loading
            // rows 32 (w % 2) + l/16 + 4 m (m < 8) of tile 2 h + w / 2
            p->tileg2w_off = n_base + n_t4 + n_g + n_t4f + n_t4w + n_tgw + n_t2w + n_t1w;
            uint32_t* f = &ht[p->tileg2w_off];
            const uint64_t D = 4ull * sq;
            const uint32_t c96 = xpow8_inv(12);
            const GroupEnt* gm = reinterpret_cast<const GroupEnt*>(&ht[p->g_off_map]);
            const int64_t gstep = (int64_t)p->sstride[p->gd];
            for (uint32_t g = 0; g < p->n_groups; ++g)
                for (uint32_t h = 0; h < 2; ++h)
                    for (int t = 0; t < kThreads; ++t) {
                        const int w = t / 64, l = t % 64;
                        const int64_t p0 = (int64_t)gm[g].tbase + (int64_t)(2 * h + w / 2) * gstep +
                                           (int64_t)(32 * (w % 2) + l / 16) * (int64_t)sq + 16 * (l % 16);
                        const int64_t e = (int64_t)p->E - p0 + kWgStride - 8 * (int64_t)D;
                        const uint32_t xe = e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)(-e));
                        f[((size_t)g * 2 + h) * kThreads + t] = gf_mul(gf_mul(xe, p->c_inv), c96);
                    }
        }
        p->tile2e_off = 0;
        if (n_t2e) {
            // the four-tile constants' form for groups of two: the state carried
            // to the group's last tile (tile 2 g + 1), then shifted by its unit constant
            p->tile2e_off = n_base + n_t4 + n_g + n_t4f + n_t4w + n_tgw + n_t2w + n_t1w + n_tg2w;
            for (uint32_t g2 = 0; g2 < T / 2; ++g2) {
                const uint32_t ku = gf_mul(ht[4096 + kThreads + 2 * g2 + 1], p->t_c_inv);
                for (int t = 0; t < kThreads; ++t)
                    ht[p->tile2e_off + (size_t)g2 * kThreads + t] = gf_mul(ht[4096 + t], ku);
            }
        }
        p->tile2_off = 0;
        if (n_t2) {
            p->tile2_off = n_base + n_t4 + n_g + n_t4f + n_t4w + n_tgw + n_t2w + n_t1w + n_tg2w + n_t2e;
            uint32_t* f = &ht[p->tile2_off];
            const uint64_t D = 4ull * sq;
            build_pair_tables(f, D);
            // tile map (as tile4's): stored base, out offset relative to the chunk's out_off
            for (uint32_t ti = 0; ti < T; ++ti) {
                uint32_t r = ti;
                const uint32_t cb = r % p->n_cb;
                r /= p->n_cb;
                const uint32_t qb = r % p->n_qb;
                r /= p->n_qb;
                int64_t o = (int64_t)qb * kTileRows * L.out_stride[p->tq] +
                            (int64_t)cb * (kTileCols / L.itemsize) * L.out_stride[L.ndim - 1];
                for (int d = L.ndim - 2; d >= 0; --d) {
                    if (d == p->tq) continue;
                    o += (int64_t)(r % (uint32_t)L.shape[d]) * L.out_stride[d];
                    r /= (uint32_t)L.shape[d];
                }
                uint32_t* e = &f[kPairTabWords + 4ull * ti];
                e[0] = (uint32_t)base[ti];
                e[1] = 0;
                std::memcpy(e + 2, &o, sizeof(o));
            }
            // lane constants: wave w of pair g loads rows 32 (w % 2) + l/16 + 4 m (m < 8) of tile 2 g + w / 2
            const uint32_t c96 = xpow8_inv(12);
            uint32_t* kc = f + kPairTabWords + (size_t)T * 4;
            for (uint32_t g2 = 0; g2 < T / 2; ++g2)
                for (int t = 0; t < kThreads; ++t) {
                    const int w = t / 64, l = t % 64;
                    const int64_t p0 = (int64_t)base[2 * g2 + w / 2] + (int64_t)(32 * (w % 2) + l / 16) * (int64_t)sq +
                                       16 * (l % 16);
                    const int64_t e = (int64_t)p->E - p0 + kWgStride - 8 * (int64_t)D;
                    const uint32_t xe = e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)(-e));
                    kc[(size_t)g2 * kThreads + t] = gf_mul(gf_mul(xe, p->c_inv), c96);
                }
        }
        p->tilegl_off = 0;
        if (n_tgl) {
            // lane l of wave w: rows w + 4 m (m < 16) of tile l / 16 at column block l % 16
            p->tilegl_off = n_base + n_t4 + n_g + n_t4f + n_t4w + n_tgw + n_t2w + n_t1w + n_tg2w + n_t2e + n_t2;
            uint32_t* f = &ht[p->tilegl_off];
            const uint64_t D = 4ull * sq;
            const uint32_t c96 = xpow8_inv(12);
            const GroupEnt* gm = reinterpret_cast<const GroupEnt*>(&ht[p->g_off_map]);
            const int64_t gstep = (int64_t)p->sstride[p->gd];
            for (uint32_t g = 0; g < p->n_groups; ++g)
                for (int t = 0; t < kThreads; ++t) {
                    const int w = t / 64, l = t % 64;
                    const int64_t p0 = (int64_t)gm[g].tbase + (int64_t)(l / 16) * gstep + (int64_t)w * (int64_t)sq +
                                       16 * (l % 16);
                    const int64_t e = (int64_t)p->E - p0 + kWgStride - 16 * (int64_t)D;
                    const uint32_t xe = e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)(-e));
                    f[(size_t)g * kThreads + t] = gf_mul(gf_mul(xe, p->c_inv), c96);
                }
        }
        p->tilebt_off = 0;
        if (n_tbt) {
            p->tilebt_off = n_base + n_t4 + n_g + n_t4f + n_t4w + n_tgw + n_t2w + n_t1w + n_tg2w + n_t2e + n_t2 + n_tgl;
            uint32_t* f = &ht[p->tilebt_off];
            const uint32_t x = xpow8(4ull * sq), x4 = xpow8(4);
            for (int sl = 0; sl < 4; ++sl)
                for (uint32_t b = 0; b < 256; ++b) {
                    f[sl * 256 + b] = gf_mul(x, b << (8 * sl));
                    f[1024 + sl * 256 + b] = gf_mul(x4, b << (8 * sl));
                }
        }
        p->tilegw = tgw ? 1u : 0u;
        p->tilegw_off = n_base + n_t4 + n_g + n_t4f + n_t4w;
        if (tgw) {
            // as k_decode_tile4w, tile w of group g at gm[g].tbase + w step(gd)
            uint32_t* f = &ht[p->tilegw_off];
            const uint64_t D = 4ull * sq;
            build_pair_tables(f, D);
            const uint32_t c96 = xpow8_inv(12);
            const GroupEnt* gm = reinterpret_cast<const GroupEnt*>(&ht[p->g_off_map]);
            const int64_t gstep = (int64_t)p->sstride[p->gd];
            for (uint32_t g = 0; g < p->n_groups; ++g)
                for (int t = 0; t < kThreads; ++t) {
                    const int w = t / 64, l = t % 64;
                    const int64_t p0 = (int64_t)gm[g].tbase + w * gstep + (int64_t)(l / 16) * (int64_t)sq +
                                       16 * (l % 16);
                    const int64_t e = (int64_t)p->E - p0 + kWgStride - 16 * (int64_t)D;
                    const uint32_t xe = e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)(-e));
                    f[kPairTabWords + (size_t)g * kThreads + t] = gf_mul(gf_mul(xe, p->c_inv), c96);
                }
        }
        if (p->d_tile_tables) (void)hipFree(p->d_tile_tables);
        p->d_tile_tables = nullptr;
        HIP_TRY(hipMalloc(&p->d_tile_tables, ht.size() * sizeof(uint32_t)));
        HIP_TRY(hipMemcpy(p->d_tile_tables, ht.data(), ht.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
        p->max_grid = prop.multiProcessorCount * 8;
    p->device = dev;
    return ZHIP_OK;
}

int zhip_plan_destroy(zhip_plan* p) {
    if (!p) return ZHIP_OK;
    if (p->d_tables) (void)hipFree(p->d_tables);
    if (p->d_tile_tables) (void)hipFree(p->d_tile_tables);
    delete p;
    return ZHIP_OK;
}

int zhip_plan_kernel_flags(const zhip_plan* p, uint32_t* flags) {
    if (!p || !flags) return set_err(ZHIP_E_INVALID, "null argument");
    *flags = (p->tile4 ? ZHIP_PK_TILE4 : 0u) | (p->tile4 && p->t_per_chunk <= 64 ? ZHIP_PK_TILE4_ENCODE : 0u) |
             (p->tq >= 0 ? ZHIP_PK_TILE : 0u) |
             (p->gd >= 0 && p->layout.shape[p->tq] % (16 / p->layout.itemsize) == 0 ? ZHIP_PK_TILEG : 0u) |
             (p->il_S == 8u && (p->layout.flags & ZHIP_LF_CRC) ? ZHIP_PK_IL : 0u);
    return ZHIP_OK;
}

int zhip_plan_info(const zhip_plan* p, uint32_t* units_per_chunk, uint32_t* workspace_words) {
    if (!p) return set_err(ZHIP_E_INVALID, "null plan");
    if (units_per_chunk) *units_per_chunk = p->nseg;
    // + the grouped kernels' / k_decode_xw's arrival subwords
    // (CRC layouts: >= kPubLine, the il / tile4 publication lines)
    // (k_decode_tilegw's two-tile form: arrival subwords for twice the groups)
    // (known at plan creation, before the tile tables exist)
    const bool tg2w = p->gd >= 0 && (p->layout.flags & ZHIP_LF_CRC);
    uint32_t n_sub2 = (tg2w && 2 * p->n_groups > 16u && 2 * p->n_groups <= 256u)
                          ? (2 * p->n_groups + 15u) / 16u : 0u;
    // (the tile-pair decode, tuning builds: subwords of 16 for 33..256 workgroups per chunk)
    const uint32_t wpc2 = (ZHIP_TUNING && p->tile2) ? p->t_per_chunk / 2u : 0u;
    if (wpc2 > 32u && wpc2 <= 256u) n_sub2 = std::max(n_sub2, (wpc2 + 15u) / 16u);
    // (k_decode_tile4w, four tiles per workgroup: the same subwords past 32 workgroups per chunk)
    const uint32_t wpc4 = (p->tile4 && (p->layout.flags & ZHIP_LF_CRC)) ? p->t_per_chunk / 4u : 0u;
    if (wpc4 > 32u && wpc4 <= 256u) n_sub2 = std::max(n_sub2, (wpc4 + 15u) / 16u);
    uint32_t w = std::max(4 + 2 * std::max(std::max(p->n_sub, p->xw_nsub), n_sub2),
                          (p->layout.flags & ZHIP_LF_CRC) ? kPubLine : 0u);
    // (k_decode_tilegw's two-tile form, tuning arm 47's k_encode_tileg: the
    // arrival words on 128-byte lines of their own, tileg_arrive SPR)
    if (tg2w) w = std::max(w, kPubLine * (1u + (ZHIP_TUNING ? std::max(p->n_sub, n_sub2) : n_sub2)));
    // (tuning arm 49: k_decode_il / k_decode_ilw / two-tile k_decode_tile4w publish
    // through two subwords on lines of their own)
    if (ZHIP_TUNING && (p->layout.flags & ZHIP_LF_CRC) && (p->il_S || p->tile4)) w = std::max(w, 3u * kPubLine);
    // (tuning arm 39, tile pairs past 32 workgroups per chunk: spread subwords)
    if (wpc2 > 32u && wpc2 <= 256u) w = std::max(w, kPubLine * (1u + (wpc2 + 15u) / 16u));
    if (workspace_words) *workspace_words = w;
    return ZHIP_OK;
}

int zhip_decode(const zhip_plan* plan, const void* src, uint64_t src_size, void* out,
                const zhip_chunk* d_chunks, uint32_t n_chunks, const zhip_sel* d_sels,
                zhip_status* d_status, uint32_t* d_workspace, uint32_t* d_errflag, uint32_t decode_flags,
                void* stream) {
    return zhip_decode_indexed(plan, src, src_size, out, d_chunks, n_chunks, d_sels, d_status, d_workspace,
                               d_errflag, nullptr, 0, nullptr, decode_flags, stream);
}

int zhip_decode_indexed(const zhip_plan* plan, const void* src, uint64_t src_size, void* out,
                        const zhip_chunk* d_chunks, uint32_t n_chunks, const zhip_sel* d_sels,
                        zhip_status* d_status, uint32_t* d_workspace, uint32_t* d_errflag,
                        const zhip_chunk* d_index_chunks, uint32_t n_index, zhip_status* d_index_status,
                        uint32_t decode_flags, void* stream) {
    return zhip_decode_predicted(plan, src, src_size, out, d_chunks, n_chunks, d_sels, d_status, d_workspace,
                                 d_errflag, d_index_chunks, n_index, d_index_status, decode_flags, nullptr, stream);
}

int zhip_decode_predicted(const zhip_plan* plan, const void* src, uint64_t src_size, void* out,
                          const zhip_chunk* d_chunks, uint32_t n_chunks, const zhip_sel* d_sels,
                          zhip_status* d_status, uint32_t* d_workspace, uint32_t* d_errflag,
                          const zhip_chunk* d_index_chunks, uint32_t n_index, zhip_status* d_index_status,
                          uint32_t decode_flags, const zhip_predict* pred, void* stream) {
    return zhip_decode_mapped(plan, src, src_size, out, d_chunks, n_chunks, d_sels, d_status, d_workspace,
                              d_errflag, d_index_chunks, n_index, d_index_status, decode_flags, pred, nullptr,
                              stream);
}

uint64_t zhip_rows_map_len(const zhip_plan* plan, uint32_t n_sels) {
    if (!plan) return 0;
    return (uint64_t)n_sels * plan->nseg * (uint64_t)kDefaultBlocks;
}

// The destination arithmetic of the row decode (per step: row R of the
// chunk's flattened leading dims, its place in dims 0..ndim-2 and in the
// selection), evaluated once per (selection, unit, step) on the host.
// Entry of the row map for the step whose first output byte is base_o
// (>= 0) of the chunk: 0 ok (e set, possibly empty), 1 offset beyond 32 bits.
static int rows_entry(const zhip_layout& L, uint32_t shift, const zhip_sel& sel, int64_t base_o, zhip_rowblk& e) {
    const int nd = L.ndim, nd2 = nd - 2;
    const int64_t rps = (int64_t)kWgStride >> shift;  // rows per step
    const int64_t sy = L.shape[nd - 2];
    const int64_t oy = L.out_stride[nd - 2];
    const int64_t sy0 = sel.start[nd2], cy = sel.count[nd2];
    e.rel = 0;
    e.lo = e.hi = 0;
    const int64_t R = base_o >> shift;
    int64_t r = R / sy;
    const int64_t y0 = R - r * sy;
    int64_t dst = (y0 - sy0) * oy;
    bool ok = true;
    for (int d = nd2 - 1; d >= 0; --d) {
        const int64_t qd = d > 0 ? r / L.shape[d] : 0;
        const int64_t rel = r - qd * L.shape[d] - sel.start[d];
        r = qd;
        ok = ok && rel >= 0 && rel < sel.count[d];
        dst += rel * L.out_stride[d];
    }
    const int64_t lo = std::min(std::max(sy0 - y0, (int64_t)0), rps);
    const int64_t hi = std::min(std::max(sy0 - y0 + cy, (int64_t)0), rps);
    if (!ok || hi <= lo) return 0;
    if (dst < INT32_MIN || dst > INT32_MAX) return 1;
    e.rel = (int32_t)dst;
    e.lo = (uint16_t)lo;
    e.hi = (uint16_t)hi;
    return 0;
}

static bool rows_layout(const zhip_plan* plan) {  // zhip_rows_map's admission
    const zhip_layout& L = plan->layout;
    const uint32_t rb = plan->row_bytes;
    const int nd = L.ndim;
    return !(nd < 2 || rb < 16 || rb > (uint32_t)kWgStride || (rb & (rb - 1)) != 0 ||
             (uint32_t)L.shape[nd - 2] % ((uint32_t)kWgStride / rb) != 0 ||
             plan->seg != (uint32_t)kWgStride * kDefaultBlocks);
}

// The whole-chunk selection's row map in two-level affine form (ZHIP_DF_WHOLE
// launches): rel(st) = (st >> sh) B + (st & (2^sh - 1)) C + D with every row
// of every step written, st = (base_o - lo_frame) / 4 KiB; only chunks that
// end on a unit boundary (lo_frame 0).  aff_ok = 0 when no shift fits.
static void plan_affine(zhip_plan* p) {
    p->aff_ok = 0;
    if (!rows_layout(p) || p->E != p->nseg * p->seg || p->nseg == 0) return;
    const zhip_layout& L = p->layout;
    const uint32_t shift = (uint32_t)__builtin_ctz(p->row_bytes);
    const uint16_t rps = (uint16_t)((uint32_t)kWgStride >> shift);
    zhip_sel full{};
    for (int d = 0; d < L.ndim; ++d) full.count[d] = (int32_t)L.shape[d];
    const uint32_t n_st = p->nseg * (uint32_t)kDefaultBlocks;
    std::vector<int32_t> rel(n_st);
    for (uint32_t st = 0; st < n_st; ++st) {
        zhip_rowblk e;
        if (rows_entry(L, shift, full, (int64_t)kWgStride * st, e) || e.lo != 0 || e.hi != rps) return;
        rel[st] = e.rel;
    }
    for (uint32_t sh = 0; sh <= 12; ++sh) {
        const uint32_t mask = (1u << sh) - 1u;
        const int64_t D = rel[0];
        const int64_t C = (sh > 0 && n_st > 1) ? (int64_t)rel[1] - D : 0;
        const int64_t B = ((1u << sh) < n_st) ? (int64_t)rel[1u << sh] - D : 0;
        bool fit = true;
        for (uint32_t st = 0; st < n_st && fit; ++st)
            fit = (int64_t)(st >> sh) * B + (int64_t)(st & mask) * C + D == rel[st];
        if (fit && B >= INT32_MIN && B <= INT32_MAX && C >= INT32_MIN && C <= INT32_MAX) {
            p->aff_ok = 1;
            p->aff_sh = sh;
            p->aff_B = (int32_t)B;
            p->aff_C = (int32_t)C;
            p->aff_D = (int32_t)D;
            return;
        }
    }
}

extern "C++" {
template <class P>
static void set_affine(P& p, const zhip_plan* plan) {  // DecodeParams / EncodeParams
    p.aff_sh = plan->aff_sh;
    p.aff_mask = (1u << plan->aff_sh) - 1u;
    p.aff_B = plan->aff_B;
    p.aff_C = plan->aff_C;
    p.aff_D = plan->aff_D;
}
}

int zhip_rows_map(const zhip_plan* plan, const zhip_sel* h_sels, uint32_t n_sels, zhip_rowblk* h_map,
                  uint64_t map_len) {
    if (!plan) return set_err(ZHIP_E_INVALID, "null plan");
    if (n_sels && (!h_sels || !h_map)) return set_err(ZHIP_E_INVALID, "null host pointer");
    if (map_len < zhip_rows_map_len(plan, n_sels)) return set_err(ZHIP_E_INVALID, "row map too short");
    if (!rows_layout(plan)) return set_err(ZHIP_E_UNSUPPORTED, "not a whole-row layout with 32 KiB units");
    const zhip_layout& L = plan->layout;
    const uint32_t shift = (uint32_t)__builtin_ctz(plan->row_bytes);
    for (uint32_t s = 0; s < n_sels; ++s) {
        for (uint32_t u = 0; u < plan->nseg; ++u) {
            const int64_t seg_lo = (int64_t)(int32_t)plan->E - (int64_t)(u + 1) * plan->seg;
            for (int k = 0; k < kDefaultBlocks; ++k) {
                zhip_rowblk& e = h_map[((uint64_t)s * plan->nseg + u) * kDefaultBlocks + k];
                e.rel = 0;
                e.lo = e.hi = 0;
                const int64_t base_o = seg_lo + (int64_t)kWgStride * k;
                if (base_o < 0) continue;  // before the chunk start: nothing written
                if (rows_entry(L, shift, h_sels[s], base_o, e))
                    return set_err(ZHIP_E_UNSUPPORTED, "row offset does not fit 32 bits");
            }
        }
    }
    return ZHIP_OK;
}

int zhip_decode_mapped(const zhip_plan* plan, const void* src, uint64_t src_size, void* out,
                       const zhip_chunk* d_chunks, uint32_t n_chunks, const zhip_sel* d_sels,
                       zhip_status* d_status, uint32_t* d_workspace, uint32_t* d_errflag,
                       const zhip_chunk* d_index_chunks, uint32_t n_index, zhip_status* d_index_status,
                       uint32_t decode_flags, const zhip_predict* pred, const zhip_rowblk* d_rowmap,
                       void* stream) {
    if (!plan) return set_err(ZHIP_E_INVALID, "null plan");
    if (!plan->d_tables) return set_err(ZHIP_E_INVALID, "plan not uploaded (zhip_plan_upload)");
    if (n_chunks == 0 && n_index == 0) return ZHIP_OK;
    if (!src || !d_chunks || !d_sels || !d_status || !d_workspace || !d_errflag)
        return set_err(ZHIP_E_INVALID, "null device pointer");
    if (n_index) {
        if (!d_index_chunks || !d_index_status) return set_err(ZHIP_E_INVALID, "null index pointer");
        // inner chunks without a CRC: only the mapped pair decode carries the
        // index checks (k_decode_lead, leading workgroups)
        const bool lead_ok = d_rowmap && (decode_flags & ZHIP_DF_ROWS) && (decode_flags & ZHIP_DF_FAST_ROWS) &&
                             plan->nseg <= 32u && plan->seg == (uint32_t)kWgStride * kDefaultBlocks;
        if (!(plan->layout.flags & ZHIP_LF_SHARDED) || (!(plan->layout.flags & ZHIP_LF_CRC) && !lead_ok) ||
            (decode_flags & ZHIP_DF_TILE) || plan->idx_nbytes == 0)
            return set_err(ZHIP_E_UNSUPPORTED, "index check cannot be fused for this plan");
    }
    const zhip_layout& L = plan->layout;
    if (!(L.flags & ZHIP_LF_NO_WRITE) && !out) return set_err(ZHIP_E_INVALID, "null out");
    const uint64_t units = (uint64_t)n_chunks * plan->nseg;
    if (units >= (1ull << 32)) return set_err(ZHIP_E_UNSUPPORTED, "too many units in one batch");
    DecodeParams p{};
    p.src = static_cast<const uint8_t*>(src);
    p.src_size = src_size;
    p.out = static_cast<uint8_t*>(out);
    p.chunks = d_chunks;
    p.sels = d_sels;
    p.status = d_status;
    p.ws = d_workspace;
    p.errflag = d_errflag;
    p.horner = plan->d_tables;
    p.kthread = plan->d_tables + 4096;
    p.kunit = plan->d_tables + 4096 + kThreads;
    p.kpair = plan->d_tables + 4096 + kThreads + plan->nseg;
    p.pair_tab = plan->d_tables + plan->off_pair;
    p.kpair11 = p.pair_tab + kPairTabWords;
    p.kthread11 = p.kpair11 + (size_t)plan->nseg * kThreads;
    // k_decode_il needs its tables, and a fused index check of one step per lane
    p.il_S = (plan->il_S && (n_index == 0 || plan->idx_E <= (uint32_t)kWgStride)) ? plan->il_S : 0u;
    // the widest interleave the plan built (S = 32, else 16, else 8); tuning
    // arms 69 / 70 / 71 force 16 / 32 / 8
    int si = plan->off_il_s[1] ? 1 : plan->off_il_s[0] ? 0 : -1;
#if ZHIP_TUNING
    if (g_tune_arm == 69) si = plan->off_il_s[0] ? 0 : -1;
    if (g_tune_arm == 70) si = plan->off_il_s[1] ? 1 : -1;
    if (g_tune_arm == 71) si = -1;
#endif
    if (p.il_S && si >= 0) {  // groups of 16 / 32 workgroups: the plan's second / third table set
        p.il_S = 16u << si;
        p.il_tab = plan->d_tables + plan->off_il_s[si];
        p.il_klane = p.il_tab + kPairTabWords;
        p.il_kidx = p.il_klane + (size_t)plan->nseg * kThreads;
        p.il_basis = p.il_kidx + kThreads;
    } else if (p.il_S) {
        p.il_tab = plan->d_tables + plan->off_il;
        p.il_klane = p.il_tab + kPairTabWords;
        p.il_kidx = p.il_klane + (size_t)plan->nseg * kThreads;
        p.il_basis = p.il_kidx + kThreads;
    }
    p.xw = (plan->xw_P && (n_index == 0 || plan->idx_E <= (uint32_t)kWgStride)) ? plan->xw_P : 0u;
    if (p.xw) {
        p.xw_nsub = plan->xw_nsub;
        p.xw_tab = plan->d_tables + plan->off_xw;
        p.xw_klane = p.xw_tab + kPairTabWords;
        p.xw_kidx = p.xw_klane + (size_t)plan->xw_P * 64;
    }
    // k_decode_ilw: 512 lanes per unit for grids of at most kIlwMaxUnits
    // units (launch_decode; tuning arms 26 / 31 force 1024 lanes, 27 / 32 512)
    {
        int wi = (n_index == 0 || plan->idx_E <= (uint32_t)kWgStride) && units <= kIlwMaxUnits ? 1 : -1;
#if ZHIP_TUNING
        if (g_tune_arm == 26 || g_tune_arm == 31) wi = 0;
        else if (g_tune_arm == 27 || g_tune_arm == 32 || g_tune_arm == 42) wi = 1;
        if (((g_tune_arm >= 26 && g_tune_arm <= 32) || g_tune_arm == 42) &&
            !(n_index == 0 || plan->idx_E <= (uint32_t)kWgStride)) wi = -1;
#endif
        p.ilw_nt = (wi >= 0 && plan->off_ilw[wi]) ? (1024u >> wi) : 0u;
        if (p.ilw_nt) {
            p.ilw_tab = plan->d_tables + plan->off_ilw[wi];
            p.ilw_klane = p.ilw_tab + kPairTabWords;
            p.ilw_kidx = p.ilw_klane + (size_t)plan->nseg * p.ilw_nt;
        }
    }
    if (plan->off_ilh) p.ilh_klane = plan->d_tables + plan->off_ilh;
    // whole-chunk selections (ZHIP_DF_WHOLE, with a row map) of a plan whose
    // whole-chunk row map is affine: the row kernels compute destinations
    // (tuning arm 45 keeps the map loads: the A/B reference)
    p.aff_ok = (decode_flags & ZHIP_DF_WHOLE) && (decode_flags & ZHIP_DF_ROWS) && d_rowmap && plan->aff_ok &&
               !(ZHIP_TUNING && g_tune_arm == 45);
    if (p.aff_ok) set_affine(p, plan);
    for (int op = 0; op < 4; ++op) p.hx[op] = plan->hx[op];
    for (int i = 0; i < 32; ++i) p.kq[i] = plan->kq[i];
    p.n_chunks = n_chunks;
    p.nseg = plan->nseg;
    p.n_units = (uint32_t)units;
    p.n_idx = n_index;
    p.idx_chunks = d_index_chunks;
    p.idx_status = d_index_status;
    p.idx_nbytes = plan->idx_nbytes;
    p.idx_E = plan->idx_E;
    p.idx_c_inv = plan->idx_c_inv;
    p.idx_c3 = plan->idx_c3;
    p.c_inv = plan->c_inv;
    p.c3 = plan->c3;
    p.lflags = L.flags;
    fill_geom(p.g, *plan);
    p.seg = plan->seg;
    p.E = plan->E;
    p.index_size = L.index_size;
    p.n_inner = L.n_inner;
    std::memcpy(p.fill, plan->fill, sizeof(p.fill));
    p.fast = (decode_flags & ZHIP_DF_FAST_ROWS) ? 1u : 0u;
    p.dv_bank = (decode_flags & ZHIP_DF_BANK1) ? 1u : 0u;
    p.defer = (decode_flags & ZHIP_DF_DEFER) ? 1u : 0u;
    p.tune = g_tune_bits;
    p.tq = -1;
    p.rows = 0;
    p.rowmap = nullptr;
    p.pred = 0;
    if (decode_flags & ZHIP_DF_ROWS) {
        const uint32_t rb = plan->row_bytes;
        const int nd = L.ndim;
        const bool pow2 = rb >= 16 && rb <= (uint32_t)kWgStride && (rb & (rb - 1)) == 0;
        if (!(decode_flags & ZHIP_DF_FAST_ROWS) || (decode_flags & ZHIP_DF_TILE) || nd < 2 || !pow2 ||
            (L.flags & ZHIP_LF_NO_WRITE) || (uint32_t)L.shape[nd - 2] % ((uint32_t)kWgStride / rb) != 0)
            return set_err(ZHIP_E_INVALID, "ZHIP_DF_ROWS preconditions do not hold for this layout");
        p.rows = 1;
        p.rowmap = d_rowmap;
        if (pred) {
            if (pred->per == 0) return set_err(ZHIP_E_INVALID, "zhip_predict.per must be >= 1");
            // every predicted unit range must lie inside src (the kernel reads it before checking)
            const uint64_t last = n_chunks ? (uint64_t)(n_chunks - 1) : 0;
            const uint64_t gl = last / pred->per;
            uint64_t top = gl * pred->outer + (last % pred->per) * pred->inner;
            if (gl >= 1) {
                const uint64_t full = (gl - 1) * pred->outer + (uint64_t)(pred->per - 1) * pred->inner;
                if (full > top) top = full;
            }
            const uint64_t hi = pred->base + top + plan->E;
            if (n_chunks && hi > src_size) return set_err(ZHIP_E_INVALID, "zhip_predict range outside src");
            p.pred = 1;
            p.pred_base = pred->base;
            p.pred_outer = pred->outer;
            p.pred_inner = pred->inner;
            p.pred_per = pred->per;
        }
        p.row_shift = (uint32_t)__builtin_ctz(rb);
        p.r_sy = (uint32_t)L.shape[nd - 2];
        p.r_dy = make_fdiv(p.r_sy);
        p.r_oy = L.out_stride[nd - 2];
        p.nd2 = nd - 2;
    }
    if ((decode_flags & ZHIP_DF_TILE) && plan->tq >= 0 && plan->d_tile_tables) {
        p.tq = plan->tq;
        p.t_per_chunk = plan->t_per_chunk;
        p.n_qb = plan->n_qb;
        p.n_cb = plan->n_cb;
        for (int d = 0; d < ZHIP_MAX_DIMS; ++d) p.sstride[d] = plan->sstride[d];
        p.d_qb = make_fdiv(plan->n_qb);
        p.d_cb = make_fdiv(plan->n_cb);
        p.horner = plan->d_tile_tables;
        p.kthread = plan->d_tile_tables + 4096;
        p.kunit = plan->d_tile_tables + 4096 + kThreads;
        p.c_inv = plan->t_c_inv;
        p.tile4 = plan->tile4 && !(g_tune_bits & (kTuneTile1 | kTuneNoTile4));
        if (p.tile4) {
            p.tz = plan->d_tile_tables + plan->tile4_off_tz;
            p.kq4 = plan->d_tile_tables + plan->tile4_off_kq;
            p.tmap = reinterpret_cast<const TileEnt*>(plan->d_tile_tables + plan->tile4_off_map);
            if (plan->tile4f && (g_tune_bits & kTuneTile4F)) {  // arm: measured 0.3-0.4 us slower on C3
                p.t4f_tab = plan->d_tile_tables + plan->tile4f_off;
                p.t4f_kq = p.t4f_tab + kPairTabWords;
            } else if (plan->tile4w && g_tune_arm != 1 && g_tune_arm != 2 && g_tune_arm != 5) {
                // production for CRC layouts: a wave per tile, one chain per lane (k_decode_tile4w:
                // C3 28.9 vs 30.3-30.6 us, profiles/r04/k); arms 1 / 2 / 5: k_decode_tile4
                p.t4w_tab = plan->d_tile_tables + plan->tile4w_off;
                p.t4w_kq = p.t4w_tab + kPairTabWords;
                if (plan->tilebt_off) p.tbt_tab = plan->d_tile_tables + plan->tilebt_off;
                if (plan->tile2w_off) p.t2w_kq = plan->d_tile_tables + plan->tile2w_off;
                if (plan->tile1w_off) p.t1w_kq = plan->d_tile_tables + plan->tile1w_off;
            }
        } else if (plan->tile2 && plan->tile2_off && !(g_tune_bits & kTuneTile1) && g_tune_arm == 39) {
            // consecutive tile pairs (k_decode_tile4w<2>) where tile4 declines
            // (tuning arm 39; the grouped kernels are faster)
            p.tile2 = 1;
            p.t4w_tab = plan->d_tile_tables + plan->tile2_off;
            p.tmap = reinterpret_cast<const TileEnt*>(p.t4w_tab + kPairTabWords);
            p.t4w_kq = p.t4w_tab + kPairTabWords + (size_t)plan->t_per_chunk * 4;
        } else if (plan->gd >= 0 && !(g_tune_bits & kTuneTile1) &&
                   L.shape[plan->tq] % (16 / L.itemsize) == 0) {
            // k_decode_tileg: tiles grouped by four along gd, whole out pieces
            p.tileg = 1;
            p.gtz = plan->d_tile_tables + plan->g_off_tz;
            p.gmap = reinterpret_cast<const GroupEnt*>(plan->d_tile_tables + plan->g_off_map);
            p.n_groups = plan->n_groups;
            p.n_sub = plan->n_sub;
            p.g_step_t = plan->sstride[plan->gd];
            p.g_step_o = L.out_stride[plan->gd];
            if (plan->tilegw && g_tune_arm != 2 && g_tune_arm != 5) {  // a wave per tile, one chain per lane
                p.t4w_tab = plan->d_tile_tables + plan->tilegw_off;
                p.t4w_kq = p.t4w_tab + kPairTabWords;
                if (plan->tileg2w_off) p.t2w_kq = plan->d_tile_tables + plan->tileg2w_off;  // two tiles per workgroup
                if (plan->tilegl_off) p.tglt_kq = plan->d_tile_tables + plan->tilegl_off;    // (arm 40)
                if (plan->tilebt_off) p.tbt_tab = plan->d_tile_tables + plan->tilebt_off;    // (arm 66)
            }
        }
        const uint64_t tunits = (uint64_t)n_chunks * plan->t_per_chunk;
        if (tunits >= (1ull << 32)) return set_err(ZHIP_E_UNSUPPORTED, "too many tiles in one batch");
        p.n_units = (uint32_t)tunits;
        p.fast = 0;
    }
    if (p.rows && units >= (1ull << 31)) return set_err(ZHIP_E_UNSUPPORTED, "too many units for a row decode");
    fill_pair_hot(p);
    int rc = launch_decode(p, static_cast<hipStream_t>(stream), plan->max_grid);
    if (rc == ZHIP_E_UNSUPPORTED) return set_err(rc, "no kernel for this layout");
    if (rc != ZHIP_OK) return set_err(rc, std::string("launch failed: ") + hipGetErrorString(hipGetLastError()));
    return ZHIP_OK;
}

int zhip_encode(const zhip_plan* plan, const void* arr, void* dst, const zhip_chunk* d_chunks, uint32_t n_chunks,
                const zhip_sel* d_sels, zhip_status* d_status, uint32_t* d_workspace, uint32_t* d_nonempty,
                uint32_t encode_flags, void* stream) {
    return zhip_encode_mapped(plan, arr, dst, d_chunks, n_chunks, d_sels, d_status, d_workspace, d_nonempty,
                              encode_flags, nullptr, stream);
}

int zhip_encode_mapped(const zhip_plan* plan, const void* arr, void* dst, const zhip_chunk* d_chunks,
                       uint32_t n_chunks, const zhip_sel* d_sels, zhip_status* d_status, uint32_t* d_workspace,
                       uint32_t* d_nonempty, uint32_t encode_flags, const zhip_rowblk* d_rowmap, void* stream) {
    if (!plan) return set_err(ZHIP_E_INVALID, "null plan");
    if (!plan->d_tables) return set_err(ZHIP_E_INVALID, "plan not uploaded (zhip_plan_upload)");
    if (n_chunks == 0) return ZHIP_OK;
    if (!arr || !dst || !d_chunks || !d_sels || !d_status || !d_workspace || !d_nonempty)
        return set_err(ZHIP_E_INVALID, "null device pointer");
    if (plan->kblocks != (uint32_t)kDefaultBlocks) return set_err(ZHIP_E_UNSUPPORTED, "encode needs K=8 plans");
    const zhip_layout& L = plan->layout;
    const uint64_t units = (uint64_t)n_chunks * plan->nseg;
    if (units >= (1ull << 32)) return set_err(ZHIP_E_UNSUPPORTED, "too many units in one batch");
    EncodeParams p{};
    // chunks' publication words a 128-byte line apart (zhip_plan_info's >= kPubLine
    // workspace words for CRC layouts); arm ZHIP_TUNE_ARM = 9: 16 bytes apart
    p.pub_stride = ((plan->layout.flags & ZHIP_LF_CRC) && g_tune_arm != 9) ? kPubLine / 2u : 2u;
    p.arr = static_cast<const uint8_t*>(arr);
    p.dst = static_cast<uint8_t*>(dst);
    p.chunks = d_chunks;
    p.sels = d_sels;
    p.status = d_status;
    p.ws = d_workspace;
    p.nonempty = d_nonempty;
    p.horner = plan->d_tables;
    p.kthread = plan->d_tables + 4096;
    p.kunit = plan->d_tables + 4096 + kThreads;
    p.n_chunks = n_chunks;
    p.nseg = plan->nseg;
    p.n_units = (uint32_t)units;
    p.c_inv = plan->c_inv;
    p.c3 = plan->c3;
    p.lflags = L.flags;
    fill_geom(p.g, *plan);
    p.seg = plan->seg;
    p.E = plan->E;
    std::memcpy(p.fill, plan->fill, sizeof(p.fill));
    p.fill_nan = 0;
    if (L.flags & ZHIP_LF_FLOAT) {
        if (L.itemsize == 4) p.fill_nan = (p.fill[0] & 0x7FFFFFFFu) > 0x7F800000u;
        else if (L.itemsize == 2) p.fill_nan = (p.fill[0] & 0x7FFFu) > 0x7C00u;
        else if (L.itemsize == 8)
            p.fill_nan = ((((uint64_t)p.fill[1] << 32) | p.fill[0]) & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull;
    }
    p.fast = (encode_flags & ZHIP_DF_FAST_ROWS) ? 1u : 0u;
    p.tune = g_tune_bits;
    p.rowmap = nullptr;
    p.tile4 = 0;
    if ((encode_flags & ZHIP_DF_TILE) && plan->tile4 && plan->t_per_chunk <= 64 && plan->d_tile_tables &&
        !(g_tune_bits & (kTuneTile1 | kTuneNoTile4))) {
        // transposed chunks, full tiles, at most 16 workgroups per chunk (the
        // arrival / non-empty bits of one 64-bit word): k_encode_tile4
        p.tile4 = 1;
        p.tq = plan->tq;
        p.t_per_chunk = plan->t_per_chunk;
        for (int d = 0; d < ZHIP_MAX_DIMS; ++d) p.sstride[d] = plan->sstride[d];
        p.horner = plan->d_tile_tables;
        p.tz = plan->d_tile_tables + plan->tile4_off_tz;
        p.kq4 = plan->d_tile_tables + plan->tile4_off_kq;
        if (plan->tile2e_off) p.kq2 = plan->d_tile_tables + plan->tile2e_off;
        p.tmap = reinterpret_cast<const TileEnt*>(plan->d_tile_tables + plan->tile4_off_map);
        d_rowmap = nullptr;
    } else if ((encode_flags & ZHIP_DF_TILE) && plan->gd >= 0 && plan->d_tile_tables && !(g_tune_bits & kTuneTile1) &&
               L.shape[plan->tq] % (16 / L.itemsize) == 0 && plan->n_groups < 65536u) {
        // (whole 16-byte pieces along tq: a piece never reaches past the chunk)
        // full selections, tiles grouped by four at a uniform step: k_encode_tileg
        p.tile = 2;
        p.tq = plan->tq;
        p.t_per_chunk = plan->t_per_chunk;
        for (int d = 0; d < ZHIP_MAX_DIMS; ++d) p.sstride[d] = plan->sstride[d];
        p.horner = plan->d_tile_tables;
        p.kthread = plan->d_tile_tables + 4096;
        p.gtz = plan->d_tile_tables + plan->g_off_tz;
        p.gmap = reinterpret_cast<const GroupEnt*>(plan->d_tile_tables + plan->g_off_map);
        p.n_groups = plan->n_groups;
        p.n_sub = plan->n_sub;
        p.g_step_t = plan->sstride[plan->gd];
        p.g_z2 = xpow8(2ull * plan->sstride[plan->gd]);
        p.g_step_o = L.out_stride[plan->gd];
        if (plan->tilebt_off) p.g_a4 = plan->d_tile_tables + plan->tilebt_off + 1024;  // (arm 68)
        p.g_c96 = xpow8_inv(12);
        d_rowmap = nullptr;
    } else if ((encode_flags & (ZHIP_DF_TILE | ZHIP_DF_TILE_PREFIX)) && plan->tq >= 0 && plan->d_tile_tables &&
               (plan->t_per_chunk + 3u) / 4u < 65536u) {
        // every other transposed batch (partial tiles, many tiles per chunk,
        // edge chunks with prefix selections): k_encode_tile
        p.tile = 1;
        p.tq = plan->tq;
        p.t_per_chunk = plan->t_per_chunk;
        p.n_qb = plan->n_qb;
        p.n_cb = plan->n_cb;
        p.d_qb = make_fdiv(plan->n_qb);
        p.d_cb = make_fdiv(plan->n_cb);
        for (int d = 0; d < ZHIP_MAX_DIMS; ++d) p.sstride[d] = plan->sstride[d];
        p.horner = plan->d_tile_tables;
        p.kthread = plan->d_tile_tables + 4096;
        p.kunit = plan->d_tile_tables + 4096 + kThreads;
        p.c_inv = plan->t_c_inv;
        d_rowmap = nullptr;
    }
    if (d_rowmap) {
        const uint32_t rb = plan->row_bytes;
        const int nd = L.ndim;
        if (!p.fast || nd < 2 || rb < 16 || rb > (uint32_t)kWgStride || (rb & (rb - 1)) != 0 ||
            (uint32_t)L.shape[nd - 2] % ((uint32_t)kWgStride / rb) != 0)
            return set_err(ZHIP_E_INVALID, "row map given for a layout without whole-row encode");
        p.rowmap = d_rowmap;
        p.kpair = plan->d_tables + 4096 + kThreads + plan->nseg;
        p.pair_tab = plan->d_tables + plan->off_pair;
        p.kpair11 = p.pair_tab + kPairTabWords;
        p.row_shift = (uint32_t)__builtin_ctz(rb);
        p.r_oy = L.out_stride[nd - 2];
        if (plan->il_S == 8u && (L.flags & ZHIP_LF_CRC)) {  // k_encode_il (launch_encode)
            // the decode's widest interleave (S = 32 / 16 where the steps tile
            // it; tuning arm 73 keeps S = 8)
            int si = plan->off_il_s[1] ? 1 : plan->off_il_s[0] ? 0 : -1;
            if (ZHIP_TUNING && g_tune_arm == 73) si = -1;
            p.il_S = si >= 0 ? 16u << si : plan->il_S;
            p.il_tab = plan->d_tables + (si >= 0 ? plan->off_il_s[si] : plan->off_il);
            p.il_klane = p.il_tab + kPairTabWords;
            // whole-chunk selections: destinations computed (ZHIP_DF_WHOLE, as the
            // decode) only in tuning arm 46 -- graph-timed 29.1 vs 28.6 us on the
            // C2 encode (profiles/r05/x/): the encode keeps the row map
            p.aff_ok = (encode_flags & ZHIP_DF_WHOLE) && plan->aff_ok && ZHIP_TUNING && g_tune_arm == 46;
            if (p.aff_ok) set_affine(p, plan);
        }
    }
    int rc = launch_encode(p, static_cast<hipStream_t>(stream), plan->max_grid);
    if (rc == ZHIP_E_UNSUPPORTED) return set_err(rc, "no encode kernel for this layout");
    if (rc != ZHIP_OK) return set_err(rc, std::string("launch failed: ") + hipGetErrorString(hipGetLastError()));
    return ZHIP_OK;
}

int zhip_shard_pack(const zhip_plan* plan, void* dst, const zhip_shard* d_shards, uint32_t n_shards,
                    uint32_t n_inner, uint32_t elen, uint32_t index_size, uint32_t pack_flags,
                    const uint32_t* d_nonempty, uint32_t* d_newrank, const uint32_t* d_rank_of_slot,
                    uint64_t* d_blob_len, void* stream) {
    std::call_once(g_once, init_tables);
    if (!plan || !plan->d_tables) return set_err(ZHIP_E_INVALID, "plan not uploaded");
    if (n_shards == 0) return ZHIP_OK;
    if (!dst || !d_shards || !d_nonempty || !d_newrank || !d_rank_of_slot || !d_blob_len)
        return set_err(ZHIP_E_INVALID, "null device pointer");
    if (n_inner == 0) return set_err(ZHIP_E_INVALID, "n_inner == 0");
    PackParams p{};
    p.dst = static_cast<uint8_t*>(dst);
    p.shards = d_shards;
    p.nonempty = d_nonempty;
    p.newrank = d_newrank;
    p.rank_of_slot = d_rank_of_slot;
    p.blob_len = d_blob_len;
    p.horner = plan->d_tables;
    p.kthread = plan->d_tables + 4096;
    p.n_inner = n_inner;
    p.elen = elen;
    p.index_size = index_size;
    p.index_start = (pack_flags & ZHIP_PF_INDEX_START) ? 1u : 0u;
    p.index_crc = (pack_flags & ZHIP_PF_INDEX_CRC) ? 1u : 0u;
    p.keep_empty = (pack_flags & ZHIP_PF_KEEP_EMPTY) ? 1u : 0u;
    // index CRC constants: thread t's Horner state lands at 16t + 4096*kiters,
    // shifted by kthread[t] to R = 4096*(kiters+1); payload = 16*n_inner bytes
    const uint64_t nidx = 16ull * n_inner;
    const uint64_t kiters = (n_inner + kThreads - 1) / kThreads;
    const uint64_t R = (uint64_t)kWgStride * (kiters + 1);
    p.idx_c_inv = xpow8_inv(R - nidx);
    p.idx_c3 = gf_mul(xpow8(nidx), 0xFFFFFFFFu);
    int rc = launch_shard_pack(p, n_shards, static_cast<hipStream_t>(stream));
    if (rc != ZHIP_OK) return set_err(rc, std::string("launch failed: ") + hipGetErrorString(hipGetLastError()));
    return ZHIP_OK;
}

uint32_t zhip_fdiv_eval(uint32_t n, uint32_t d) {
    const zhip_fdiv f = make_fdiv(d);
    return fdiv_apply(n, f.m, f.s);
}

// CPU emulation of the device CRC combine for one chunk of a plan (the exact
// decomposition, tables and constants the kernel uses).  Test hook: lets the
// CPU suite prove the algebra without a GPU.
uint32_t zhip_crc32c_host(const void* data, uint64_t nbytes) {
    std::call_once(g_once, init_tables);
    const uint8_t* p = static_cast<const uint8_t*>(data);
    if (!nbytes) return 0u;
    static const bool hw = __builtin_cpu_supports("sse4.2");
    return hw ? crc_sse42(p, nbytes) : crc_bytewise(p, nbytes);
}

uint32_t zhip_emulate_chunk_crc(const zhip_plan* plan, const uint8_t* data) {
    std::call_once(g_once, init_tables);
    std::vector<uint32_t> tab(4096);
    build_horner(tab.data());
    const uint32_t N = (uint32_t)plan->layout.nbytes;
    uint32_t V = 0;
    for (uint32_t s = 0; s < plan->nseg; ++s) {
        const int32_t hi = (int32_t)plan->E - (int32_t)(s * plan->seg);
        const int32_t lo = hi - (int32_t)plan->seg;
        uint32_t unit = 0;
        for (int t = 0; t < kThreads; ++t) {
            uint32_t acc = 0;
            for (int k = 0; k < (int)plan->kblocks; ++k) {
                const int32_t o = lo + kWgStride * k + 16 * t;
                uint8_t b[16] = {0};
                for (int i = 0; i < 16; ++i) {
                    const int64_t q = (int64_t)o + i;
                    if (q >= 0 && q < (int64_t)N) b[i] = data[q];
                }
                uint32_t w[4];
                std::memcpy(w, b, 16);
                auto ap = [&](int op, uint32_t x) {
                    const uint32_t* tb = tab.data() + op * 1024;
                    return tb[x & 255u] ^ tb[256 + ((x >> 8) & 255u)] ^ tb[512 + ((x >> 16) & 255u)] ^
                           tb[768 + (x >> 24)];
                };
                acc = ap(0, acc ^ w[0]) ^ ap(1, w[1]) ^ ap(2, w[2]) ^ ap(3, w[3]);
            }
            unit ^= gf_mul(acc, xpow8((uint64_t)kWgStride - 16u * t));
        }
        V ^= gf_mul(unit, xpow8((uint64_t)s * plan->seg));
    }
    return ~(gf_mul(V, plan->c_inv) ^ plan->c3);
}

// CPU emulation of k_decode_pair's CRC for one chunk: 11/11/10-bit A4096
// tables, four word accumulators per lane folded with the A4 tables, the
// windowed per-lane multiply by kpair11 (3-bit windows + a 2-bit top window,
// as the kernel's LDS tables), unit contributions xor-combined.  Test hook.
uint32_t zhip_emulate_chunk_crc_pair(const zhip_plan* plan, const uint8_t* data) {
    std::call_once(g_once, init_tables);
    std::vector<uint32_t> tab(kPairTabWords);
    build_pair_tables(tab.data());
    const uint32_t* T = tab.data();
    auto a11 = [&](uint32_t w) { return T[kPairT1 + (w & 2047u)] ^ T[kPairT2 + ((w >> 11) & 2047u)] ^ T[kPairT3 + (w >> 22)]; };
    auto a4 = [&](uint32_t w) {
        const uint32_t* t4 = T + kPairA4;
        return t4[w & 255u] ^ t4[256 + ((w >> 8) & 255u)] ^ t4[512 + ((w >> 16) & 255u)] ^ t4[768 + (w >> 24)];
    };
    auto mulx = [](uint32_t b) { return (b >> 1) ^ (kPoly & (0u - (b & 1u))); };
    auto lanemul3 = [&](uint32_t a, uint32_t k) {  // the kernel's windowed multiply
        uint32_t m3[8], m2[4];
        const uint32_t k1 = mulx(k), k2 = mulx(k1);
        for (uint32_t v = 0; v < 8; ++v) m3[v] = ((v & 4u) ? k : 0u) ^ ((v & 2u) ? k1 : 0u) ^ ((v & 1u) ? k2 : 0u);
        for (uint32_t v = 0; v < 4; ++v) m2[v] = ((v & 2u) ? k : 0u) ^ ((v & 1u) ? k1 : 0u);
        uint32_t p = m3[a & 7u];
        for (int j = 1; j < 10; ++j) p = mulx(mulx(mulx(p))) ^ m3[(a >> (3 * j)) & 7u];
        return mulx(mulx(p)) ^ m2[a >> 30];
    };
    const uint32_t N = (uint32_t)plan->layout.nbytes;
    const uint32_t c96 = xpow8_inv(12);
    uint32_t V = 0;
    for (uint32_t s = 0; s < plan->nseg; ++s) {
        const int32_t hi = (int32_t)plan->E - (int32_t)(s * plan->seg);
        const int32_t lo = hi - (int32_t)plan->seg;
        const uint32_t ku = gf_mul(xpow8((uint64_t)s * plan->seg), plan->c_inv);
        for (int t = 0; t < kThreads; ++t) {
            uint32_t a[4] = {0, 0, 0, 0};
            for (int k = 0; k < (int)plan->kblocks; ++k) {
                const int32_t o = lo + kWgStride * k + 16 * t;
                uint8_t b[16] = {0};
                for (int i = 0; i < 16; ++i) {
                    const int64_t q = (int64_t)o + i;
                    if (q >= 0 && q < (int64_t)N) b[i] = data[q];
                }
                uint32_t w[4];
                std::memcpy(w, b, 16);
                for (int j = 0; j < 4; ++j) a[j] = a11(a[j] ^ w[j]);
            }
            const uint32_t S = a4(a4(a4(a[0]) ^ a[1]) ^ a[2]) ^ a[3];
            const uint32_t k11 = gf_mul(gf_mul(xpow8((uint64_t)kWgStride - 16u * t), ku), c96);
            V ^= lanemul3(S, k11);
        }
    }
    return ~(V ^ plan->c3);
}

// CPU emulation of k_decode_il's CRC for one chunk: workgroup r takes steps
// (r / S) S 8 + r % S + S k (k < 8); each lane's four word accumulators run
// through the A_(4096 S) tables, fold with the A4 tables and are multiplied by
// the workgroup's lane constant (windowed, as the kernel); -1 when the plan
// has no interleaved layout.  Test hook.
uint32_t zhip_emulate_chunk_crc_il(const zhip_plan* plan, const uint8_t* data) {
    std::call_once(g_once, init_tables);
    if (!plan || !plan->il_S) return 0xFFFFFFFFu;
    // the interleave the decode launches take (zhip_decode_mapped): the widest
    // that tiles the chunk's steps (the rule zhip_plan_upload builds tables by)
    uint32_t S = plan->il_S;
    const uint64_t n_st = (uint64_t)plan->nseg * kDefaultBlocks;
    if (S == 8u) S = n_st % (32ull * kDefaultBlocks) == 0 ? 32u : n_st % (16ull * kDefaultBlocks) == 0 ? 16u : 8u;
    const uint32_t K = kDefaultBlocks;
    std::vector<uint32_t> tab(kPairTabWords);
    build_pair_tables(tab.data(), (uint64_t)kWgStride * S);
    const uint32_t* T = tab.data();
    auto a11 = [&](uint32_t w) { return T[kPairT1 + (w & 2047u)] ^ T[kPairT2 + ((w >> 11) & 2047u)] ^ T[kPairT3 + (w >> 22)]; };
    auto a4 = [&](uint32_t w) {
        const uint32_t* t4 = T + kPairA4;
        return t4[w & 255u] ^ t4[256 + ((w >> 8) & 255u)] ^ t4[512 + ((w >> 16) & 255u)] ^ t4[768 + (w >> 24)];
    };
    const uint32_t N = (uint32_t)plan->layout.nbytes;
    const uint32_t c96 = xpow8_inv(12);
    const int64_t n_steps = (int64_t)plan->nseg * K;
    const int64_t lo_frame = (int64_t)plan->E - n_steps * kWgStride;
    uint32_t V = 0;
    for (uint32_t r = 0; r < plan->nseg; ++r) {
        const int64_t st0 = (int64_t)(r / S) * S * K + (int64_t)(r % S);
        for (int t = 0; t < kThreads; ++t) {
            uint32_t a[4] = {0, 0, 0, 0};
            for (uint32_t k = 0; k < K; ++k) {
                const int64_t o = lo_frame + (int64_t)kWgStride * (st0 + (int64_t)S * k) + 16 * t;
                uint8_t b[16] = {0};
                for (int i = 0; i < 16; ++i) {
                    const int64_t q = o + i;
                    if (q >= 0 && q < (int64_t)N) b[i] = data[q];
                }
                uint32_t w[4];
                std::memcpy(w, b, 16);
                for (int j = 0; j < 4; ++j) a[j] = a11(a[j] ^ w[j]);
            }
            const uint32_t Sx = a4(a4(a4(a[0]) ^ a[1]) ^ a[2]) ^ a[3];
            const int64_t e = (int64_t)kWgStride * (n_steps - st0 + 1 - (int64_t)S * K) - 16 * t;
            const uint32_t xe = e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)(-e));
            V ^= gf_mul(Sx, gf_mul(gf_mul(xe, plan->c_inv), c96));
        }
    }
    return ~(V ^ plan->c3);
}

// CPU emulation of k_decode_xw's CRC for one chunk: lane l of span r takes
// blocks at 8192 r + 1024 k + 16 l (k < 8) through the A_1024 tables, folds
// with the A4 tables and multiplies by the (r, l) lane constant; -1 when the
// plan has no xw layout.  Test hook.
uint32_t zhip_emulate_chunk_crc_xw(const zhip_plan* plan, const uint8_t* data) {
    std::call_once(g_once, init_tables);
    if (!plan || !plan->xw_P) return 0xFFFFFFFFu;
    std::vector<uint32_t> tab(kPairTabWords);
    build_pair_tables(tab.data(), 1024);
    const uint32_t* T = tab.data();
    auto a11 = [&](uint32_t w) { return T[kPairT1 + (w & 2047u)] ^ T[kPairT2 + ((w >> 11) & 2047u)] ^ T[kPairT3 + (w >> 22)]; };
    auto a4 = [&](uint32_t w) {
        const uint32_t* t4 = T + kPairA4;
        return t4[w & 255u] ^ t4[256 + ((w >> 8) & 255u)] ^ t4[512 + ((w >> 16) & 255u)] ^ t4[768 + (w >> 24)];
    };
    const uint32_t N = (uint32_t)plan->layout.nbytes;
    const uint32_t c96 = xpow8_inv(12);
    const int64_t n_steps = (int64_t)plan->nseg * kDefaultBlocks;
    const int64_t lo_frame = (int64_t)plan->E - n_steps * kWgStride;
    uint32_t V = 0;
    for (uint32_t r = 0; r < plan->xw_P; ++r)
        for (int l = 0; l < 64; ++l) {
            uint32_t a[4] = {0, 0, 0, 0};
            for (int k = 0; k < kDefaultBlocks; ++k) {
                const int64_t o = lo_frame + 8192 * (int64_t)r + 1024 * k + 16 * l;
                uint8_t b[16] = {0};
                for (int i = 0; i < 16; ++i) {
                    const int64_t q = o + i;
                    if (q >= 0 && q < (int64_t)N) b[i] = data[q];
                }
                uint32_t w[4];
                std::memcpy(w, b, 16);
                for (int j = 0; j < 4; ++j) a[j] = a11(a[j] ^ w[j]);
            }
            const uint32_t Sx = a4(a4(a4(a[0]) ^ a[1]) ^ a[2]) ^ a[3];
            const int64_t e = (int64_t)kWgStride * (n_steps - 2 * (int64_t)r - 1) - 16 * l;
            const uint32_t xe = e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)(-e));
            V ^= gf_mul(Sx, gf_mul(gf_mul(xe, plan->c_inv), c96));
        }
    return ~(V ^ plan->c3);
}

// CPU self-test of the identities the kernels rely on.  Returns 0 when all hold.
int zhip_selftest(void) {
    std::call_once(g_once, init_tables);
    // 1. top byte of T[i] is a bijection (needed for the inverse byte step)
    bool seen[256] = {false};
    for (int i = 0; i < 256; ++i) seen[g_T[i] >> 24] = true;
    for (int i = 0; i < 256; ++i)
        if (!seen[i]) return set_err(1, "T top-byte map is not a bijection");
    // 2. A_1(v) == gf_mul(v, x^8) and inverse round trip
    uint32_t v = 0x12345678u;
    for (int it = 0; it < 1000; ++it) {
        v = v * 1664525u + 1013904223u;
        const uint32_t a = (v >> 8) ^ g_T[v & 255u];
        if (a != gf_mul(v, xpow8(1))) return set_err(2, "A_1 != multiply by x^8");
        if (gf_mul(gf_mul(v, xpow8(777)), xpow8_inv(777)) != v) return set_err(3, "x^-8n inverse wrong");
    }
    // 3. crc of "123456789"
    if (crc_bytewise((const uint8_t*)"123456789", 9) != 0xE3069283u) return set_err(4, "check value");
    // 4. fast division
    const uint32_t ds[] = {1, 2, 3, 5, 7, 10, 15, 60, 64, 100, 255, 256, 1000, 4096, 65537, 1000003u};
    for (uint32_t d : ds) {
        const zhip_fdiv f = make_fdiv(d);
        uint32_t x = 1;
        for (int it = 0; it < 20000; ++it) {
            x = x * 1103515245u + 12345u;
            const uint32_t n = (it < 1000) ? (uint32_t)it : (x & 0x7FFFFFFFu);
            if (fdiv_apply(n, f.m, f.s) != n / d) return set_err(5, "fdiv wrong");
        }
        const uint32_t nmax = 0x7FFFFFFFu;
        if (fdiv_apply(nmax, f.m, f.s) != nmax / d) return set_err(5, "fdiv wrong at 2^31-1");
    }
    // 5. kernel decomposition == bytewise CRC for several sizes
    const uint64_t sizes[] = {0, 1, 3, 4, 15, 16, 17, 100, 4095, 4096, 4097, 32768, 32769, 100000, 262148};
    std::vector<uint8_t> buf(262148);
    uint32_t r = 7;
    for (auto& b : buf) {
        r = r * 1664525u + 1013904223u;
        b = (uint8_t)(r >> 24);
    }
    for (uint64_t n : sizes) {
        zhip_layout L{};
        L.ndim = 1;
        L.itemsize = 1;
        L.shape[0] = (int32_t)n;
        L.nbytes = n;
        zhip_plan* p = nullptr;
        if (zhip_plan_create(&L, &p) != ZHIP_OK) return 6;
        const uint32_t got = zhip_emulate_chunk_crc(p, buf.data());
        const uint32_t got_pair = zhip_emulate_chunk_crc_pair(p, buf.data());
        zhip_plan_destroy(p);
        if (got != crc_bytewise(buf.data(), n)) return set_err(7, "emulated kernel CRC wrong at n=" + std::to_string(n));
        if (got_pair != crc_bytewise(buf.data(), n))
            return set_err(8, "emulated pair-kernel CRC wrong at n=" + std::to_string(n));
    }
    return 0;
}

}  // extern "C"
