// Internal (non-ABI) structures shared by the plan builder and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/zarrhip.h"

namespace zhip {

constexpr int kThreads = 256;                            // one workgroup = 4 waves
constexpr int kWgStride = kThreads * 16;                 // 4 KiB per workgroup step
constexpr int kDefaultBlocks = 8;                        // 16-byte blocks per thread per unit
// workspace words per chunk of CRC layouts (zhip_plan_info): k_decode_il /
// k_decode_tile4 publish into word kPubLine * c, one 128-byte line per chunk
// (32 workgroups' returning atomics per line instead of 8 chunks' 256)
constexpr uint32_t kPubLine = 32;

// Stored-chunk geometry + out mapping (shared by decode and encode).
struct Geom {
    int32_t ndim, itemsize;
    int32_t shape[ZHIP_MAX_DIMS];
    int64_t ostride[ZHIP_MAX_DIMS];
    zhip_fdiv dshape[ZHIP_MAX_DIMS];
    uint32_t nbytes;  // N (< 2^31)
    uint32_t row_bytes;
    zhip_fdiv drow;
};

// Kernel argument block (passed by value; indexed only with compile-time
// subscripts inside the kernels so it stays in SGPRs / kernarg memory).
// One tile of a chunk (k_decode_tile4): source offset of its first row in the
// stored chunk, out offset relative to the chunk's out_off.
struct TileEnt {
    uint32_t tbase, _pad;
    int64_t orel;
};

// One group of k_encode_tileg: its first tile's stored offset and array
// offset (relative to the chunk), the tiles' row / byte extent (partial tiles
// at the chunk's edges), and kunit[its last tile] * t_c_inv.
struct GroupEnt {
    uint32_t tbase;
    uint16_t rows, cols;
    int64_t orel;
    uint32_t ku, _pad;
};

// k_decode_pair CRC table layout (u32 words): A4096 by the 11 low, 11 middle
// and 10 high bits of a word, then the four byte slices of A4 (x^32).
constexpr int kPairT1 = 0, kPairT2 = 2048, kPairT3 = 4096, kPairA4 = 5120;
constexpr int kPairTabWords = 6144;
// the byte-table form of the same operator (tuning arms 66 / 67: k_decode_tile4w
// / k_decode_tilegw): A_D's four 256-entry byte tables, then the A4 fold tables
constexpr int kByteTabWords = 2048;
extern const char* g_last_kernel;  // zhip_last_kernel: the kernel the last decode / mapped encode launched
constexpr uint32_t kIlwMaxUnits = 512;  // k_decode_ilw (512 lanes) for grids of at most 2 units per CU
constexpr int kIlBasisWords = 64;  // T1 / T2 / T3 bases (11 + 11 + 10, padded to 32), A4 bases (4 x 8)

// What k_decode_lead (and the k_decode_il arm) need before their first vector loads,
// FIRST in the kernel arguments and read as one scalar batch (pair_hot): the
// lazily scheduled kernarg loads of the full struct put five to seven
// dependent round trips (and software divisions) between the kernel start and
// the first data load.  Divisors are host-built magic numbers (zhip_fdiv).
struct PairHot {
    uint32_t n_units, nseg, n_idx, xcd_run;
    zhip_fdiv d_nseg, d_xcd, d_per;
    uint32_t pred, pred_per, E, seg;
    uint32_t tune, pad;
    uint64_t pred_base, pred_outer, pred_inner;
    uint64_t src, pair_tab, kpair11, kthread11;
    // k_decode_il
    uint32_t il_S, n_chunks;
    uint64_t il_tab, il_klane, il_kidx;
};

struct DecodeParams {
    PairHot h;
    const uint8_t* src;
    uint64_t src_size;
    uint8_t* out;
    const zhip_chunk* chunks;
    const zhip_sel* sels;
    zhip_status* status;
    uint32_t* ws;
    uint32_t* errflag;
    const uint32_t* horner;   // [4 operators][4 byte slices][256]
    uint32_t hx[4];           // x^(8(4096 - 4k)): the operators, for in-kernel table builds
    uint32_t kq[32];          // lane-shift factors (lane_kthread)
    const uint32_t* kthread;  // [kThreads]
    const uint32_t* kunit;    // [nseg]
    const uint32_t* kpair;    // [nseg][kThreads]: kthread * kunit * c_inv (k_decode_pair)
    // k_decode_pair's CRC tables (kPairTab* layout): A4096 in 11/11/10-bit
    // slices (one operator for all four words: four accumulators per lane) and
    // the A4 byte tables that combine them, then kpair and kthread times
    // x^(-96) (the frame of the combined state), [nseg][kThreads] and [kThreads]
    const uint32_t* pair_tab;
    const uint32_t* kpair11;
    const uint32_t* kthread11;
    uint32_t n_chunks, nseg, n_units;
    uint32_t c_inv, c3;
    uint32_t lflags;
    Geom g;
    uint32_t seg;     // bytes per unit = kWgStride * K
    uint32_t E;       // align16(N)
    uint32_t index_size, n_inner;
    uint32_t fill[4];
    uint32_t fast;
    uint32_t tune;  // kTune* ablation bits (0 in production)
    // tile mode (transposed chunks: stored dim tq is contiguous in out)
    int32_t tq;
    uint32_t t_per_chunk, n_qb, n_cb;
    uint32_t sstride[ZHIP_MAX_DIMS];  // stored-stream byte stride of each dim
    zhip_fdiv d_qb, d_cb;
    // k_decode_tile4 (tile4 != 0): see zhip_plan
    uint32_t tile4;
    uint32_t tile2;  // k_decode_tile4w's two-tile form over consecutive tile pairs (plans without tile4)
    const uint32_t* tz;
    const uint32_t* kq4;
    const struct TileEnt* tmap;
    // k_decode_tile4f (non-null: the layout qualifies): A_64 pair tables, lane constants
    const uint32_t* t4f_tab;
    const uint32_t* t4f_kq;
    // k_decode_tile4w / k_decode_tilegw (non-null: taken): A_(4 sq) pair
    // tables, lane constants [T/4 or n_groups][kThreads]
    const uint32_t* t4w_tab;
    const uint32_t* t4w_kq;
    const uint32_t* t2w_kq;  // k_decode_tile4w with two tiles per workgroup (production when set): lane constants
    const uint32_t* t1w_kq;  // tuning arm 37 (one tile per workgroup)
    const uint32_t* tglt_kq; // tuning arm 40 (k_decode_tilegw, lanes pick the tile): lane constants
    const uint32_t* tbt_tab; // tuning arms 66 / 67: A_(4 sq) as byte tables + A4 (kByteTabWords)
    // k_decode_tileg (tileg != 0): group map, step multiply table, steps
    uint32_t tileg;
    const struct GroupEnt* gmap;
    const uint32_t* gtz;
    uint32_t n_groups, g_step_t, n_sub;
    int64_t g_step_o;
    // fused shard-index CRC verification: workgroup g checks indexes g, g+G, ...
    const zhip_chunk* idx_chunks;
    zhip_status* idx_status;
    uint32_t n_idx, idx_nbytes, idx_E, idx_c_inv, idx_c3;
    // whole-row affine mapping (ZHIP_DF_ROWS, k_decode_rows): rows of 2^row_shift
    // bytes, 4096 / row_bytes rows per workgroup step, never crossing dim ndim-2
    uint32_t row_shift, r_sy;  // log2(row_bytes), shape[ndim-2]
    zhip_fdiv r_dy;            // division by shape[ndim-2]
    int64_t r_oy;              // out stride of dim ndim-2
    int32_t nd2;               // ndim - 2
    uint32_t rows;             // 1: launch k_decode_rows
    uint32_t xcd_run;          // k_decode_pair: pairs per XCD-contiguous run (0: dispatch order)
    const zhip_rowblk* rowmap; // per (sel, unit, step) destinations (zhip_rows_map); k_decode_pair
    // k_decode_il: interleave stride (steps), its A_(4096 S) tables, lane
    // constants per workgroup-in-chunk and for the fused index check
    uint32_t il_S;
    const uint32_t* il_tab;
    const uint32_t* il_klane;
    const uint32_t* il_kidx;
    const uint32_t* il_basis;  // kIlBasisWords: the il tables' single-bit entries (k_decode_ilc)
    uint32_t dv_bank;  // deferred CRC verdicts: bank this launch publishes into (ZHIP_DF_BANK1)
    uint32_t defer;    // ZHIP_DF_DEFER: the caller reads deferred verdicts (tileg / tilegw publish so)
    // k_decode_xw: 8 KiB spans per chunk (0: not available), arrival subwords
    // per chunk in the workspace tail (0: one level or xor + count), its A_1024
    // tables, lane constants per (span, lane) and for the fused index check
    uint32_t xw, xw_nsub;
    const uint32_t* xw_tab;
    const uint32_t* xw_klane;
    const uint32_t* xw_kidx;
    // k_decode_ilw (small shares): ilw_nt lanes per 32 KiB unit (0: not
    // available), its A_(16 ilw_nt) tables, lane constants per (unit, lane),
    // the fused index check's lane constants
    uint32_t ilw_nt;
    const uint32_t* ilh_klane;  // tuning arm 41 (k_decode_ilh, 16 KiB per workgroup): lane constants [2 nseg][kThreads]
    const uint32_t* ilw_tab;
    const uint32_t* ilw_klane;
    const uint32_t* ilw_kidx;
    // ZHIP_DF_WHOLE launches of a plan with aff_ok: the row map of the whole
    // chunk as rel(st) = (st >> aff_sh) aff_B + (st & aff_mask) aff_C + aff_D
    // (zhip_plan aff_*); k_decode_il / k_decode_ilw take their AFF form
    uint32_t aff_ok, aff_sh, aff_mask;
    int32_t aff_B, aff_C, aff_D;
    // load-address prediction (zhip_predict; k_decode_pair): payload of chunk c
    // predicted at src + pred_base + (c / pred_per) * pred_outer + (c % pred_per) * pred_inner
    uint32_t pred, pred_per;
    uint64_t pred_base, pred_outer, pred_inner;
};

// n / d == (n * m) >> s for 0 <= n < 2^31 (host side; fdiv_apply on the device)
inline zhip_fdiv make_fdiv(uint32_t d) {
    zhip_fdiv f;
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    f.s = 31 + l;
    f.m = (uint32_t)(((1ull << (31 + l)) + d - 1) / d);  // ceil(2^(31+l) / d) < 2^32 for d >= 1
    return f;
}

// PairHot from the full parameters (after every field is final); xcd_run and
// its divisor are set again by launch_decode
inline void fill_pair_hot(DecodeParams& p) {
    PairHot& h = p.h;
    h.n_units = p.n_units;
    h.nseg = p.nseg;
    h.n_idx = p.n_idx;
    h.xcd_run = p.xcd_run;
    h.d_nseg = make_fdiv(p.nseg ? p.nseg : 1u);
    h.d_xcd = make_fdiv(p.xcd_run ? p.xcd_run : 1u);
    h.d_per = make_fdiv(p.pred_per ? p.pred_per : 1u);
    h.pred = p.pred;
    h.pred_per = p.pred_per;
    h.E = p.E;
    h.seg = p.seg;
    h.tune = p.tune;
    h.pad = 0;
    h.pred_base = p.pred_base;
    h.pred_outer = p.pred_outer;
    h.pred_inner = p.pred_inner;
    h.src = reinterpret_cast<uint64_t>(p.src);
    h.pair_tab = reinterpret_cast<uint64_t>(p.pair_tab);
    h.kpair11 = reinterpret_cast<uint64_t>(p.kpair11);
    h.kthread11 = reinterpret_cast<uint64_t>(p.kthread11);
    h.il_S = p.il_S;
    h.n_chunks = p.n_chunks;
    h.il_tab = reinterpret_cast<uint64_t>(p.il_tab);
    h.il_klane = reinterpret_cast<uint64_t>(p.il_klane);
    h.il_kidx = reinterpret_cast<uint64_t>(p.il_kidx);
}

constexpr int kTileRows = 64;    // rows of the contiguous-in-out dim per tile
constexpr int kTileCols = 256;   // bytes of the innermost stored row per tile

// Ablation / tuning knobs (zhip_set_tuning): never set on the product path.
constexpr uint32_t kTuneSkipCrc = 1u;   // replace the CRC lookups by a plain xor
constexpr uint32_t kTuneAcqRel = 2u;    // acq_rel ticket (the round-1 first version)
constexpr uint32_t kTuneNoTicket = 4u;  // xor only, no last-arriver finalize
constexpr uint32_t kTuneNT = 8u;        // nontemporal loads / stores (fast rows path)
constexpr uint32_t kTuneNoLaneMul = 16u; // rows kernel: skip the per-lane shift multiply
constexpr uint32_t kTunePersist = 64u;   // whole-row layouts: persistent k_decode_rows instead of k_decode_pair
constexpr uint32_t kTuneSingle = 128u;   // k_decode_pair with one unit per workgroup
constexpr uint32_t kTuneSerialize = 256u; // k_decode_pair: wait for every load before the first store
constexpr uint32_t kTuneNoTables = 512u;  // k_decode_pair: skip the in-LDS table build (results invalid)
constexpr uint32_t kTuneTrailingCrc = 2048u; // k_decode_pair: CRC lookups after all stores (default: per block; headline type)
constexpr uint32_t kTuneNoRunEnd = 4096u;  // k_decode_pair: skip the run-end reduction entirely (results invalid)
constexpr uint32_t kTuneNoBarrier = 8192u; // k_decode_pair: skip the table barrier (results invalid)
constexpr uint32_t kTuneNoConsts = 32768u; // k_decode_pair: skip the lane-constant and trailer loads (results invalid)
constexpr uint32_t kTuneTile1 = 65536u;  // transposed layouts: the one-tile persistent k_decode_tile
constexpr uint32_t kTuneSplitChain = 262144u; // k_decode_pair: independent Horner chains for the two units
constexpr uint32_t kTuneEncNoFlags = 524288u; // k_encode_pair: skip the non-empty flag atomics (results invalid)
constexpr uint32_t kTuneNoTile4 = 1048576u;   // transposed layouts: grouped k_*_tileg where k_*_tile4 would run
constexpr uint32_t kTuneDuo = 2097152u;       // whole-row layouts: k_decode_duo (one unit per half of a 512-thread workgroup)
constexpr uint32_t kTuneNoXcd = 8388608u;     // k_decode_pair: plain dispatch order (no XCD-contiguous runs)
constexpr uint32_t kTunePrio = 16777216u;     // k_decode_pair arm: s_setprio(1) once a wave's loads are out
constexpr uint32_t kTuneDeferB = 33554432u;   // k_decode_pair arm: unit B's loads interleaved with A's stores
constexpr uint32_t kTuneIl = 67108864u;       // whole-row layouts: k_decode_il wherever the layout admits it
constexpr uint32_t kTuneNoIl = 134217728u;    // whole-row layouts: never k_decode_il (k_decode_pair)
constexpr uint32_t kTuneXw = 268435456u;      // whole-row layouts: k_decode_xw where admitted
constexpr uint32_t kTuneNoXw = 536870912u;    // whole-row layouts: never k_decode_xw
constexpr uint32_t kTuneNoPub = 1073741824u;  // timing arm: k_decode_il / k_decode_xw skip the CRC publication
constexpr uint32_t kTuneIlLean = 16384u;    // k_decode_il arm: lean predicted prologue (data loads before the header chain)
constexpr uint32_t kTuneTile4F = 2147483648u;   // transposed layouts arm: k_decode_tile4f where the layout admits it
constexpr uint32_t kTuneIlRegMul = 32u;      // k_decode_il arm: lane multiply in registers (no LDS column)
constexpr uint32_t kTuneIlOcc6 = 4194304u;   // k_decode_il arm: register lane multiply, 6 workgroups per CU
constexpr uint32_t kTuneCfLookup = 131072u;  // k_decode_il timing arm: conflict-free lookup addresses (results invalid)
constexpr uint32_t kTuneStamp = 1024u;    // k_decode_pair: per-workgroup phase timestamps (zhip_debug_stamps)
constexpr uint32_t kStampWG = 8192u;      // workgroups stamped per launch
constexpr uint32_t kStampSlots = 8u;
}  // namespace zhip
extern "C" void zhip_stage_set_streams(uint32_t n);  // staging.cpp (ZHIP_TUNE_STAGE_STREAMS)
extern "C" void zhip_stage_set_copy(uint32_t nt);     // staging.cpp (ZHIP_TUNE_STAGE_COPY)
namespace zhip {
// The kernel knobs (zhip_set_tuning ZHIP_TUNE_MAX_GRID / ABLATION / BLOCKS /
// ARM) and every measurement-arm kernel exist only in the tuning build
// (make tune -> libzarrhip_tune.so, -DZHIP_TUNING=1; scripts/armbench.py).
// The shipped library has them as compile-time zeros: no arm is compiled in
// and no variable of a user's environment can change a launch.
#ifndef ZHIP_TUNING
#define ZHIP_TUNING 0
#endif
#if ZHIP_TUNING
extern int g_tune_max_grid;
extern int g_tune_blocks;
extern uint32_t g_tune_bits;
extern int g_tune_arm;  // ZHIP_TUNE_ARM: experimental kernel variant (0 = production)
#else
constexpr int g_tune_max_grid = 0;
constexpr int g_tune_blocks = 0;
constexpr uint32_t g_tune_bits = 0;
constexpr int g_tune_arm = 0;
#endif

struct EncodeParams {
    const uint8_t* arr;   // source array base (device)
    uint8_t* dst;         // encoded destination buffer
    const zhip_chunk* chunks;  // src = dst offset of the encoded chunk, out_off = arr offset
    const zhip_sel* sels;
    zhip_status* status;
    uint32_t* ws;
    uint32_t* nonempty;
    const uint32_t* horner;
    const uint32_t* kthread;
    const uint32_t* kunit;
    uint32_t n_chunks, nseg, n_units;
    uint32_t c_inv, c3;
    uint32_t lflags;
    Geom g;
    uint32_t seg, E;
    uint32_t fill[4];
    uint32_t fill_nan;
    uint32_t fast;
    // k_encode_pair (zhip_encode_mapped): row map and per-lane constants as in
    // the two-unit decode; rows of 2^row_shift bytes, r_oy = arr stride of dim ndim-2
    const zhip_rowblk* rowmap;
    const uint32_t* kpair;
    const uint32_t* pair_tab;  // k_encode_pair: the 11/11/10 tables and their lane constants (kpair11)
    const uint32_t* kpair11;
    uint32_t row_shift;
    int64_t r_oy;
    uint32_t tune;
    // k_encode_tile4 (ZHIP_DF_TILE on a tile4 plan): see zhip_plan / k_decode_tile4
    int32_t tq;
    uint32_t t_per_chunk, tile4;
    uint32_t sstride[ZHIP_MAX_DIMS];
    const uint32_t* tz;
    const uint32_t* kq4;
    const uint32_t* kq2;  // k_encode_tile4's two-tile form: lane constants [T/2][kThreads] (null: four tiles)
    const struct TileEnt* tmap;
    // k_encode_tile (ZHIP_DF_TILE / ZHIP_DF_TILE_PREFIX, not tile4): one tile
    // per workgroup; horner / kthread / kunit / c_inv are the tile tables then
    uint32_t tile, n_qb, n_cb;
    zhip_fdiv d_qb, d_cb;
    // k_encode_tileg (tile == 2): group map, step multiply table, steps
    const struct GroupEnt* gmap;
    const uint32_t* gtz;
    uint32_t n_groups, g_step_t, n_sub;
    uint32_t g_z2;  // k_encode_tileg's two-tile form: x^(8 * 2 g_step_t), the first half's shift to ku's frame
    // tuning arm 68 (k_encode_tileg, four accumulators through one byte-table
    // operator): the A4 fold tables and x^(-96), the folded state's frame
    const uint32_t* g_a4;
    uint32_t g_c96;
    int64_t g_step_o;
    uint32_t xcd_run;     // k_encode_pair: pairs per XCD-contiguous run (0: dispatch order)
    // 64-bit words between chunks' publication words (k_encode_pair / k_encode_tile4):
    // kPubLine / 2 for CRC layouts (a 128-byte line per chunk), else 2
    uint32_t pub_stride;
    // k_encode_il: k_decode_il's interleave stride, tables and lane constants
    // (0: not available for this plan)
    uint32_t il_S;
    const uint32_t* il_tab;
    const uint32_t* il_klane;
    // ZHIP_DF_WHOLE (k_encode_il's AFF form): DecodeParams' aff_* fields
    uint32_t aff_ok, aff_sh, aff_mask;
    int32_t aff_B, aff_C, aff_D;
};

struct PackParams {
    uint8_t* dst;
    const zhip_shard* shards;
    const uint32_t* nonempty;      // per inner chunk, chunk id = first_chunk + Morton rank
    uint32_t* newrank;             // scratch per inner chunk
    const uint32_t* rank_of_slot;  // C-order slot -> Morton rank
    uint64_t* blob_len;            // out, per shard
    const uint32_t* horner;
    const uint32_t* kthread;
    uint32_t n_inner, elen, index_size, index_start, index_crc, keep_empty;
    uint32_t idx_c_inv, idx_c3;
};

int launch_decode(const DecodeParams& p, hipStream_t stream, int max_grid);
int launch_encode(const EncodeParams& p, hipStream_t stream, int max_grid);
int launch_shard_pack(const PackParams& p, uint32_t n_shards, hipStream_t stream);
int launch_dv_check(const zhip_dv_ref* d_refs, uint32_t n_refs, hipStream_t stream);
int debug_stamps(uint64_t* host_out, uint32_t n_wg);

}  // namespace zhip

struct zhip_plan;
namespace zhip {
void fill_geom(Geom& g, const zhip_plan& plan);
}

struct zhip_plan {
    zhip_layout layout;
    uint32_t kblocks;  // K: blocks per thread per unit (4, 8 or 16)
    uint32_t seg;      // kWgStride * K
    uint32_t nseg;
    uint32_t E;
    uint64_t R;
    uint32_t c_inv, c3;
    uint32_t hx[4];    // x^(8(4096 - 4k)), k = 0..3: the Horner operators
    uint32_t kq[32];   // x^(8(4096 - 256a)), a < 16 | x^(-128b), b < 16 (lane_kthread)
    zhip_fdiv dshape[ZHIP_MAX_DIMS];
    uint32_t row_bytes;
    zhip_fdiv drow;
    uint32_t fill[4];
    int device;
    int max_grid;
    uint32_t* d_tables;  // horner (4096) | kthread (256) | kunit (nseg) | kpair (nseg * 256) |
                         // pair tables (kPairTabWords) | kpair11 (nseg * 256) | kthread11 (256)
    uint64_t off_pair;   // u32 offset of the pair tables in d_tables
    // tile mode (layouts with a transposed dim that is contiguous in out)
    int32_t tq;          // -1: no tile mode
    uint32_t t_per_chunk, n_qb, n_cb;
    uint32_t sstride[ZHIP_MAX_DIMS];
    uint32_t t_c_inv;
    // k_decode_tile4 (full tiles, groups of 4 tiles at a uniform base step):
    // d_tile_tables continues with tz (1024: multiply by x^(8 step)) | kq4
    // ((T/4) * 256: kthread * kunit[last tile of the group] * t_c_inv) | tmap (T)
    uint32_t tile4;
    uint64_t tile4_step;                                 // base step between consecutive tiles
    uint64_t tile4_off_tz, tile4_off_kq, tile4_off_map;  // u32 offsets in d_tile_tables
    // k_decode_tile4f (tile step 256 B, CRC): A_64 tables in the kPairTab*
    // layout | lane constants [T/4][kThreads], at tile4f_off in d_tile_tables
    uint32_t tile4f;
    uint64_t tile4f_off;
    // k_decode_tile4w (tile4 layouts with a CRC): A_(4 sq) tables in the
    // kPairTab* layout | lane constants [T/4][kThreads], at tile4w_off
    uint32_t tile4w;
    uint64_t tile4w_off;
    uint64_t tile2w_off;  // lane constants [T/2][kThreads] of k_decode_tile4w's two-tile form (0: none)
    uint64_t tile1w_off;  // tuning builds: lane constants [T][kThreads] of the one-tile form (0: none)
    uint64_t tileg2w_off; // lane constants [2 n_groups][kThreads] of k_decode_tilegw's two-tile form (0: none)
    uint64_t tilegl_off;  // tuning builds: lane constants [n_groups][kThreads] of its lane-tile form (0: none)
    uint64_t tilebt_off;  // tuning builds: A_(4 sq) byte tables + A4 (kByteTabWords) for arms 66 / 67 (0: none)
    uint64_t tile2e_off;  // lane constants [T/2][kThreads] of k_encode_tile4's two-tile form (0: none)
    // full-tile layouts that tile4 declines (e.g. 128^3 chunks: the four tiles
    // of a natural group at two steps) but whose consecutive tile pairs are the
    // two column blocks of one row band: k_decode_tile4w<2> over pairs (2 k,
    // 2 k + 1), tuning arm 39; d_tile_tables at tile2_off (tuning builds): A_(4 sq)
    // pair tables | tile map (T TileEnt) | lane constants [T/2][kThreads]
    uint32_t tile2;
    uint64_t tile2_off;
    // the whole-chunk row map of a whole-row layout in two-level affine form
    // (plan_affine; ZHIP_DF_WHOLE launches): aff_ok, shift, B, C, D
    uint32_t aff_ok, aff_sh;
    int32_t aff_B, aff_C, aff_D;
    // k_decode_tilegw (grouped tile layouts with a CRC): the same for groups
    uint32_t tilegw;
    uint64_t tilegw_off;
    // k_encode_tileg (full selections): tiles grouped by four along the
    // innermost other stored dim gd with shape[gd] % 4 == 0 (uniform step
    // sstride[gd] inside every group, whatever the natural tile order); tables
    // tzg (1024: multiply by x^(8 sstride[gd])) | gmap (n_groups GroupEnt)
    int32_t gd;                      // -1: no such dim
    uint32_t n_groups;
    uint32_t n_sub;                  // > 16 groups per chunk: arrival subgroups of 16 (workspace tail)
    uint64_t g_off_tz, g_off_map;    // u32 offsets in d_tile_tables
    uint32_t* d_tile_tables;
    // shard index (sharded layouts): payload 16*n_inner, E, CRC constants
    uint32_t idx_nbytes, idx_E, idx_c_inv, idx_c3;  // horner (stride 16*sstride[tq]) | kthread (256) | kunit (t_per_chunk)
    // k_decode_il (interleaved steps, decode_rows.hip): a workgroup takes K = 8
    // of the chunk's 4 KiB steps at a stride of il_S steps (il_S = 0: not
    // available for this layout).  d_tables continues at off_il with the
    // 11/11/10 tables of A_(4096 il_S) (kPairTabWords) | klane (nseg x 256:
    // per workgroup-in-chunk lane constants) | kidx (256: the fused index
    // check's lane constants under those tables)
    uint32_t il_S;
    uint64_t off_il;
    // k_decode_xw (decode_rows.hip): xw_P = 8 KiB spans per chunk (0: not
    // available), xw_nsub = two-level arrival subwords (P > 32, P <= 1024).
    // d_tables continues at off_xw with the tables of A_1024 | klane (P x 64) |
    // kidx (256)
    uint32_t xw_P, xw_nsub;
    uint64_t off_xw;
    // k_decode_ilw (decode_rows.hip): one 32 KiB unit per workgroup of NT =
    // 512 / 1024 lanes (2048 / NT blocks per lane); d_tables continues at
    // off_ilw[0] (NT = 1024) / off_ilw[1] (NT = 512) with the tables of
    // A_(16 NT) | klane (nseg x NT) | kidx (256); 0: not built
    uint64_t off_ilw[2];
    uint64_t off_ilh;
    uint64_t off_il_s[2];  // tuning builds: k_decode_il's tables for S = 16 / 32 (arms 69 / 70; 0: none)  // tuning builds: k_decode_ilh's lane constants [2 nseg][kThreads] (0: none)
};
