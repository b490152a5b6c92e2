/*
 * zarrhip.h — C ABI of the MI355X-native zarr v3 codec-pipeline kernels.
 *
 * This is the drop-in boundary below zarr-python's CodecPipeline interface
 * (src/zarr/abc/codec.py:315-508 in the reference).  A host planner (the
 * Python package zarr_hip, mirroring CodecPipeline.read/write) turns a batch of
 * (ByteGetter, ArraySpec, chunk_selection, out_selection, is_complete) tuples
 * into the flat tables below and calls these entry points through ctypes.  No
 * torch or C++ types cross the boundary: plain pointers, sizes, POD structs.
 *
 * Entry points and the reference interface each one replaces:
 *
 *   zhip_decode       FusedCodecPipeline.read_sync's per-chunk body
 *                     (src/zarr/core/codec_pipeline.py:1095-1172):
 *                       Crc32cCodec._decode_sync   (src/zarr/codecs/crc32c_.py:34-50)
 *                       BytesCodec._decode_sync    (src/zarr/codecs/bytes.py:97-131)
 *                       TransposeCodec._decode_sync(src/zarr/codecs/transpose.py:98-104)
 *                       decode_and_scatter_chunk / scatter_chunk
 *                                                  (src/zarr/core/chunk_utils.py:88-214)
 *                     and, for sharded batches, the sub-chunk extraction of
 *                       ShardingCodec._decode_partial_sync (src/zarr/codecs/sharding.py:1222-1309)
 *                       _ShardIndex.get_chunk_slice        (sharding.py:248-254)
 *                     With ZHIP_LF_NO_WRITE the same entry point is the
 *                     shard-index CRC check of _decode_shard_index_sync
 *                     (sharding.py:624-631) run over many shards at once.
 *   zhip_decode_indexed  zhip_decode with that index check fused into the
 *                     same launch.
 *   zhip_encode       ChunkTransform.encode_chunk for fixed-size chains
 *                     (chunk_utils.py:335-363): transpose/bytes/crc32c _encode_sync
 *                     (transpose.py:113-118, bytes.py:140-158, crc32c_.py:59-68) plus
 *                     chunk_is_empty (chunk_utils.py:74-85, buffer/core.py:534-558).
 *   zhip_shard_pack   ShardingCodec._build_shard_layout / _assemble_shard /
 *                     _encode_shard_index_sync (sharding.py:887-950, 633-640).
 *   zhip_plan_*       host-side constant tables (no reference counterpart:
 *                     the CRC-combine operators the GPU kernels need).
 *
 * Error model: every function returns 0 on success or a negative ZHIP_E_*
 * code; zhip_last_error() gives a message.  Per-chunk outcomes are written to
 * device-resident zhip_status records; the host raises the reference's
 * exceptions (ValueError "Stored and computed checksum do not match ...") after
 * the batch completes.  No exception crosses the ABI.
 */
#ifndef ZARRHIP_H
#define ZARRHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZHIP_ABI_VERSION 1
#define ZHIP_MAX_DIMS 8

/* return codes */
#define ZHIP_OK 0
#define ZHIP_E_INVALID -1
#define ZHIP_E_HIP -2
#define ZHIP_E_UNSUPPORTED -3
#define ZHIP_E_IO -4          /* a file piece could not be read in full (zhip_stage_*) */
#define ZHIP_E_BOUNDS -5      /* an output table is too small (the counts are still returned),
                                 or a shard blob is shorter than its index */

/* per-chunk status codes (zhip_status.code) */
#define ZHIP_ST_OK 0u
#define ZHIP_ST_MISSING 1u            /* chunk absent: fill value scattered  */
#define ZHIP_ST_CRC_MISMATCH 2u       /* Crc32cCodec._decode_sync ValueError */
#define ZHIP_ST_INDEX_OOB 3u          /* shard index entry outside the blob  */
#define ZHIP_ST_LENGTH_MISMATCH 4u    /* encoded length != fixed-size chain  */

/* layout flags (zhip_layout.flags) */
#define ZHIP_LF_CRC 1u            /* chain ends in crc32c (4-byte LE trailer)        */
#define ZHIP_LF_SWAP 2u           /* stored endian != native: byteswap items        */
#define ZHIP_LF_SHARDED 4u        /* chunk source = inner chunk of a shard blob     */
#define ZHIP_LF_INDEX_START 8u    /* sharding index_location == "start"             */
#define ZHIP_LF_NO_WRITE 16u      /* verify only (shard index CRC)                  */
#define ZHIP_LF_FLOAT 32u         /* items are IEEE floats (NaN-aware fill equality) */

/* chunk flags (zhip_chunk.flags) */
#define ZHIP_CF_MISSING 1u        /* store returned None: scatter fill value        */

typedef struct zhip_fdiv {  /* n / d == (n * m) >> s  for 0 <= n < 2^31 */
    uint32_t m;
    uint32_t s;
} zhip_fdiv;

/* Geometry shared by every chunk of one launch (one array, one codec chain).
 * All per-dimension arrays are in STORED (encoded) dimension order: stored
 * dim i is decoded dim order[i] of the transpose codec (transpose.py:89-96),
 * so out_stride[i] is the out byte-stride of decoded dim order[i]. */
typedef struct zhip_layout {
    int32_t ndim;
    int32_t itemsize;                  /* 1, 2, 4 or 8 */
    int32_t shape[ZHIP_MAX_DIMS];      /* stored chunk shape (inner chunk if sharded) */
    int64_t out_stride[ZHIP_MAX_DIMS]; /* bytes; arbitrary (F order, views, drops)   */
    uint64_t nbytes;                   /* decoded bytes per chunk = prod(shape)*item */
    uint32_t flags;                    /* ZHIP_LF_*                                   */
    uint32_t n_inner;                  /* sharded: inner chunks per shard             */
    uint32_t index_size;               /* sharded: encoded index bytes (16n [+4])     */
    uint32_t _pad;
    uint8_t fill[16];                  /* fill value bytes, native order              */
} zhip_layout;

/* One chunk (decode unit) of a batch. */
typedef struct zhip_chunk {
    uint64_t src;      /* byte offset in src: encoded chunk | shard blob (SHARDED) */
    uint64_t src_len;  /* encoded chunk length | shard blob length                 */
    int64_t out_off;   /* byte offset in out of the selection's first element      */
    uint32_t flags;    /* ZHIP_CF_*                                                */
    uint32_t slot;     /* SHARDED: C-order index of the inner chunk in its shard   */
    uint32_t sel;      /* index into the selection table                           */
    uint32_t _pad[3];
} zhip_chunk;

/* Per-chunk selection (chunk_selection of a ChunkProjection), stored dim order:
 * element s of dim i is selected iff s = start + k*step, 0 <= k < count; it
 * lands at out_off + sum_i k_i * out_stride[i]. */
typedef struct zhip_sel {
    int32_t start[ZHIP_MAX_DIMS];
    int32_t count[ZHIP_MAX_DIMS];
    int32_t step[ZHIP_MAX_DIMS];
    zhip_fdiv div_step[ZHIP_MAX_DIMS];
} zhip_sel;

/* Per-chunk outcome, written by the device. */
typedef struct zhip_status {
    uint32_t code;     /* ZHIP_ST_* */
    uint32_t stored;   /* stored CRC (LE trailer), when ZHIP_LF_CRC              */
    uint32_t computed; /* CRC-32C computed on the device, when ZHIP_LF_CRC       */
    uint32_t aux;
} zhip_status;

/* One shard of an encode batch (zhip_shard_pack). */
typedef struct zhip_shard {
    uint64_t blob;         /* byte offset of the shard blob in dst                */
    uint32_t first_chunk;  /* id of its Morton-rank-0 inner chunk in the batch    */
    uint32_t _pad;
} zhip_shard;

typedef struct zhip_plan zhip_plan;

int zhip_abi_version(void);
const char *zhip_last_error(void);
int zhip_device_count(void);

/* Build the constant tables for one layout (host math + one upload to the
 * current device).  Not for the timed path: cache the plan per array. */
int zhip_plan_create(const zhip_layout *layout, zhip_plan **plan);
int zhip_plan_destroy(zhip_plan *plan);
/* Units (workgroup work items) per chunk and workspace words per chunk
 * (>= 32 for layouts with a crc32c: one 128-byte publication line per chunk). */
int zhip_plan_info(const zhip_plan *plan, uint32_t *units_per_chunk, uint32_t *workspace_words);
/* Which specialised kernels the plan's layout admits (ZHIP_PK_* bits). */
#define ZHIP_PK_TILE4 1u  /* transposed layout with full 64 x 256-byte tiles: k_decode_tile4 */
#define ZHIP_PK_TILE4_ENCODE 2u  /* ... and at most 64 tiles per chunk: zhip_encode_mapped with
                                    ZHIP_DF_TILE runs k_encode_tile4 (writes every non-empty flag) */
#define ZHIP_PK_TILE 4u  /* transposed layout tiled through LDS (a stored dim other than the
                            innermost is contiguous in out, rows of 16-byte multiples):
                            ZHIP_DF_TILE / ZHIP_DF_TILE_PREFIX encodes take k_encode_tile
                            when k_encode_tile4 does not apply */
#define ZHIP_PK_TILEG 8u /* ... and its tiles group by four along a stored dim with shape % 4 == 0
                            (whole 16-byte pieces along the out-contiguous dim): where
                            k_decode_tile4 / k_encode_tile4 do not apply, full-selection
                            batches run k_decode_tileg / k_encode_tileg */
#define ZHIP_PK_IL 16u   /* whole-row layout whose chunks decode in k_decode_il by default
                            (groups of eight 32 KiB workgroups, a trailing crc32c): that
                            kernel resolves its units itself, a load-address prediction
                            (zhip_predict) is not used */
int zhip_plan_kernel_flags(const zhip_plan *plan, uint32_t *flags);

/* decode flags (zhip_decode decode_flags) */
#define ZHIP_DF_FAST_ROWS 1u  /* every chunk selects whole innermost rows that are
                                 contiguous in out, 16-byte multiples and 16-byte
                                 aligned: one 16-byte store per 16 input bytes */
#define ZHIP_DF_TILE 2u       /* transposed layout: every chunk fully selected, the
                                 out-contiguous stored dim is tiled through LDS;
                                 out offsets/strides 16-byte aligned */
#define ZHIP_DF_TILE_PREFIX 8u /* encode, transposed layout (ZHIP_PK_TILE): every
                                  selection is a prefix box (start 0, unit steps,
                                  counts <= shape); elements past it are fill */
#define ZHIP_DF_ROWS 4u       /* with ZHIP_DF_FAST_ROWS: every selection has unit
                                 steps, innermost rows are 2^k <= 4096 bytes and
                                 shape[ndim-2] is a multiple of 4096/row_bytes
                                 (ndim >= 2): affine per-step addressing */
#define ZHIP_DF_BANK1 16u     /* deferred CRC verdicts (below): this launch publishes
                                 into workspace bank 1 and checks bank 0 (else the
                                 reverse); the caller alternates it per launch */
#define ZHIP_DF_DEFER 32u     /* opt in to deferred CRC verdicts (below).  Without it
                                 every decode reports a chunk's CRC mismatch in its own
                                 launch (d_status + d_errflag), as zhip_decode documents */
#define ZHIP_DF_WHOLE 64u     /* with a row map (zhip_decode_mapped with ZHIP_DF_ROWS;
                                 accepted by zhip_encode_mapped, whose kernels keep the
                                 map): the caller states that every
                                 selection of d_sels is its chunk's whole region (start 0,
                                 count = shape, unit steps).  Where the plan's whole-chunk
                                 row map is two-level affine in the step (zhip_plan_info
                                 reports it), the row kernels then compute each step's
                                 destination instead of loading it from the map; the map
                                 is still required and used otherwise.  The statement is
                                 checked, not trusted: each workgroup reads its chunk's
                                 selection record and keeps the map for any selection that
                                 is not whole, so a wrong flag costs speed, never placement */

/* Deferred CRC verdicts (opt-in: ZHIP_DF_DEFER).  With the flag,
 * k_decode_tileg / k_decode_tilegw (the transposing decodes of chunks
 * larger than 64 tiles) publish each
 * workgroup's CRC contribution with a NON-returning atomic xor into the
 * chunk's workspace word of the launch's bank (4 words per chunk: bank b's
 * word at 4c + 2b, its stored trailer at 4c + 2b + 1, i.e.
 * {w0, s0, w1, s1}); the chunk's first workgroup also folds in the stored
 * trailer, so after the launch w_b = computed ^ stored: 0 for a matching
 * chunk, and s_b holds the stored trailer.  The verdict is read, and a
 * nonzero word cleared, by the next launch (its first workgroup per chunk
 * checks the other bank: status CRC_MISMATCH + errflag, sticky across graph
 * replays), by zhip_dv_check, or by the host after synchronising (a nonzero
 * w_b is Crc32cCodec's mismatch with stored s_b, computed w_b ^ s_b).  Every
 * other kernel leaves w0 and w1 zero once its launch completes (the returning
 * publications of k_decode_il / k_decode_tile4 use word 32 c of the
 * workspace, zhip_plan_info's >= 32 words per chunk of CRC layouts, and
 * clear it when the chunk's last workgroup arrives). */
typedef struct zhip_dv_ref {
    uint32_t *workspace;   /* a launch's d_workspace (4 words per chunk first) */
    zhip_status *status;   /* its d_status */
    uint32_t *errflag;     /* its d_errflag */
    uint32_t n_chunks, pad;
} zhip_dv_ref;
/* Fold the deferred verdicts of n_refs launches' workspaces (a device array
 * of zhip_dv_ref) into their statuses and error words and clear them: one
 * small kernel, e.g. the last node of a captured read loop. */
int zhip_dv_check(const zhip_dv_ref *d_refs, uint32_t n_refs, void *stream);

/* The per-call read's result check, generalised: n device ranges (srcs[i],
 * sizes[i] bytes) copied back behind the launches on `stream` into one
 * page-locked buffer, one stream synchronise, then concatenated into
 * host_out. */
int zhip_wait_ranges(const void *const *srcs, const uint64_t *sizes, uint32_t n, void *host_out, void *stream);

/* A launch's host tables in ONE host -> device copy on `stream`: part i
 * (sizes[i] bytes at parts[i]) lands at dev + offsets[i] (each part inside
 * [0, total)).  The parts are packed into a page-locked per-thread buffer of
 * the current device, reused once its previous copy has finished; the host
 * parts may be freed when the call returns. */
int zhip_upload(const void *const *parts, const uint64_t *sizes, const uint64_t *offsets, uint32_t n, void *dev,
                uint64_t total, void *stream);

/* Host planner for a batch of basic selections (zhip_plan_batch).  One item
 * of a CodecPipeline batch: its chunk (or shard) bytes, its chunk selection
 * per DECODED dim (step 0: an integer index `start`; slices normalised to
 * the chunk shape, step >= 1) and the byte offset of its out selection's
 * first element.  Replaces BasicIndexer's per-chunk projections
 * (src/zarr/core/indexing.py:390-468, 571-621) and, for sharded items,
 * ShardingCodec._decode_partial_sync's inner-chunk expansion
 * (src/zarr/codecs/sharding.py:1222-1309). */
typedef struct zhip_item {
    uint64_t src;
    uint64_t src_len;
    int64_t out_off;
    uint32_t missing;
    int32_t res;       /* with a zhip_resolved table: the item's shard row (-1: shard absent) */
    int64_t start[ZHIP_MAX_DIMS];
    int64_t stop[ZHIP_MAX_DIMS];
    int64_t step[ZHIP_MAX_DIMS];
} zhip_item;

typedef struct zhip_batch_geom {
    int32_t ndim;
    int32_t perm[ZHIP_MAX_DIMS];   /* stored dim s is decoded dim perm[s]                  */
    int64_t shape[ZHIP_MAX_DIMS];  /* decoded chunk (shard) shape                          */
    int64_t ost[ZHIP_MAX_DIMS];    /* out byte stride per decoded dim (0: absent from out) */
    int64_t inner[ZHIP_MAX_DIMS];  /* sharded: inner chunk shape; inner[0] == 0: unsharded */
    uint32_t index_size;           /* sharded: encoded index bytes                          */
    uint32_t index_start;          /* sharded: index_location == "start"                   */
    uint32_t index_crc;            /* sharded: the index chain ends in crc32c               */
    uint32_t _pad;
} zhip_batch_geom;

/* Host-staged partial shard reads (the touched inner chunks already fetched
 * and staged by the host, staging.gather_sharded_partial): per shard row r
 * and inner slot j, the staged offset / length / absence of the inner chunk
 * (row-major [n_rows][n_inner]) and the staged offset of the row's index
 * bytes (-1: no index check).  Entries then read src[r][slot] directly (an
 * unsharded layout); index check entries are one per distinct index offset. */
typedef struct zhip_resolved {
    const uint64_t *src;
    const uint64_t *len;
    const uint8_t *missing;
    const int64_t *index_src;
    uint32_t n_rows, n_inner;
} zhip_resolved;

/* aggregate flags over the planned entries (layout-independent halves of the
 * kernel choice) */
#define ZHIP_AGG_LAST_FULL 1u    /* every entry selects whole innermost stored rows        */
#define ZHIP_AGG_OUT_ALIGNED 2u  /* every entry's out offset is a multiple of 16 bytes     */
#define ZHIP_AGG_UNIT_STEPS 4u   /* every stored dim has step 1 or selects one index       */
#define ZHIP_AGG_ALL_FULL 8u     /* every entry selects its whole chunk                    */

/* Plan a batch: chunk entries (inner chunks of sharded items, in item order,
 * C order within an item) with their deduplicated selections (sorted rows),
 * the item of each entry, and for sharded items with a CRC'd index one index
 * check entry per distinct shard.  `res` (NULL: none) plans host-staged
 * partial shard reads (zhip_resolved).  Capacities too small: ZHIP_E_BOUNDS with
 * *n_chunks / *n_sels / *n_idx set to the sizes needed. */
int zhip_plan_batch(const zhip_batch_geom *g, const zhip_item *items, uint32_t n_items,
                    const zhip_resolved *res, zhip_chunk *chunks, uint64_t chunks_cap, uint64_t *n_chunks,
                    zhip_sel *sels, uint32_t sels_cap, uint32_t *n_sels, uint32_t *item_of,
                    zhip_chunk *idx_chunks, uint32_t *idx_item, uint32_t *n_idx, uint32_t *agg);

/* Upload the plan's constant tables to the current HIP device (once). */
int zhip_plan_upload(zhip_plan *plan);

/* Decode `n_chunks` chunks of `src` (device) into `out` (device).
 * src must stay readable for 64 bytes past src_size (loads are 16-byte wide).
 * d_chunks/d_sels/d_status/d_workspace/d_errflag are device pointers;
 * d_workspace holds workspace_words (zhip_plan_info; 4 for most layouts) * n_chunks zeroed
 * uint32 words (8-byte aligned) (self-resetting: keep it
 * for the next call).  *d_errflag gets the OR of (1 << status code) over all
 * chunks whose status is an error (not OK, not MISSING).  `stream` is a
 * hipStream_t (NULL = default stream).  Asynchronous.  With ZHIP_LF_NO_WRITE
 * (shard-index CRC verification, itemsize 1) `out` may be NULL.  A CRC
 * mismatch is in d_status / d_errflag once the launch completes, unless the
 * caller opts in to deferred verdicts (ZHIP_DF_DEFER: then read them from the
 * workspace bank words, zhip_dv_check or the next launch). */
int zhip_decode(const zhip_plan *plan, const void *src, uint64_t src_size, void *out,
                const zhip_chunk *d_chunks, uint32_t n_chunks, const zhip_sel *d_sels,
                zhip_status *d_status, uint32_t *d_workspace, uint32_t *d_errflag,
                uint32_t decode_flags, void *stream);

/* zhip_decode plus, in the same launch, the shard-index CRC check of
 * _decode_shard_index_sync (sharding.py:624-631) for `n_index` indexes:
 * d_index_chunks[j].src / src_len locate index j (16*n_inner payload bytes +
 * the 4-byte CRC trailer) in src; its outcome goes to d_index_status[j].
 * Workgroup g of the decode grid checks indexes g, g+G, ... while its first
 * data unit loads (no second launch).  Needs a sharded plan (ZHIP_LF_SHARDED)
 * with ZHIP_LF_CRC (the CRC tables) and no ZHIP_DF_TILE; otherwise returns
 * ZHIP_E_UNSUPPORTED and the caller verifies the indexes with a separate
 * ZHIP_LF_NO_WRITE zhip_decode. */
int zhip_decode_indexed(const zhip_plan *plan, const void *src, uint64_t src_size, void *out,
                        const zhip_chunk *d_chunks, uint32_t n_chunks, const zhip_sel *d_sels,
                        zhip_status *d_status, uint32_t *d_workspace, uint32_t *d_errflag,
                        const zhip_chunk *d_index_chunks, uint32_t n_index,
                        zhip_status *d_index_status, uint32_t decode_flags, void *stream);

/* Load-address prediction for whole-row batches (ZHIP_DF_ROWS): the host
 * asserts that the payload of chunk entry c starts at byte
 *     base + (c / per) * outer + (c % per) * inner
 * of src (e.g. inner chunks packed in Morton order inside equally spaced shard
 * blobs, entries sorted by address), every predicted range lying inside its
 * entry's blob.  The kernel issues the unit loads from the predicted address
 * before the chunk record / shard-index entry arrive, then checks the
 * prediction against the live index and reloads on a mismatch: results never
 * depend on the prediction being right, only the start-up latency does. */
typedef struct zhip_predict {
    uint64_t base, outer, inner;
    uint32_t per;    /* >= 1 */
    uint32_t _pad;
} zhip_predict;

/* zhip_decode_indexed with an optional prediction (NULL = none). */
int zhip_decode_predicted(const zhip_plan *plan, const void *src, uint64_t src_size, void *out,
                          const zhip_chunk *d_chunks, uint32_t n_chunks, const zhip_sel *d_sels,
                          zhip_status *d_status, uint32_t *d_workspace, uint32_t *d_errflag,
                          const zhip_chunk *d_index_chunks, uint32_t n_index,
                          zhip_status *d_index_status, uint32_t decode_flags,
                          const zhip_predict *pred, void *stream);

/* Row map for ZHIP_DF_ROWS launches: where each 4096-byte step of every unit
 * lands in `out`, precomputed on the host from the same selections the device
 * table holds (the scatter of chunk_utils.py:88-214 for whole-row layouts,
 * evaluated once per plan instead of per workgroup).  Entry
 * [(s * nseg + u) * 8 + k] covers step k of unit u (u = 0 ends at the chunk's
 * last byte) of selection s: lane rows [lo, hi) of the step are inside the
 * selection and row 0 goes to out + chunk.out_off + rel. */
typedef struct zhip_rowblk {
    int32_t rel;
    uint16_t lo, hi;
} zhip_rowblk;

/* Number of zhip_rowblk entries zhip_rows_map writes for n_sels selections. */
uint64_t zhip_rows_map_len(const zhip_plan *plan, uint32_t n_sels);

/* Fill h_map (host memory, map_len entries) from host copies of the
 * selections.  ZHIP_E_UNSUPPORTED when the plan is not a whole-row layout or
 * an offset does not fit 32 bits (launch without a map then). */
int zhip_rows_map(const zhip_plan *plan, const zhip_sel *h_sels, uint32_t n_sels, zhip_rowblk *h_map,
                  uint64_t map_len);

/* zhip_decode_predicted with the row map uploaded to the device (d_rowmap,
 * NULL = none): whole-row launches with a map run the two-unit decode
 * (k_decode_pair), without one the persistent row decode. */
int zhip_decode_mapped(const zhip_plan *plan, const void *src, uint64_t src_size, void *out,
                       const zhip_chunk *d_chunks, uint32_t n_chunks, const zhip_sel *d_sels,
                       zhip_status *d_status, uint32_t *d_workspace, uint32_t *d_errflag,
                       const zhip_chunk *d_index_chunks, uint32_t n_index,
                       zhip_status *d_index_status, uint32_t decode_flags,
                       const zhip_predict *pred, const zhip_rowblk *d_rowmap, void *stream);

/* Process-wide tuning / ablation knobs for measurement (never needed for
 * correct operation): ZHIP_TUNE_MAX_GRID = persistent-grid cap (0 = auto),
 * ZHIP_TUNE_ABLATION = ablation bits (0 = production). */
#define ZHIP_TUNE_MAX_GRID 1
#define ZHIP_TUNE_ABLATION 2
#define ZHIP_TUNE_BLOCKS 3   /* blocks/thread per unit for plans created afterwards (4, 8, 16) */
#define ZHIP_TUNE_STAGE_STREAMS 4  /* host staging: packed windows on 1 (default) or 2 copy streams */
#define ZHIP_TUNE_STAGE_COPY 5     /* host copies into / out of pinned memory: 1 streaming stores (default), 0 memcpy */
#define ZHIP_TUNE_ARM 6            /* experimental kernel variant for timing arms (0 = production) */
/* MAX_GRID / ABLATION / BLOCKS / ARM exist in the tuning build only
 * (libzarrhip_tune.so, -DZHIP_TUNING=1); the shipped library accepts 0 and
 * returns ZHIP_E_UNSUPPORTED for anything else.  1 when this library is the
 * tuning build. */
int zhip_tuning_build(void);
int zhip_set_tuning(int key, int value);

/* Name of the kernel the last zhip_decode* (or row-mapped zhip_encode_mapped)
 * call on this process launched ("k_decode_il", "k_decode_ilw512",
 * "k_decode_pair", "k_decode_lead", "k_encode_il", ...): a diagnostic for
 * labels and tests; not synchronised across threads. */
const char *zhip_last_kernel(void);

/* Diagnostics: with ablation bit 1024 set, k_decode_pair records per-workgroup
 * phase timestamps (s_memrealtime, 100 MHz) for the first 8192 workgroups of
 * each launch; copies n_wg * 8 u64 stamps (+ hardware id) to host memory.  Not
 * used on the product path. */
int zhip_debug_stamps(uint64_t *host_out, uint32_t n_wg);

/* Encode `n_chunks` chunks gathered from the device array `arr` into `dst`.
 * Per chunk: zhip_chunk.src = byte offset of the encoded chunk in dst (its
 * N [+4] bytes are written there), out_off = byte offset in arr of the chunk's
 * selection origin, sel = selection (stored dims) — elements outside it are
 * written as the fill value (edge chunks, _merge_chunk_array).  With
 * ZHIP_LF_CRC the CRC-32C trailer is appended and also reported in
 * d_status[i].computed.  d_nonempty[i] is set to 1 if any element differs
 * from the fill value under NDBuffer.all_equal rules, else 0 (every launch
 * writes every flag: kernels that OR flags are preceded by an async zeroing
 * of d_nonempty on the same stream).
 * ZHIP_DF_FAST_ROWS: every chunk selects whole rows that are contiguous and
 * 16-byte aligned in arr.  Asynchronous. */
int zhip_encode(const zhip_plan *plan, const void *arr, void *dst, const zhip_chunk *d_chunks,
                uint32_t n_chunks, const zhip_sel *d_sels, zhip_status *d_status,
                uint32_t *d_workspace, uint32_t *d_nonempty, uint32_t encode_flags, void *stream);

/* zhip_encode with the row map of the batch's selections (zhip_rows_map over
 * the same layout, where out_stride holds the source array's strides): the
 * whole-row chunks then encode in the two-unit kernel (k_encode_pair). */
int zhip_encode_mapped(const zhip_plan *plan, const void *arr, void *dst, const zhip_chunk *d_chunks,
                       uint32_t n_chunks, const zhip_sel *d_sels, zhip_status *d_status, uint32_t *d_workspace,
                       uint32_t *d_nonempty, uint32_t encode_flags, const zhip_rowblk *d_rowmap, void *stream);

/* Host -> HBM staging (replaces the host-buffer fetches the reference's
 * pipelines do per chunk: ByteGetter.get_sync / Store.get_ranges_sync,
 * src/zarr/abc/store.py:474-539, src/zarr/core/codec_pipeline.py:1095-1172).
 * One piece = `nbytes` host bytes at `host`, bound for `dst_off` in the
 * staging buffer; pieces sorted by dst_off, non-overlapping. */
typedef struct zhip_piece {
    uint64_t host;     /* host address (ZHIP_PIECE_FILE: a NUL-terminated file path) */
    uint64_t nbytes;
    uint64_t dst_off;  /* offset in the pinned and device buffers */
    uint64_t flags;    /* ZHIP_PIECE_* */
    uint64_t file_off; /* ZHIP_PIECE_FILE: byte offset in the file */
} zhip_piece;

/* The piece's host bytes are page-locked (a pinned store's arena, a pinned
 * tensor): DMA them straight to `dev`, no packing.  Runs of such pieces that
 * are contiguous in both host and device order go as one copy. */
#define ZHIP_PIECE_PINNED 1u
/* The piece is nbytes of a file (LocalStore, src/zarr/storage/_local.py):
 * the packing thread preads them straight into the pinned window -- no
 * Python read, no intermediate bytes object. */
#define ZHIP_PIECE_FILE 2u

/* Pack the pageable pieces into `pinned` (total bytes) with `nthreads` host
 * threads, window by window; each window's packed runs are copied to `dev`
 * by hipMemcpyAsync on `stream` as soon as the window is packed (pinned
 * pieces are copied directly first).  Gaps of 256 bytes or more that no
 * piece covers are left as they are in `dev`.  Returns once every copy is enqueued (they complete
 * asynchronously on `stream`). */
int zhip_stage_h2d(const zhip_piece *pieces, uint32_t n_pieces, uint8_t *pinned, void *dev, uint64_t total,
                   uint64_t window, uint32_t nthreads, void *stream);

/* zhip_stage_h2d started on a library thread: returns at once (NULL on
 * allocation failure); the pieces array is copied.  Jobs run in the order they
 * were begun.  zhip_stage_end waits for the job's copies to be enqueued, makes
 * `wait_stream` (a hipStream_t; NULL is the default stream) wait for exactly
 * them (and earlier jobs'), and returns zhip_stage_h2d's code. */
typedef struct zhip_stage_job zhip_stage_job;
zhip_stage_job *zhip_stage_begin(const zhip_piece *pieces, uint32_t n_pieces, uint8_t *pinned, void *dev,
                                 uint64_t total, uint64_t window, uint32_t nthreads, void *stream);
int zhip_stage_end(zhip_stage_job *job, void *wait_stream);

/* 1 when p points into page-locked host memory known to HIP (a pinned
 * result buffer can take the D2H DMA directly), else 0. */
int zhip_host_pinned(const void *p);

/* Read n (<= 16) device words (each launch's 4-byte error flag) after the
 * work already on `stream`: async copies into page-locked memory, one stream
 * synchronise, the values into host_out.  The per-call read path's only
 * device -> host traffic when no chunk failed (FusedCodecPipeline.read_sync
 * returns statuses, codec_pipeline.py:1095-1172; the full status table is read
 * only when a flag is set). */
int zhip_wait_words(const uint32_t *const *words, uint32_t n, uint32_t *host_out, void *stream);

/* memcpy with `nthreads` host threads (pinned result -> a caller's host array). */
int zhip_host_copy(void *dst, const void *src, uint64_t nbytes, uint32_t nthreads);

/* shard pack flags */
#define ZHIP_PF_INDEX_START 1u   /* index_location == "start" */
#define ZHIP_PF_INDEX_CRC 2u     /* index codecs end in crc32c */
#define ZHIP_PF_KEEP_EMPTY 4u    /* write_empty_chunks: no elision */

/* Pack shards whose inner chunks zhip_encode wrote densely in Morton-rank order
 * at blob + data_start + rank*elen (data_start = index_size if the index is at
 * the start, else 0): elide empty inner chunks (compacting the rest), write the
 * index (LE u64 offset/length, 2^64-1 pairs for absent chunks) and its CRC.
 * d_rank_of_slot[i] = Morton rank of C-order slot i.  d_blob_len[s] receives
 * the final blob length (0 = every inner chunk empty: delete the shard).
 * `plan` is the inner-chunk plan (supplies the CRC tables).  Asynchronous. */
int zhip_shard_pack(const zhip_plan *plan, void *dst, const zhip_shard *d_shards, uint32_t n_shards,
                    uint32_t n_inner, uint32_t elen, uint32_t index_size, uint32_t pack_flags,
                    const uint32_t *d_nonempty, uint32_t *d_newrank, const uint32_t *d_rank_of_slot,
                    uint64_t *d_blob_len, void *stream);

/* Host CRC-32C (reflected 0x82F63B78, init / xorout 0xFFFFFFFF) of nbytes at
 * data: the host stage of a chain, where the bytes never reach the GPU -- a
 * crc32c after a host-side compressor (Crc32cCodec._decode_sync / _encode_sync,
 * src/zarr/codecs/crc32c_.py:34-68, on compressed bytes) and the index of a
 * shard whose inner chunks are compressed on the host
 * (ShardingCodec._encode_shard_index_sync, sharding.py:633-640). */
uint32_t zhip_crc32c_host(const void *data, uint64_t nbytes);

/* CPU-only test hooks (no GPU needed). */
int zhip_selftest(void);                                  /* 0 = all identities hold */
uint32_t zhip_emulate_chunk_crc(const zhip_plan *plan, const uint8_t *data);
/* The same for k_decode_pair's scheme (11/11/10-bit tables, four word
 * accumulators per lane, windowed per-lane multiply).  Test hook. */
uint32_t zhip_emulate_chunk_crc_pair(const zhip_plan *plan, const uint8_t *data);
/* The same for k_decode_il (a workgroup's eight 4 KiB steps interleaved at a
 * stride of S steps, A_(4096 S) tables); 0xFFFFFFFF when the plan has no
 * interleaved layout.  Test hook. */
uint32_t zhip_emulate_chunk_crc_il(const zhip_plan *plan, const uint8_t *data);
/* The same for k_decode_xw (lane l of 8 KiB span r: eight blocks 1 KiB apart,
 * A_1024 tables, per-(span, lane) constants); 0xFFFFFFFF when the plan has no
 * xw layout.  Test hook. */
uint32_t zhip_emulate_chunk_crc_xw(const zhip_plan *plan, const uint8_t *data);
uint32_t zhip_fdiv_eval(uint32_t n, uint32_t d);

#ifdef __cplusplus
}
#endif

#endif /* ZARRHIP_H */
