// Host planner for basic-selection batches (zhip_plan_batch): the per-call
// work of HipCodecPipeline.read_sync -- the reference's BasicIndexer
// projections of every item's chunk selection onto the inner-chunk grid
// (src/zarr/core/indexing.py:390-468, 571-621; sharded items expand into their
// touched inner chunks as ShardingCodec._decode_partial_sync does,
// src/zarr/codecs/sharding.py:1222-1309), the chunk / selection tables the
// kernels read, and the shard-index check list -- in one native call instead
// of a Python loop per item.  Produces exactly the tables
// zarr_hip/planner.py's plan_decode builds (tests/test_native_planner.py
// compares them table for table); the layout-level kernel choices stay in
// Python, fed by the aggregate flags returned here.

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/zarrhip.h"

namespace {

inline int64_t floordiv(int64_t a, int64_t b) {  // Python's a // b for b > 0
    int64_t q = a / b;
    if ((a % b != 0) && (a < 0)) --q;
    return q;
}

inline int64_t ceildiv(int64_t a, int64_t b) { return -floordiv(-a, b); }

struct DimProj {  // zarr_hip/indexing.py project_dim, one dim of one item
    std::vector<int64_t> ix, s0, cnt, out;
    int64_t step = 1;
};

bool project_dim(int64_t start, int64_t stop, int64_t step, bool is_int, int64_t dim_len, int64_t cl,
                 DimProj& d) {
    d.ix.clear();
    d.s0.clear();
    d.cnt.clear();
    d.out.clear();
    if (cl <= 0) return false;
    if (is_int) {
        if (start < 0 || start >= dim_len) return false;
        const int64_t ix = start / cl;
        d.ix.push_back(ix);
        d.s0.push_back(start - ix * cl);
        d.cnt.push_back(1);
        d.out.push_back(0);
        d.step = 1;
        return true;
    }
    if (step < 1) return false;
    d.step = step;
    if (start >= stop) return true;
    const int64_t ix_from = floordiv(start, cl), ix_to = floordiv(stop - 1, cl) + 1;
    for (int64_t ix = ix_from; ix < ix_to; ++ix) {
        const int64_t off = ix * cl;
        const int64_t clen = std::min(cl, dim_len - off);
        const int64_t limit = off + clen;
        const bool before = start < off;
        const int64_t rem = before ? (off - start) % step : 0;
        const int64_t s0 = before ? (rem > 0 ? step - rem : 0) : start - off;
        const int64_t o = before ? ceildiv(off - start, step) : 0;
        const int64_t s1 = stop > limit ? clen : stop - off;
        const int64_t cnt = std::max<int64_t>(0, ceildiv(s1 - s0, step));
        if (cnt > 0) {
            d.ix.push_back(ix);
            d.s0.push_back(s0);
            d.cnt.push_back(cnt);
            d.out.push_back(o);
        }
    }
    return true;
}

using SelKey = std::array<int64_t, 3 * ZHIP_MAX_DIMS>;

struct KeyHash {
    size_t operator()(const SelKey& k) const {
        uint64_t h = 1469598103934665603ull;
        for (int64_t v : k) {
            h ^= (uint64_t)v;
            h *= 1099511628211ull;
        }
        return (size_t)h;
    }
};

zhip_fdiv fdiv_of(uint32_t d) {
    zhip_fdiv f;
    if (d < 1) d = 1;
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    f.s = 31 + l;
    f.m = (uint32_t)(((1ull << (31 + l)) + d - 1) / d);
    return f;
}

}  // namespace

extern "C" {

int zhip_plan_batch(const zhip_batch_geom* g, const zhip_item* items, uint32_t n_items, const zhip_resolved* res,
                    zhip_chunk* chunks, uint64_t chunks_cap, uint64_t* n_chunks, zhip_sel* sels,
                    uint32_t sels_cap, uint32_t* n_sels, uint32_t* item_of, zhip_chunk* idx_chunks,
                    uint32_t* idx_item, uint32_t* n_idx, uint32_t* agg) {
    if (!g || (!items && n_items) || !n_chunks || !n_sels || !n_idx || !agg) return ZHIP_E_INVALID;
    const int nd = g->ndim;
    if (nd < 1 || nd > ZHIP_MAX_DIMS) return ZHIP_E_INVALID;
    for (int s = 0; s < nd; ++s)
        if (g->perm[s] < 0 || g->perm[s] >= nd) return ZHIP_E_INVALID;
    const bool sharded = g->inner[0] > 0;
    if (res && (!sharded || !res->src || !res->len || !res->missing || !res->index_src)) return ZHIP_E_INVALID;
    // the projection grid: inner chunks of the shard, or the chunk itself
    int64_t grid_chunk[ZHIP_MAX_DIMS], cps[ZHIP_MAX_DIMS], cps_stride[ZHIP_MAX_DIMS];
    for (int d = 0; d < nd; ++d) {
        grid_chunk[d] = sharded ? g->inner[d] : g->shape[d];
        if (grid_chunk[d] <= 0 || g->shape[d] <= 0) return ZHIP_E_INVALID;
        cps[d] = sharded ? g->shape[d] / g->inner[d] : 1;
    }
    cps_stride[nd - 1] = 1;
    for (int d = nd - 2; d >= 0; --d) cps_stride[d] = cps_stride[d + 1] * cps[d + 1];
    const int64_t* stored = sharded ? g->inner : g->shape;  // decoded shape of one decode unit
    uint64_t n = 0;
    uint32_t n_ix = 0;
    std::vector<DimProj> dp(nd);
    std::unordered_map<SelKey, uint32_t, KeyHash> sel_ix;
    std::vector<SelKey> keys;
    std::vector<uint32_t> sel_of;  // per chunk entry: index into keys (insertion order)
    std::unordered_set<uint64_t> idx_set;
    // aggregates for the layout-level kernel choice (planner._fast_ok / _rows_ok / _tile_ok)
    bool last_full = true, out_al16 = true, unit_or_single = true, all_full = true;
    const int last = nd - 1;
    for (uint32_t i = 0; i < n_items; ++i) {
        const zhip_item& it = items[i];
        const int64_t row = res ? (int64_t)it.res : -1;
        if (res && row >= (int64_t)res->n_rows) return ZHIP_E_INVALID;
        if (sharded && !res && !it.missing && it.src_len < g->index_size) {
            *n_chunks = 0;
            *n_sels = 0;
            *n_idx = 0;
            *agg = 0;
            return ZHIP_E_BOUNDS;  // a shard blob shorter than its index
        }
        size_t m = 1;
        for (int d = 0; d < nd; ++d) {
            const bool is_int = it.step[d] == 0;
            if (!sharded) {  // the item is one chunk: its selection as given (planner._sel_lists)
                DimProj& q = dp[d];
                q.ix.assign(1, 0);
                q.out.assign(1, 0);
                q.s0.assign(1, it.start[d]);
                q.cnt.assign(1, is_int ? 1 : std::max<int64_t>(0, ceildiv(it.stop[d] - it.start[d], it.step[d])));
                q.step = is_int ? 1 : it.step[d];
                if (!is_int && it.step[d] < 1) return ZHIP_E_INVALID;
                continue;
            }
            if (!project_dim(it.start[d], it.stop[d], it.step[d], is_int, g->shape[d], grid_chunk[d], dp[d]))
                return ZHIP_E_INVALID;
            m *= dp[d].ix.size();
        }
        if (m == 0) continue;
        if (n + m > chunks_cap) {  // count only: the caller sizes and calls again
            n += m;
            continue;
        }
        // C-order walk of the cartesian product (indexing.py basic_projections)
        size_t pos[ZHIP_MAX_DIMS] = {0};
        for (size_t e = 0; e < m; ++e) {
            zhip_chunk& ch = chunks[n];
            std::memset(&ch, 0, sizeof(ch));
            int64_t oo = it.out_off;
            int64_t slot = 0;
            SelKey key{};
            for (int d = 0; d < nd; ++d) {
                oo += dp[d].out[pos[d]] * g->ost[d];
                slot += dp[d].ix[pos[d]] * cps_stride[d];
            }
            for (int s = 0; s < nd; ++s) {  // stored dim s = decoded dim perm[s]
                const int d = g->perm[s];
                key[s] = dp[d].s0[pos[d]];
                key[ZHIP_MAX_DIMS + s] = dp[d].cnt[pos[d]];
                key[2 * ZHIP_MAX_DIMS + s] = dp[d].step;
            }
            ch.out_off = oo;
            ch.slot = sharded ? (uint32_t)slot : 0u;
            if (!res) {
                ch.src = it.src;
                ch.src_len = it.src_len;
                ch.flags = it.missing ? ZHIP_CF_MISSING : 0u;
            } else if (row < 0 || it.missing || (uint64_t)slot >= res->n_inner) {
                ch.flags = ZHIP_CF_MISSING;  // src / src_len stay 0
            } else {
                const size_t at = (size_t)row * res->n_inner + (size_t)slot;
                ch.src = res->src[at];
                ch.src_len = res->len[at];
                ch.flags = res->missing[at] ? ZHIP_CF_MISSING : 0u;
            }
            auto f = sel_ix.find(key);
            uint32_t k;
            if (f == sel_ix.end()) {
                k = (uint32_t)keys.size();
                sel_ix.emplace(key, k);
                keys.push_back(key);
            } else {
                k = f->second;
            }
            sel_of.push_back(k);
            if (item_of) item_of[n] = i;
            if (oo % 16 != 0) out_al16 = false;
            {
                const int64_t st = key[last], ct = key[ZHIP_MAX_DIMS + last], sp = key[2 * ZHIP_MAX_DIMS + last];
                if (!(st == 0 && ct == stored[g->perm[last]] && sp == 1)) last_full = false;
                for (int s = 0; s < nd; ++s) {
                    const int64_t c = key[ZHIP_MAX_DIMS + s], p = key[2 * ZHIP_MAX_DIMS + s];
                    if (!(p == 1 || c <= 1)) unit_or_single = false;
                    if (!(key[s] == 0 && p == 1 && c == stored[g->perm[s]])) all_full = false;
                }
            }
            ++n;
            for (int d = nd - 1; d >= 0; --d) {  // next coordinate, last dim fastest
                if (++pos[d] < dp[d].ix.size()) break;
                pos[d] = 0;
            }
        }
        // one index check per distinct shard (host-staged: per distinct staged
        // index copy, which only CRC'd indexes have)
        const bool has_ix = res ? (row >= 0 && !it.missing && res->index_src[row] >= 0)
                                : (sharded && !it.missing && g->index_crc);
        const uint64_t ix_src = res ? (has_ix ? (uint64_t)res->index_src[row] : 0)
                                    : it.src + (g->index_start ? 0 : it.src_len - g->index_size);
        if (has_ix && idx_set.insert(ix_src).second) {
            if (idx_chunks && n_ix < n_items) {
                zhip_chunk& ic = idx_chunks[n_ix];
                std::memset(&ic, 0, sizeof(ic));
                ic.src = ix_src;
                ic.src_len = g->index_size;
                if (idx_item) idx_item[n_ix] = i;
            }
            ++n_ix;
        }
    }
    *n_chunks = n;
    *n_idx = n_ix;
    if (n > chunks_cap) return ZHIP_E_BOUNDS;
    // deduplicated selections, sorted like numpy.unique(axis=0) over
    // (start..., count..., step...) rows (one row when every chunk is alike)
    const uint32_t nk = (uint32_t)keys.size();
    *n_sels = nk;
    if (nk > sels_cap) return ZHIP_E_BOUNDS;
    std::vector<uint32_t> order(nk), rank(nk);
    for (uint32_t k = 0; k < nk; ++k) order[k] = k;
    auto row = [&](uint32_t k, int j) {  // the numpy key row: nd starts, nd counts, nd steps
        return keys[k][(j / nd) * ZHIP_MAX_DIMS + (j % nd)];
    };
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        for (int j = 0; j < 3 * nd; ++j) {
            const int64_t x = row(a, j), y = row(b, j);
            if (x != y) return x < y;
        }
        return false;
    });
    for (uint32_t r = 0; r < nk; ++r) rank[order[r]] = r;
    for (uint32_t r = 0; r < nk; ++r) {
        const SelKey& k = keys[order[r]];
        zhip_sel& s = sels[r];
        std::memset(&s, 0, sizeof(s));
        for (int d = 0; d < ZHIP_MAX_DIMS; ++d) {
            const bool in = d < nd;
            s.start[d] = in ? (int32_t)k[d] : 0;
            s.count[d] = in ? (int32_t)k[ZHIP_MAX_DIMS + d] : 1;
            s.step[d] = in ? (int32_t)k[2 * ZHIP_MAX_DIMS + d] : 1;
            s.div_step[d] = fdiv_of((uint32_t)s.step[d]);
        }
    }
    for (uint64_t e = 0; e < n; ++e) chunks[e].sel = rank[sel_of[e]];
    *agg = (last_full ? ZHIP_AGG_LAST_FULL : 0u) | (out_al16 ? ZHIP_AGG_OUT_ALIGNED : 0u) |
           (unit_or_single ? ZHIP_AGG_UNIT_STEPS : 0u) | (all_full ? ZHIP_AGG_ALL_FULL : 0u);
    return ZHIP_OK;
}

}  // extern "C"
