// Measurement-only: plain HBM streaming kernels at the headline's size, to
// calibrate what a 64 MiB -> 64 MiB pass can reach on one MI355X (the
// practical ceiling for k_decode).  Not part of the product library.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int K, bool STORE, bool NTL, bool NTS = NTL>
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                              uint64_t n16, uint32_t span16) {
    const uint64_t b0 = (uint64_t)blockIdx.x * span16;
    uint64_t b1 = b0 + span16;
    if (b1 > n16) b1 = n16;
    uint32_t x = 0;
    for (uint64_t b = b0 + threadIdx.x; b < b1; b += 256ull * K) {
        uint4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t i = b + 256ull * k;
            if (i < b1) {
                if constexpr (NTL) {
                    const v4u w = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src) + i);
                    v[k] = make_uint4(w.x, w.y, w.z, w.w);
                } else v[k] = src[i];
            } else v[k] = make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t i = b + 256ull * k;
            if constexpr (STORE) {
                if (i < b1) {
                    if constexpr (NTS) {
                        v4u w = {v[k].x, v[k].y, v[k].z, v[k].w};
                        __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(dst) + i);
                    } else dst[i] = v[k];
                }
            } else x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        }
    }
    if constexpr (!STORE) if (x == 0x12345678u) dst[0] = make_uint4(x, 0, 0, 0);
}

typedef void (*Fn)(const uint4*, uint4*, uint64_t, uint32_t);

extern "C" int cb_copy(const void* src, void* dst, uint64_t nbytes, uint32_t span, int K, int store, int nt,
                       void* stream) {
    const uint64_t n16 = nbytes / 16;
    const uint32_t span16 = span / 16;
    const uint32_t grid = (uint32_t)((n16 + span16 - 1) / span16);
    Fn fn = nullptr;
// nt: 0 = default policy, 1 = nontemporal loads and stores, 2 = nontemporal
// loads only, 3 = nontemporal stores only.
#define SEL(KK)                                                                                   \
    if (K == KK)                                                                                  \
        fn = store ? (nt == 1   ? (Fn)k_copy<KK, true, true, true>                                \
                      : nt == 2 ? (Fn)k_copy<KK, true, true, false>                               \
                      : nt == 3 ? (Fn)k_copy<KK, true, false, true>                               \
                                : (Fn)k_copy<KK, true, false, false>)                             \
                   : (nt ? (Fn)k_copy<KK, false, true> : (Fn)k_copy<KK, false, false>);
    SEL(1) SEL(2) SEL(4) SEL(8) SEL(16)
    if (!fn) return -1;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint4*)src, (uint4*)dst, n16,
                       span16);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Span copy with a per-workgroup rotation of the 4 KiB step order: workgroup
// g visits steps (k + g) % K, so workgroups running in lockstep are at
// different offsets of their spans (the decode kernels' unit = 8 such steps).
template <int K, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_copy_rot(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                  uint64_t n16) {
    const uint64_t b0 = (uint64_t)blockIdx.x * 256ull * K;
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t i = b0 + 256ull * ((k + blockIdx.x) % K) + threadIdx.x;
        if constexpr (NTL) {
            const v4u w = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src) + i);
            v[k] = make_uint4(w.x, w.y, w.z, w.w);
        } else v[k] = src[i];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t i = b0 + 256ull * ((k + blockIdx.x) % K) + threadIdx.x;
        if constexpr (NTS) {
            v4u w = {v[k].x, v[k].y, v[k].z, v[k].w};
            __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(dst) + i);
        } else dst[i] = v[k];
    }
}

extern "C" int cb_copy_rot(const void* src, void* dst, uint64_t nbytes, int K, int nt, void* stream) {
    typedef void (*RFn)(const uint4*, uint4*, uint64_t);
    RFn fn = nullptr;
#define RSEL(KK)                                                                                  \
    if (K == KK) fn = nt == 1 ? (RFn)k_copy_rot<KK, true, true> : nt == 3 ? (RFn)k_copy_rot<KK, false, true> \
                                                                : (RFn)k_copy_rot<KK, false, false>;
    RSEL(8) RSEL(16)
    if (!fn) return -1;
    const uint64_t per = 4096ull * K;
    if (nbytes % per) return -3;
    hipLaunchKernelGGL(fn, dim3((uint32_t)(nbytes / per)), dim3(256), 0, (hipStream_t)stream, (const uint4*)src,
                       (uint4*)dst, nbytes / 16);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Interleaved spans: groups of S consecutive workgroups share S*K 4 KiB steps;
// workgroup j of a group takes steps j, j + S, j + 2S, ... (K of them), so a
// workgroup's footprint is spread over S*K*4 KiB while the group, like
// S*K one-step workgroups, covers it densely.
template <int K, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_copy_il(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                 uint32_t S) {
    const uint32_t grp = blockIdx.x / S, j = blockIdx.x - grp * S;
    const uint64_t b0 = (uint64_t)grp * S * K * 256ull;
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t i = b0 + 256ull * (j + S * (uint32_t)k) + threadIdx.x;
        if constexpr (NTL) {
            const v4u w = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src) + i);
            v[k] = make_uint4(w.x, w.y, w.z, w.w);
        } else v[k] = src[i];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t i = b0 + 256ull * (j + S * (uint32_t)k) + threadIdx.x;
        if constexpr (NTS) {
            v4u w = {v[k].x, v[k].y, v[k].z, v[k].w};
            __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(dst) + i);
        } else dst[i] = v[k];
    }
}

extern "C" int cb_copy_il(const void* src, void* dst, uint64_t nbytes, int K, uint32_t S, int nt, void* stream) {
    typedef void (*IFn)(const uint4*, uint4*, uint32_t);
    IFn fn = nullptr;
#define ISEL(KK)                                                                                  \
    if (K == KK) fn = nt == 1 ? (IFn)k_copy_il<KK, true, true> : nt == 3 ? (IFn)k_copy_il<KK, false, true> \
                                                               : (IFn)k_copy_il<KK, false, false>;
    ISEL(8) ISEL(16)
    if (!fn || S == 0) return -1;
    const uint64_t per = 4096ull * K * S;
    if (nbytes % per) return -3;
    hipLaunchKernelGGL(fn, dim3((uint32_t)(nbytes / (4096ull * K))), dim3(256), 0, (hipStream_t)stream,
                       (const uint4*)src, (uint4*)dst, S);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Persistent grid-stride copy: `grid` workgroups, each walking 16-byte blocks
// b = (g * 256 + t) + k * 256 * grid, K blocks in flight per thread.
template <int K, bool NT>
__global__ __launch_bounds__(256) void k_copy_persist(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                      uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256ull;
    for (uint64_t b = (uint64_t)blockIdx.x * 256ull + threadIdx.x; b < n16; b += stride * K) {
        uint4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t i = b + stride * k;
            if (i < n16) {
                if constexpr (NT) {
                    const v4u w = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src) + i);
                    v[k] = make_uint4(w.x, w.y, w.z, w.w);
                } else v[k] = src[i];
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t i = b + stride * k;
            if (i < n16) {
                if constexpr (NT) {
                    v4u w = {v[k].x, v[k].y, v[k].z, v[k].w};
                    __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(dst) + i);
                } else dst[i] = v[k];
            }
        }
    }
}

extern "C" int cb_copy_persist(const void* src, void* dst, uint64_t nbytes, uint32_t grid, int K, int nt,
                               void* stream) {
    typedef void (*PFn)(const uint4*, uint4*, uint64_t);
    PFn fn = nullptr;
#define PSEL(KK) if (K == KK) fn = nt ? (PFn)k_copy_persist<KK, true> : (PFn)k_copy_persist<KK, false>;
    PSEL(2) PSEL(4) PSEL(8)
    if (!fn) return -1;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint4*)src, (uint4*)dst,
                       nbytes / 16);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// The headline's access pattern without any codec work: 64 chunks of 64^3 f32
// (1 MiB each, at `cstride` bytes apart in src -- 1048580 for the shard's
// inner-chunk packing, 4-byte aligned) scattered as 256-byte rows into a
// 256^3 f32 out (row stride 1 KiB).  Each workgroup copies `units` consecutive
// 32 KiB units, every thread 8 x 16 bytes per unit (unaligned nt loads).
typedef unsigned int v4u_a1 __attribute__((ext_vector_type(4), aligned(1)));
template <int UNITS, bool NTL = true, int LDS_WORDS = 0>
__global__ __launch_bounds__(256) void k_scatter(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                 uint64_t cstride) {
    const int t = threadIdx.x;
    // LDS_WORDS > 0: reserve the decode kernel's LDS footprint (residency arm)
    __shared__ uint32_t s_pad[LDS_WORDS > 0 ? LDS_WORDS : 1];
    if constexpr (LDS_WORDS > 0) {
        s_pad[t] = t;
        if (t == 0 && cstride == 0) dst[0] = (uint8_t)s_pad[255];
    }
    uint4 v[UNITS][8];
#pragma unroll
    for (int u = 0; u < UNITS; ++u) {
        const uint32_t q = blockIdx.x * UNITS + u;
        const uint32_t c = q >> 5, s = q & 31;
        const uint8_t* cp = src + (uint64_t)c * cstride + (uint64_t)s * 32768;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const v4u_a1 w = NTL ? __builtin_nontemporal_load(reinterpret_cast<const v4u_a1*>(cp + 4096 * k + 16 * t))
                                 : *reinterpret_cast<const v4u_a1*>(cp + 4096 * k + 16 * t);
            v[u][k] = make_uint4(w.x, w.y, w.z, w.w);
        }
    }
#pragma unroll
    for (int u = 0; u < UNITS; ++u) {
        const uint32_t q = blockIdx.x * UNITS + u;
        const uint32_t c = q >> 5, s = q & 31;
        const uint32_t cz = c >> 4, cy = (c >> 2) & 3, cx = c & 3;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t b = s * 32768 + 4096 * k + 16 * t;  // byte in the chunk
            const uint32_t z = b >> 14, y = (b >> 8) & 63, xb = b & 255;
            const uint64_t o = ((uint64_t)(cz * 64 + z) * 256 + cy * 64 + y) * 1024 + cx * 256 + xb;
            v4u w = {v[u][k].x, v[u][k].y, v[u][k].z, v[u][k].w};
            __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(dst + o));
        }
    }
}

extern "C" int cb_scatter(const void* src, void* dst, uint64_t cstride, int units, void* stream) {
    const uint32_t n_units = 64 * 32;
    if (units == 11)  // one unit per workgroup, default-policy loads
        hipLaunchKernelGGL((k_scatter<1, false>), dim3(n_units), dim3(256), 0, (hipStream_t)stream,
                           (const uint8_t*)src, (uint8_t*)dst, cstride);
    else if (units == 22)  // two units, default-policy loads, 36 KiB of LDS reserved (4 workgroups per CU)
        hipLaunchKernelGGL((k_scatter<2, false, 9216>), dim3(n_units / 2), dim3(256), 0, (hipStream_t)stream,
                           (const uint8_t*)src, (uint8_t*)dst, cstride);
    else if (units == 12)  // two units per workgroup, default-policy loads
        hipLaunchKernelGGL((k_scatter<2, false>), dim3(n_units / 2), dim3(256), 0, (hipStream_t)stream,
                           (const uint8_t*)src, (uint8_t*)dst, cstride);
    else if (units == 1)
        hipLaunchKernelGGL(k_scatter<1>, dim3(n_units), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)src,
                           (uint8_t*)dst, cstride);
    else if (units == 2)
        hipLaunchKernelGGL(k_scatter<2>, dim3(n_units / 2), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)src,
                           (uint8_t*)dst, cstride);
    else
        return -1;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Wave-contiguous spans: a workgroup covers K * 4 KiB; wave w takes the
// contiguous quarter [w * K KiB, (w + 1) * K KiB), lane l's k-th 16-byte block
// at 1 KiB * k + 16 l of it (all K loads first, then the stores).  The decode's
// unit with a per-lane stride of 1 KiB instead of 4 KiB: each wave's loads
// are one contiguous K KiB burst.
template <int K, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_copy_wave(const uint4* __restrict__ src, uint4* __restrict__ dst) {
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;
    const uint64_t b0 = (uint64_t)blockIdx.x * 256ull * K + (uint64_t)w * 64ull * K + l;
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t i = b0 + 64ull * k;
        if constexpr (NTL) {
            const v4u x = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src) + i);
            v[k] = make_uint4(x.x, x.y, x.z, x.w);
        } else v[k] = src[i];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t i = b0 + 64ull * k;
        if constexpr (NTS) {
            v4u x = {v[k].x, v[k].y, v[k].z, v[k].w};
            __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(dst) + i);
        } else dst[i] = v[k];
    }
}

extern "C" int cb_copy_wave(const void* src, void* dst, uint64_t nbytes, int K, int nt, void* stream) {
    typedef void (*WFn)(const uint4*, uint4*);
    WFn fn = nullptr;
#define WSEL(KK)                                                                                  \
    if (K == KK) fn = nt == 1 ? (WFn)k_copy_wave<KK, true, true> : nt == 3 ? (WFn)k_copy_wave<KK, false, true> \
                                                                 : (WFn)k_copy_wave<KK, false, false>;
    WSEL(2) WSEL(4) WSEL(8) WSEL(16)
    if (!fn) return -1;
    const uint64_t per = 4096ull * K;
    if (nbytes % per) return -3;
    hipLaunchKernelGGL(fn, dim3((uint32_t)(nbytes / per)), dim3(256), 0, (hipStream_t)stream, (const uint4*)src,
                       (uint4*)dst);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// A sharded decode's access pattern without codec work: cubic chunks of
// ce^3 f32 (`cstride` bytes apart in src: the shard packing with its 4-byte
// CRC), cps^3 per shard in (z, y, x) order, sps^3 shards, scattered as
// 4 ce-byte rows into the (ce cps sps)^3 f32 out.  C4: ce 32, cps 4, sps 8;
// the headline: ce 64, cps 2, sps 2.  A "step" is 4 KiB of a chunk, one
// 16-byte block per thread.
//   MODE 0: workgroup w takes steps [wK, wK + K) (chunk-contiguous spans)
//   MODE 1: interleaved: workgroup j of a group of S takes steps j + S k
//   MODE 2: x-quads: 4 consecutive chunks, workgroup takes K/4 consecutive
//           steps of each of the four
//   MODE 3: x-quads by wave: wave v on chunk 4 (w / (chunk / 8 KiB)) + v,
//           8 KiB contiguous per wave at a 1 KiB lane stride
struct ScatterGeo {
    uint64_t cstride;
    uint32_t ce, cps, sps, spc;  // spc: 4 KiB steps per chunk
};
template <int MODE, int K, int S>
__global__ __launch_bounds__(256) void k_scatter_g(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   const ScatterGeo g) {
    const uint32_t t = threadIdx.x;
    const uint32_t w = blockIdx.x;
    uint4 v[K];
    uint32_t cc[K], bb[K];  // chunk, byte in the chunk
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint32_t c, b;
        if constexpr (MODE == 3) {
            const uint32_t per = g.spc / 2;  // 8 KiB spans per chunk
            c = (w / per) * 4 + (t >> 6);
            b = (w % per) * 8192 + 1024 * k + 16 * (t & 63);
        } else {
            uint32_t q;  // global step: chunk * spc + step
            if constexpr (MODE == 0) q = w * K + k;
            else if constexpr (MODE == 1) q = (w / S) * (S * K) + (w % S) + S * k;
            else {
                const uint32_t per = g.spc / (K / 4);
                q = ((w / per) * 4 + (k & 3)) * g.spc + (w % per) * (K / 4) + (k >> 2);
            }
            c = q / g.spc;
            b = (q % g.spc) * 4096 + 16 * t;
        }
        cc[k] = c;
        bb[k] = b;
        const v4u_a1 x = *reinterpret_cast<const v4u_a1*>(src + (uint64_t)c * g.cstride + b);
        v[k] = make_uint4(x.x, x.y, x.z, x.w);
    }
    const uint32_t row = 4 * g.ce, plane = row * g.ce, c3 = g.cps * g.cps * g.cps;
    const uint64_t N = (uint64_t)g.ce * g.cps * g.sps;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t c = cc[k], b = bb[k];
        const uint32_t s = c / c3, i = c % c3;
        const uint32_t sz = s / (g.sps * g.sps), sy = (s / g.sps) % g.sps, sx = s % g.sps;
        const uint32_t iz = i / (g.cps * g.cps), iy = (i / g.cps) % g.cps, ix = i % g.cps;
        const uint32_t z = b / plane, y = (b / row) % g.ce, xb = b % row;
        const uint64_t o = (((sz * g.cps + iz) * g.ce + z) * N + (sy * g.cps + iy) * g.ce + y) * N * 4 +
                           (uint64_t)(sx * g.cps + ix) * g.ce * 4 + xb;
        v4u x = {v[k].x, v[k].y, v[k].z, v[k].w};
        __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(dst + o));
    }
}

// mode: 0 natural (K 1, 2, 4, 8, 16), 1 interleaved (S 4 / 8, K 8), 2 x-quads
// (K 4, 8, 16), 3 x-quads by wave (K 8); ce 32 = C4, 64 = the headline
extern "C" int cb_scatter_geo(const void* src, void* dst, uint64_t cstride, int ce, int mode, int K, int S,
                              void* stream) {
    ScatterGeo g;
    g.cstride = cstride;
    g.ce = ce;
    g.cps = ce == 32 ? 4 : 2;
    g.sps = ce == 32 ? 8 : 2;
    g.spc = ce * ce * ce * 4 / 4096;
    const uint32_t n_chunks = g.cps * g.cps * g.cps * g.sps * g.sps * g.sps;
    const uint32_t n_steps = n_chunks * g.spc;
    typedef void (*SFn)(const uint8_t*, uint8_t*, const ScatterGeo);
    SFn fn = nullptr;
    if (mode == 0 && K == 1) fn = k_scatter_g<0, 1, 1>;
    if (mode == 0 && K == 2) fn = k_scatter_g<0, 2, 1>;
    if (mode == 0 && K == 4) fn = k_scatter_g<0, 4, 1>;
    if (mode == 0 && K == 8) fn = k_scatter_g<0, 8, 1>;
    if (mode == 0 && K == 16) fn = k_scatter_g<0, 16, 1>;
    if (mode == 1 && K == 8 && S == 4) fn = k_scatter_g<1, 8, 4>;
    if (mode == 1 && K == 8 && S == 8) fn = k_scatter_g<1, 8, 8>;
    if (mode == 2 && K == 4) fn = k_scatter_g<2, 4, 1>;
    if (mode == 2 && K == 8) fn = k_scatter_g<2, 8, 1>;
    if (mode == 2 && K == 16) fn = k_scatter_g<2, 16, 1>;
    if (mode == 3 && K == 8) fn = k_scatter_g<3, 8, 1>;
    if (!fn) return -1;
    const uint32_t grid = mode == 3 ? n_chunks / 4 * (g.spc / 2) : n_steps / K;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)src, (uint8_t*)dst, g);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Wide workgroups: `threads` (256 / 512 / 1024) lanes per 32 KiB span, K =
// 8 * 256 / threads blocks per lane (the small-share geometry: one span per
// workgroup, lane t's blocks at 16 t + k * 16 * threads).
template <int K>
__global__ __launch_bounds__(1024) void k_copy_wide(const uint4* __restrict__ src, uint4* __restrict__ dst) {
    const uint32_t nt = blockDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * 2048ull + threadIdx.x;
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const v4u w = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src) + b0 + (uint64_t)nt * k);
        v[k] = make_uint4(w.x, w.y, w.z, w.w);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        v4u w = {v[k].x, v[k].y, v[k].z, v[k].w};
        __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(dst) + b0 + (uint64_t)nt * k);
    }
}

__global__ void k_empty(int* x) {
    if (x && threadIdx.x == 1024) x[0] = 1;
}

extern "C" int cb_copy_wide(const void* src, void* dst, uint64_t nbytes, int threads, void* stream) {
    typedef void (*WFn)(const uint4*, uint4*);
    WFn fn = threads == 256 ? (WFn)k_copy_wide<8> : threads == 512 ? (WFn)k_copy_wide<4>
           : threads == 1024 ? (WFn)k_copy_wide<2> : nullptr;
    if (!fn || nbytes % 32768) return -1;
    hipLaunchKernelGGL(fn, dim3((uint32_t)(nbytes / 32768)), dim3(threads), 0, (hipStream_t)stream,
                       (const uint4*)src, (uint4*)dst);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int cb_empty(uint32_t grid, int threads, void* stream) {
    hipLaunchKernelGGL(k_empty, dim3(grid), dim3(threads), 0, (hipStream_t)stream, (int*)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
