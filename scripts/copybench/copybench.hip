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
