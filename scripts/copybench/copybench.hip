// Measurement-only: plain HBM streaming kernels at the headline's size, to
// calibrate what a 64 MiB -> 64 MiB pass can reach on one MI355X (the
// practical ceiling for k_decode).  Not part of the product library.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int K, bool STORE, bool NT>
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
                if constexpr (NT) {
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
                    if constexpr (NT) {
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
#define SEL(KK)                                                                                   \
    if (K == KK) fn = store ? (nt ? (Fn)k_copy<KK, true, true> : (Fn)k_copy<KK, true, false>)     \
                            : (nt ? (Fn)k_copy<KK, false, true> : (Fn)k_copy<KK, false, false>);
    SEL(1) SEL(2) SEL(4) SEL(8) SEL(16)
    if (!fn) return -1;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint4*)src, (uint4*)dst, n16,
                       span16);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
