// GF(2) arithmetic for CRC-32C (reflected polynomial 0x82F63B78), shared by
// host plan building and device kernels.
//
// Representation (the zlib crc32_combine convention): a 32-bit word is a
// polynomial of degree < 32 with bit 31 = x^0 ... bit 0 = x^31.  The raw CRC
// register after a message is such a polynomial; advancing the register over k
// zero bytes ("A_k") is multiplication by x^(8k) mod P.  A 4-byte
// little-endian word w xor-ed into the register at byte position p contributes
// A_(q-p)(w) to the register value observed at position q >= p + 4; the whole
// register is the XOR of all such contributions (linearity), which is what lets
// every lane of the GPU own its own bytes and combine at the end.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define ZHIP_HD __host__ __device__ __forceinline__
#else
#define ZHIP_HD inline
#endif

namespace zhip {

constexpr uint32_t kPoly = 0x82F63B78u;
constexpr uint32_t kOne = 0x80000000u;  // the polynomial "1"

// a(x) * b(x) mod P, branch-free (32 steps of shift/xor).
// Rolled by 4 on purpose: fully unrolled, the compiler materialises all 32
// shifted copies of a uniform operand in SGPRs and 32 bit-masks in VGPRs at
// once (80+ spilled SGPRs, +60 VGPRs); it runs a few times per 32 KiB unit.
ZHIP_HD uint32_t gf_mul(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll 4
    for (int i = 31; i >= 0; --i) {
        p ^= b & (0u - ((a >> i) & 1u));
        b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
    }
    return p;
}

// Division by an invariant d (1 <= d < 2^31) for 0 <= n < 2^31.
ZHIP_HD uint32_t fdiv_apply(uint32_t n, uint32_t m, uint32_t s) {
    return (uint32_t)(((uint64_t)n * (uint64_t)m) >> s);
}

}  // namespace zhip
