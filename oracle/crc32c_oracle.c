/*
 * ORACLE — test infrastructure only. Nothing in the product path may link,
 * load or call this file; only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, as the checker / CPU baseline.
 *
 * CRC-32C (Castagnoli) restated from its published definition, the algorithm
 * behind the reference's only checksum call sites:
 *   src/zarr/codecs/crc32c_.py:44   google_crc32c.value(data[:-4])   (decode)
 *   src/zarr/codecs/crc32c_.py:66   google_crc32c.value(data)        (encode)
 * The dependency is google-crc32c==1.8.0 (uv.lock:1002-1005), NOT vendored
 * under /root/reference: reflected polynomial 0x82F63B78, init 0xFFFFFFFF,
 * final xor 0xFFFFFFFF.  google_crc32c uses the SSE4.2 `crc32` instruction
 * (same polynomial) when available, a table method otherwise.
 *
 * Three independent implementations are provided so they can pin each other
 * and the published known-answer vectors (tests/test_oracle.py):
 *   - bitwise  : one bit per step, straight from the polynomial definition;
 *   - slice8   : slicing-by-8 tables;
 *   - hw       : the x86 SSE4.2 crc32 instruction (what google_crc32c uses),
 *                compiled per-function with the target attribute and selected
 *                only when the running CPU has SSE4.2.
 * Also exported: a multi-chunk helper used by the CPU baseline (one call per
 * chunk list so ctypes releases the GIL for the whole batch).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define CRC32C_POLY_REFLECTED 0x82F63B78u

uint32_t oracle_crc32c_bitwise(const uint8_t *data, size_t n, uint32_t crc) {
    crc = ~crc;
    for (size_t i = 0; i < n; ++i) {
        crc ^= data[i];
        for (int k = 0; k < 8; ++k)
            crc = (crc >> 1) ^ (CRC32C_POLY_REFLECTED & (0u - (crc & 1u)));
    }
    return ~crc;
}

static uint32_t g_t8[8][256];
static int g_t8_ready = 0;

static void init_tables(void) {
    if (g_t8_ready) return;
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (CRC32C_POLY_REFLECTED & (0u - (c & 1u)));
        g_t8[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
        for (int s = 1; s < 8; ++s)
            g_t8[s][i] = (g_t8[s - 1][i] >> 8) ^ g_t8[0][g_t8[s - 1][i] & 0xFFu];
    g_t8_ready = 1;
}

uint32_t oracle_crc32c_slice8(const uint8_t *data, size_t n, uint32_t crc) {
    init_tables();
    crc = ~crc;
    while (n && ((uintptr_t)data & 7u)) {
        crc = (crc >> 8) ^ g_t8[0][(crc ^ *data++) & 0xFFu];
        --n;
    }
    while (n >= 8) {
        uint32_t lo, hi;
        memcpy(&lo, data, 4);
        memcpy(&hi, data + 4, 4);
        lo ^= crc;
        crc = g_t8[7][lo & 0xFF] ^ g_t8[6][(lo >> 8) & 0xFF] ^ g_t8[5][(lo >> 16) & 0xFF] ^
              g_t8[4][lo >> 24] ^ g_t8[3][hi & 0xFF] ^ g_t8[2][(hi >> 8) & 0xFF] ^
              g_t8[1][(hi >> 16) & 0xFF] ^ g_t8[0][hi >> 24];
        data += 8;
        n -= 8;
    }
    while (n--) crc = (crc >> 8) ^ g_t8[0][(crc ^ *data++) & 0xFFu];
    return ~crc;
}

#if defined(__x86_64__) || defined(__i386__)
#include <cpuid.h>
#include <nmmintrin.h>

__attribute__((target("sse4.2"))) static uint32_t crc32c_sse42(const uint8_t *data, size_t n,
                                                               uint32_t crc) {
    uint64_t c = ~crc;
    while (n && ((uintptr_t)data & 7u)) {
        c = _mm_crc32_u8((uint32_t)c, *data++);
        --n;
    }
    while (n >= 32) {
        uint64_t a, b, d, e;
        memcpy(&a, data, 8);
        memcpy(&b, data + 8, 8);
        memcpy(&d, data + 16, 8);
        memcpy(&e, data + 24, 8);
        c = _mm_crc32_u64(c, a);
        c = _mm_crc32_u64(c, b);
        c = _mm_crc32_u64(c, d);
        c = _mm_crc32_u64(c, e);
        data += 32;
        n -= 32;
    }
    while (n >= 8) {
        uint64_t a;
        memcpy(&a, data, 8);
        c = _mm_crc32_u64(c, a);
        data += 8;
        n -= 8;
    }
    while (n--) c = _mm_crc32_u8((uint32_t)c, *data++);
    return ~(uint32_t)c;
}

int oracle_has_hw_crc(void) {
    unsigned a, b, c, d;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return 0;
    return (c & bit_SSE4_2) ? 1 : 0;
}

uint32_t oracle_crc32c_hw(const uint8_t *data, size_t n, uint32_t crc) {
    if (oracle_has_hw_crc()) return crc32c_sse42(data, n, crc);
    return oracle_crc32c_slice8(data, n, crc);
}
#else
int oracle_has_hw_crc(void) { return 0; }
uint32_t oracle_crc32c_hw(const uint8_t *data, size_t n, uint32_t crc) {
    return oracle_crc32c_slice8(data, n, crc);
}
#endif

/* The fastest available implementation: what google_crc32c.value() does. */
uint32_t oracle_crc32c(const uint8_t *data, size_t n) { return oracle_crc32c_hw(data, n, 0); }

/* CRC of many (ptr, len) buffers in one call (the CPU baseline's per-chunk loop
 * without per-chunk ctypes overhead).  out[i] = crc32c(ptrs[i][0:lens[i]]). */
void oracle_crc32c_many(const uint8_t *const *ptrs, const uint64_t *lens, uint32_t *out,
                        uint64_t count) {
    for (uint64_t i = 0; i < count; ++i) out[i] = oracle_crc32c(ptrs[i], (size_t)lens[i]);
}
