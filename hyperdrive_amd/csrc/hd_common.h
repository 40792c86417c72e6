// hd_common.h -- shared definitions for the hyperdrive_amd device math.
//
// Every header in this directory compiles both as gfx950 device code (hipcc)
// and as plain host C++ (g++), so that the exact arithmetic the kernels run can
// be unit-tested on a CPU-only machine (tests/native/).  The host build is a
// test harness only; the product library never falls back to it.
#pragma once
#include <stdint.h>

#include <type_traits>
#include <utility>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define HD __host__ __device__ __forceinline__
#define HD_MEMBER __host__ __device__ __forceinline__
#define HD_NOINLINE static __host__ __device__ __noinline__
#define HD_HOSTONLY static inline __host__
#else
#define HD static inline
#define HD_MEMBER inline
#define HD_NOINLINE static
#define HD_HOSTONLY static inline
#endif

#if defined(__HIP_DEVICE_COMPILE__)
#define HD_UNROLL _Pragma("unroll")
#define HD_NOUNROLL _Pragma("unroll 1")
#else
#define HD_UNROLL
#define HD_NOUNROLL
#endif

namespace hd {

// Compile-time loop: f(std::integral_constant<int, j>) for j = 0 .. N-1, each
// call a separate copy (arrays indexed by j stay in registers, whatever the
// unroller's size limits).
template <typename F, int... J>
HD void static_for_impl(F&& f, std::integer_sequence<int, J...>) {
    (f(std::integral_constant<int, J>{}), ...);
}
template <int N, typename F>
HD void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// Verdict enum -- mirrors include/hd_verify.h (HD_VERDICT_*).
enum Verdict : uint8_t {
    V_VALID = 0,
    V_BAD_RECID = 1,
    V_BAD_RS = 2,
    V_NO_POINT = 3,
    V_INFINITY = 4,
    V_SIGNATORY_MISMATCH = 5,
    V_NOT_ADMITTED = 6,
    V_BAD_TYPE = 7,
    V_NOT_AUTHENTIC = 8,   // hd_authenticate_batch_device only: failed the known-key check
};

// process/message.go:11-22
enum MsgType : uint8_t { T_PROPOSE = 1, T_PREVOTE = 2, T_PRECOMMIT = 3 };

HD uint32_t load_be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
HD void store_be32(uint8_t* p, uint32_t x) {
    p[0] = (uint8_t)(x >> 24);
    p[1] = (uint8_t)(x >> 16);
    p[2] = (uint8_t)(x >> 8);
    p[3] = (uint8_t)x;
}

HD uint32_t bswap32(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}

// Row i of an array of 32-byte records (value32 / from32) as 8 big-endian
// words.  On the device, when the array base is 16-byte aligned (torch and
// hipMalloc buffers are), two 16-byte loads replace 32 byte loads -- the
// base is a kernel argument, so the test is a uniform branch.
HD void load_row32_be(uint32_t w[8], const uint8_t* base, size_t i) {
    const uint8_t* p = base + 32 * i;
#if defined(__HIP_DEVICE_COMPILE__)
    if (((uintptr_t)base & 15u) == 0) {
        const uint4 a = *(const uint4*)p, b = *(const uint4*)(p + 16);
        w[0] = bswap32(a.x); w[1] = bswap32(a.y); w[2] = bswap32(a.z); w[3] = bswap32(a.w);
        w[4] = bswap32(b.x); w[5] = bswap32(b.y); w[6] = bswap32(b.z); w[7] = bswap32(b.w);
        return;
    }
#endif
    for (int k = 0; k < 8; k++) w[k] = load_be32(p + 4 * k);
}

// Row i of a 32-byte record array written from 8 big-endian words (16-byte
// stores when the base is 16-byte aligned, as load_row32_be).
HD void store_row32_be(uint8_t* base, size_t i, const uint32_t w[8]) {
    uint8_t* p = base + 32 * i;
#if defined(__HIP_DEVICE_COMPILE__)
    if (((uintptr_t)base & 15u) == 0) {
        *(uint4*)p = make_uint4(bswap32(w[0]), bswap32(w[1]), bswap32(w[2]), bswap32(w[3]));
        *(uint4*)(p + 16) = make_uint4(bswap32(w[4]), bswap32(w[5]), bswap32(w[6]), bswap32(w[7]));
        return;
    }
#endif
    for (int k = 0; k < 8; k++) store_be32(p + 4 * k, w[k]);
}

// Signature i of an array of 65-byte R || S || V records: r and s as 8
// big-endian words each, v the recovery byte.  Record i starts at byte 65 i,
// i.e. i mod 4 bytes past a 4-byte boundary; on the device (4-byte aligned
// base) 17 aligned dword loads cover it and a funnel shift per word extracts
// it, instead of 65 byte loads.  The dword span ends up to 3 bytes past the
// record, inside record i + 1, so the last record takes the byte path.
HD void load_sig65(uint32_t r_be[8], uint32_t s_be[8], uint32_t& v, const uint8_t* base, size_t i, size_t n) {
    const uint8_t* p = base + 65 * i;
#if defined(__HIP_DEVICE_COMPILE__)
    if (((uintptr_t)base & 3u) == 0 && i + 1 < n) {
        const uint32_t off = (uint32_t)(i & 3u);
        const uint32_t* q = (const uint32_t*)(p - off);
        uint32_t d[17];
#pragma unroll
        for (int k = 0; k < 17; k++) d[k] = q[k];
        const uint32_t sh = 8u * off;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t le = (uint32_t)(((((uint64_t)d[k + 1]) << 32) | d[k]) >> sh);
            if (k < 8) r_be[k] = bswap32(le);
            else s_be[k - 8] = bswap32(le);
        }
        v = (d[16] >> sh) & 0xFFu;
        return;
    }
#else
    (void)n;
#endif
    for (int k = 0; k < 8; k++) {
        r_be[k] = load_be32(p + 4 * k);
        s_be[k] = load_be32(p + 32 + 4 * k);
    }
    v = p[64];
}

}  // namespace hd
