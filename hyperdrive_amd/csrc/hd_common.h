// hd_common.h -- shared definitions for the hyperdrive_amd device math.
//
// Every header in this directory compiles both as gfx950 device code (hipcc)
// and as plain host C++ (g++), so that the exact arithmetic the kernels run can
// be unit-tested on a CPU-only machine (tests/native/).  The host build is a
// test harness only; the product library never falls back to it.
#pragma once
#include <stdint.h>

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

}  // namespace hd
