// Probe (round 6): are device-scope atomics of one kernel
// visible to plain loads of the next kernel on the same stream, on every XCD?
//
// The round-5 mq capacity prefilter (never committed) dropped 1-4 messages
// per 1M insert; DESIGN blamed a histogram kernel that read the key ranges
// -- written by the previous kernel's atomicMin / atomicMax -- with plain
// loads.  This probe tests that theory directly, in the mq's own pattern:
//   prime: every block (grid spread over all 8 XCDs) plain-reads every word,
//          so each XCD's L2 holds the lines before the atomics;
//   A:     every thread of a large grid does atomicMin / atomicMax on 32- and
//          64-bit words (the key-range reduction of k_mq_keys);
//   B:     every block, launched right after on the same stream, plain-loads
//          every word and records what it saw;
// and the host compares every block's view with the true min / max.  R
// rounds with fresh values, no host synchronisation between A and B.
// Output: one line per round (blocks that saw a wrong word, and which XCD
// they ran on), then a summary.  Build: hipcc --offload-arch=gfx950 -O2.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                    \
        }                                                                               \
    } while (0)

constexpr int NW = 64;          // words of each kind
constexpr int GA = 8192;        // blocks of A
constexpr int GB = 2048;        // blocks of B (and of the priming reads)

__host__ __device__ inline uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

__device__ inline uint32_t xcc_id() {
    // HW_ID: XCC_ID register (gfx94x/gfx950: hwreg 20); read-only register access
    return __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)) & 0xF;
}

__global__ void k_prime(const uint32_t* w32, const unsigned long long* w64, uint32_t* sink) {
    uint32_t acc = 0;
    for (int k = threadIdx.x; k < NW; k += blockDim.x) acc ^= w32[k] ^ (uint32_t)w64[k] ^ (uint32_t)(w64[NW + k] >> 7);
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;   // practically never: keeps the loads
}

__global__ void k_atomics(uint32_t* w32, unsigned long long* w64, uint64_t salt) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t v = mix(g ^ salt);
    const int k = (int)(g % NW);
    atomicMin(&w32[k], (uint32_t)v | 1u);
    atomicMin(&w64[k], (unsigned long long)(v >> 1));
    atomicMax(&w64[NW + k], (unsigned long long)(v >> 3));
}

__global__ void k_read(const uint32_t* w32, const unsigned long long* w64, uint32_t* o32, unsigned long long* o64,
                       uint32_t* xcc) {
    for (int k = threadIdx.x; k < NW; k += blockDim.x) {
        o32[(size_t)blockIdx.x * NW + k] = w32[k];
        o64[(size_t)blockIdx.x * 2 * NW + k] = w64[k];
        o64[(size_t)blockIdx.x * 2 * NW + NW + k] = w64[NW + k];
    }
    if (threadIdx.x == 0) xcc[blockIdx.x] = xcc_id();
}

int main(int argc, char** argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 20;
    uint32_t *w32, *o32, *xcc, *sink;
    unsigned long long *w64, *o64;
    CHK(hipMalloc(&w32, 4 * NW));
    CHK(hipMalloc(&w64, 8 * 2 * NW));
    CHK(hipMalloc(&o32, 4 * (size_t)GB * NW));
    CHK(hipMalloc(&o64, 8 * (size_t)GB * 2 * NW));
    CHK(hipMalloc(&xcc, 4 * GB));
    CHK(hipMalloc(&sink, 4 * GB));
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<uint32_t> h32((size_t)GB * NW), hx(GB);
    std::vector<unsigned long long> h64((size_t)GB * 2 * NW);
    long bad_total = 0;
    int xcds_seen = 0;
    for (int r = 0; r < R; r++) {
        const uint64_t salt = mix(0x5EED0000ull + r);
        // expected extremes (host)
        std::vector<uint32_t> e32(NW, 0xFFFFFFFFu);
        std::vector<unsigned long long> e64(2 * NW);
        for (int k = 0; k < NW; k++) { e64[k] = ~0ull; e64[NW + k] = 0; }
        for (uint64_t g = 0; g < (uint64_t)GA * 256; g++) {
            const uint64_t v = mix(g ^ salt);
            const int k = (int)(g % NW);
            e32[k] = std::min(e32[k], (uint32_t)v | 1u);
            e64[k] = std::min(e64[k], (unsigned long long)(v >> 1));
            e64[NW + k] = std::max(e64[NW + k], (unsigned long long)(v >> 3));
        }
        // initial values: the reduction's identities, written by a memset
        // (min words) and a copy, all in stream order
        CHK(hipMemsetAsync(w32, 0xFF, 4 * NW, s));
        CHK(hipMemsetAsync(w64, 0xFF, 8 * NW, s));
        CHK(hipMemsetAsync(w64 + NW, 0x00, 8 * NW, s));
        k_prime<<<GB, 64, 0, s>>>(w32, w64, sink);
        k_atomics<<<GA, 256, 0, s>>>(w32, w64, salt);
        k_read<<<GB, 64, 0, s>>>(w32, w64, o32, o64, xcc);
        CHK(hipGetLastError());
        CHK(hipMemcpyAsync(h32.data(), o32, 4 * h32.size(), hipMemcpyDeviceToHost, s));
        CHK(hipMemcpyAsync(h64.data(), o64, 8 * h64.size(), hipMemcpyDeviceToHost, s));
        CHK(hipMemcpyAsync(hx.data(), xcc, 4 * hx.size(), hipMemcpyDeviceToHost, s));
        CHK(hipStreamSynchronize(s));
        int bad_blocks = 0;
        uint32_t bad_xcd_mask = 0, xmask = 0;
        for (int b = 0; b < GB; b++) {
            xmask |= 1u << (hx[b] & 31);
            bool ok = true;
            for (int k = 0; k < NW; k++) {
                ok &= h32[(size_t)b * NW + k] == e32[k];
                ok &= h64[(size_t)b * 2 * NW + k] == e64[k];
                ok &= h64[(size_t)b * 2 * NW + NW + k] == e64[NW + k];
            }
            if (!ok) {
                bad_blocks++;
                bad_xcd_mask |= 1u << (hx[b] & 31);
            }
        }
        xcds_seen = __builtin_popcount(xmask);
        bad_total += bad_blocks;
        printf("round %d: reader blocks %d on %d XCDs (mask 0x%x), blocks with a stale word %d (XCD mask 0x%x)\n", r,
               GB, xcds_seen, xmask, bad_blocks, bad_xcd_mask);
    }
    printf("summary: %d rounds x %d reader blocks x %d words (32-bit min, 64-bit min, 64-bit max): %ld stale views; "
           "%d XCDs\n", R, GB, NW, bad_total, xcds_seen);
    return bad_total ? 1 : 0;
}
