// hd_probe.hip -- VALU issue-rate probes for the roofline denominators
// (INT32 add, v_mad_u64_u32, 32-bit multiplies) on the running device.
// Each lane runs 8 independent dependency chains so the measurement is the
// issue rate, not latency.
#include <hip/hip_runtime.h>

#include "../../include/hd_probe.h"

template <int OP>
__global__ __launch_bounds__(256) void k_probe(uint32_t iters, uint32_t seed, uint32_t* out) {
    uint32_t a = threadIdx.x * 2654435761u + seed, b = blockIdx.x | 1u;
    uint64_t acc[8];
    uint32_t x[8];
    uint64_t cy[8];
#pragma unroll
    for (int k = 0; k < 8; k++) { acc[k] = a + k; x[k] = a ^ (k * 0x9E3779B9u); cy[k] = 0; }
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 16; u++) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[k]) : "v"(b));
                if (OP == 1) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cy[k]) : "v"(x[k]), "v"(b));
                if (OP == 2) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[k]) : "v"(b));
                if (OP == 3) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[k]) : "v"(b));
            }
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= (uint32_t)cy[k] ^ x[k] ^ (uint32_t)acc[k] ^ (uint32_t)(acc[k] >> 32);
    if (r == 0x12345678u) out[0] = r;
}

extern "C" int hd_probe_valu(int device, int op, uint32_t iters, double* ops_per_s) {
    if (!ops_per_s || op < 0 || op > 3) return -1;
    if (hipSetDevice(device) != hipSuccess) return -3;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return -3;
    uint32_t blocks = (uint32_t)prop.multiProcessorCount * 8;
    uint32_t* d = nullptr;
    if (hipMalloc(&d, 4) != hipSuccess) return -2;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto launch = [&](uint32_t it) {
        switch (op) {
            case 0: k_probe<0><<<blocks, 256>>>(it, 7, d); break;
            case 1: k_probe<1><<<blocks, 256>>>(it, 7, d); break;
            case 2: k_probe<2><<<blocks, 256>>>(it, 7, d); break;
            default: k_probe<3><<<blocks, 256>>>(it, 7, d); break;
        }
    };
    launch(8);  // warm
    (void)hipEventRecord(e0, 0);
    launch(iters);
    (void)hipEventRecord(e1, 0);
    hipError_t err = hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(d);
    if (err != hipSuccess) return -3;
    double ops = (double)blocks * 256.0 * iters * 16.0 * 8.0;
    *ops_per_s = ops / (ms * 1e-3);
    return 0;
}
