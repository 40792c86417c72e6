// pcie_probe.hip -- host <-> device bandwidth on the GPU box, for the
// host-buffer (cgo) path of hd_verify_submit: one C2 batch is 154 MB up
// (7 columns) and 33 MB down per 1M messages.
//   a) one pinned H2D copy of the batch's bytes
//   b) the batch as 7 column copies (hd_verify_submit's upload)
//   c) H2D on one stream while D2H (33 MB) runs on another
//   d) a kernel reading the pinned host buffer (zero-copy, 16-B loads) into
//      device memory
//   e) two H2D copies on two streams at once
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/pcie_probe scripts/pcie_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

__global__ void k_pull(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n16; i += stride) dst[i] = src[i];
}

static float elapsed(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    const size_t N = 1u << 20;
    const size_t cols[7] = {N, 8 * N, 8 * N, 8 * N, 32 * N, 32 * N, 65 * N};
    size_t up = 0;
    for (size_t c : cols) up += c;
    const size_t down = 33 * N;
    void *h_up, *h_down, *d_up, *d_down, *d_up2;
    CK(hipHostMalloc(&h_up, up, hipHostMallocDefault));
    CK(hipHostMalloc(&h_down, down, hipHostMallocDefault));
    CK(hipMalloc(&d_up, up));
    CK(hipMalloc(&d_up2, up));
    CK(hipMalloc(&d_down, down));
    memset(h_up, 1, up);
    memset(h_down, 2, down);
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    void* h_up_dev = nullptr;
    CK(hipHostGetDevicePointer(&h_up_dev, h_up, 0));
    for (int rep = 0; rep < 3; rep++) {
        // a) one copy
        CK(hipEventRecord(e0, s0));
        CK(hipMemcpyAsync(d_up, h_up, up, hipMemcpyHostToDevice, s0));
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        const float a = elapsed(e0, e1);
        // b) 7 columns
        CK(hipEventRecord(e0, s0));
        size_t off = 0;
        for (size_t c : cols) {
            CK(hipMemcpyAsync((char*)d_up + off, (char*)h_up + off, c, hipMemcpyHostToDevice, s0));
            off += c;
        }
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        const float b = elapsed(e0, e1);
        // c) H2D with a concurrent D2H
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, s0));
        CK(hipStreamWaitEvent(s1, e0, 0));
        CK(hipMemcpyAsync(d_up, h_up, up, hipMemcpyHostToDevice, s0));
        CK(hipMemcpyAsync(h_down, d_down, down, hipMemcpyDeviceToHost, s1));
        CK(hipEventRecord(e2, s1));
        CK(hipStreamWaitEvent(s0, e2, 0));
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        const float c = elapsed(e0, e1);
        // d) zero-copy pull by a kernel
        CK(hipEventRecord(e0, s0));
        k_pull<<<2048, 256, 0, s0>>>((const uint4*)h_up_dev, (uint4*)d_up, up / 16);
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        const float d = elapsed(e0, e1);
        // e) two H2D copies on two streams
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, s0));
        CK(hipStreamWaitEvent(s1, e0, 0));
        CK(hipMemcpyAsync(d_up, h_up, up / 2, hipMemcpyHostToDevice, s0));
        CK(hipMemcpyAsync((char*)d_up2 + up / 2, (char*)h_up + up / 2, up - up / 2, hipMemcpyHostToDevice, s1));
        CK(hipEventRecord(e2, s1));
        CK(hipStreamWaitEvent(s0, e2, 0));
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        const float e = elapsed(e0, e1);
        printf("{\"rep\": %d, \"up_MB\": %.1f, \"a_one_copy_GBs\": %.1f, \"b_7_columns_GBs\": %.1f, "
               "\"c_up_with_down_ms\": %.3f, \"c_GBs_both\": %.1f, \"d_kernel_pull_GBs\": %.1f, "
               "\"e_two_streams_GBs\": %.1f}\n",
               rep, up / 1e6, up / (a * 1e-3) / 1e9, up / (b * 1e-3) / 1e9, c, (up + down) / (c * 1e-3) / 1e9,
               up / (d * 1e-3) / 1e9, up / (e * 1e-3) / 1e9);
    }
    return 0;
}
