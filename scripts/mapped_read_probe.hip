// Host read speed of device-written pinned host memory by allocation flags
// (the mq consume stage is hipHostMallocMapped | hipHostMallocCoherent):
// a kernel fills 4 MB through the mapped pointer, then the host copies it
// into a malloc'd buffer (and reads 160 scattered 160-byte rows), timed.
//   hipcc --offload-arch=gfx950 -O2 -o scripts/mapped_read_probe scripts/mapped_read_probe.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__global__ void fill(uint32_t* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)i * 2654435761u;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t bytes = 4u << 20, n = bytes / 4;
    struct Cfg { const char* name; unsigned flags; } cfgs[] = {
        {"mapped|coherent", hipHostMallocMapped | hipHostMallocCoherent},
        {"mapped|noncoherent", hipHostMallocMapped | hipHostMallocNonCoherent},
        {"mapped(default)", hipHostMallocMapped},
    };
    std::vector<uint8_t> dst(bytes);
    for (auto& c : cfgs) {
        void* h = nullptr;
        if (hipHostMalloc(&h, bytes, c.flags) != hipSuccess) { printf("%s: alloc failed\n", c.name); continue; }
        void* d = nullptr;
        (void)hipHostGetDevicePointer(&d, h, 0);
        double best_copy = 1e30, best_rows = 1e30;
        for (int rep = 0; rep < 5; rep++) {
            fill<<<256, 256>>>((uint32_t*)d, n);
            (void)hipDeviceSynchronize();
            double t0 = now_us();
            uint64_t acc = 0;
            for (int r = 0; r < 160; r++) {   // 160 rows of 160 B at scattered offsets
                const uint8_t* row = (const uint8_t*)h + ((size_t)r * 26141 % (bytes / 160)) * 160;
                memcpy(dst.data() + 160 * r, row, 160);
                acc += dst[160 * r];
            }
            double t1 = now_us();
            memcpy(dst.data(), h, bytes);
            double t2 = now_us();
            best_rows = std::min(best_rows, t1 - t0);
            best_copy = std::min(best_copy, t2 - t1);
            if (acc == 12345) printf(" ");
        }
        printf("{\"alloc\": \"%s\", \"rows160_us\": %.2f, \"copy4MB_us\": %.1f, \"GBs\": %.2f}\n", c.name, best_rows,
               best_copy, bytes / best_copy / 1e3);
        (void)hipHostFree(h);
    }
    return 0;
}
