// fieldbench.hip -- per-operation cost of the device field / group code.
// Each kernel runs a dependent chain of one operation in a loop; the loop
// body's ISA gives the static instruction mix (scripts/isa_cost.py) and the
// run on the box gives measured cycles per operation per wave.
//
// Build: hipcc --offload-arch=gfx950 -O3 -I include -o scripts/fieldbench scripts/fieldbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include "../hyperdrive_amd/csrc/hd_group.h"

using namespace hd;

__device__ void seed_fe(fe& a, uint32_t s) {
    HD_UNROLL for (int i = 0; i < 9; i++) { s = s * 1664525u + 1013904223u; a.n[i] = s & HD_M29; }
    a.n[8] &= HD_M24;
}

template <int OP>
__global__ __launch_bounds__(256, 3) void k_bench(uint32_t iters, uint32_t* out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    fe a, b;
    seed_fe(a, t * 7 + 1);
    seed_fe(b, t * 13 + 5);
    gej p;
    p.x = a; p.y = b; fe_set_u32(p.z, 3);
    ge q;
    q.x = b; q.y = a;
    gej pj;
    pj.x = b; pj.y = a; pj.z = b;
    fe_mul(pj.z, pj.z, a);
    for (uint32_t it = 0; it < iters; it++) {
        if (OP == 0) fe_mul(a, a, b);
        if (OP == 1) fe_sqr(a, a);
        if (OP == 2) gej_dbl(p, p);
        if (OP == 3) gej_add_ge(p, p, q);
        if (OP == 4) gej_add(p, p, pj);
        if (OP == 5) fe_normalize(a);
        if (OP == 6) { fe x = a; fe_inv_divsteps(a, x); }
    }
    uint32_t r = 0;
    HD_UNROLL for (int i = 0; i < 9; i++) r ^= a.n[i] ^ p.x.n[i] ^ p.z.n[i];
    out[t] = r;
}

static const char* NAMES[] = {"fe_mul", "fe_sqr", "gej_dbl", "gej_add_ge", "gej_add", "fe_normalize", "fe_inv_divsteps"};
#define NOPS 7

template <int OP>
static void run(int blocks, uint32_t iters, uint32_t* d, int ncu) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    k_bench<OP><<<blocks, 256>>>(2, d);
    (void)hipEventRecord(e0, 0);
    k_bench<OP><<<blocks, 256>>>(iters, d);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // waves per SIMD = blocks * 4 / (ncu * 4); cycles at a nominal 2.1 GHz
    double waves_per_simd = (double)blocks / ncu;
    double cyc = ms * 1e-3 * 2.1e9 / (waves_per_simd * iters);
    printf("%-16s %8.3f ms  %8.0f SIMD-cycles/op/wave (at 2.1 GHz)\n", NAMES[OP], ms, cyc);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

template <int OP>
static void run_all(int blocks, uint32_t* d, int ncu) {
    run<OP>(blocks, OP == 6 ? 20 : 2000, d, ncu);
    if constexpr (OP + 1 < NOPS) run_all<OP + 1>(blocks, d, ncu);
}

int main(int argc, char** argv) {
    int wps = argc > 1 ? atoi(argv[1]) : 3;
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    int ncu = prop.multiProcessorCount;
    uint32_t* d;
    (void)hipMalloc(&d, 4u * 256 * ncu * 8);
    printf("%d CUs, %d waves/SIMD\n", ncu, wps);
    run_all<0>(ncu * wps, d, ncu);
    return 0;
}
