// valu_probe.hip -- standalone VALU issue-rate microbenchmark for gfx950.
// Measures wave-instruction throughput (cycles per wave-instruction per SIMD)
// of the integer / fp64 instructions a 256-bit field multiply can be built
// from, at a chosen occupancy, plus the effective shader clock (clock64 vs
// the constant-rate wall clock) while the probe runs.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/valu_probe scripts/valu_probe.hip
// Run:   scripts/valu_probe [waves_per_simd]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHAINS 8
#define UNROLL 16

template <int OP>
__global__ __launch_bounds__(256) void k_probe(uint32_t iters, uint32_t seed, uint32_t* out, uint64_t* clk) {
    uint32_t a = threadIdx.x * 2654435761u + seed, b = blockIdx.x | 1u;
    uint64_t acc[CHAINS];
    uint32_t x[CHAINS], y[CHAINS];
    double f[CHAINS];
    uint64_t cy[CHAINS], z64[CHAINS];
#pragma unroll
    for (int k = 0; k < CHAINS; k++) {
        acc[k] = a + k; z64[k] = a ^ k; x[k] = a ^ (k * 0x9E3779B9u); y[k] = x[k] * 3u; cy[k] = 0; f[k] = (double)x[k];
    }
    double fb = 1.0000001;
    uint64_t t0 = clock64(), w0 = wall_clock64();
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < UNROLL; u++) {
#pragma unroll
            for (int k = 0; k < CHAINS; k++) {
                if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[k]) : "v"(b));
                if (OP == 1) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cy[k]) : "v"(x[k]), "v"(b));
                if (OP == 2) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[k]) : "v"(b));
                if (OP == 3) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[k]) : "v"(b));
                if (OP == 4) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(f[k]) : "v"(fb));
                if (OP == 5) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(acc[k]));
                if (OP == 6) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x[k]) : "v"(b));
                if (OP == 7) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(x[k]) : "v"(b));
                if (OP == 8) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x[k]) : "v"(b));
                if (OP == 9) asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(x[k]) : "v"(b));
                if (OP == 10) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, %2, %1, vcc"
                                           : "+v"(x[k]), "=v"(y[k]) : "v"(b) : "vcc");
                if (OP == 11) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x[k]) : "v"(b));
                if (OP == 12) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[k]) : "v"(b));
                if (OP == 13) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x[k]) : "v"(b));
                if (OP == 14) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[k]) : "v"(b));
                if (OP == 15) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0\n\tv_add_u32 %4, %4, %3"
                                           : "+v"(acc[k]), "=s"(cy[k]), "+v"(x[k]) : "v"(y[k]), "v"(b));
                if (OP == 16) asm volatile("v_dot2_u32_u16 %0, %0, %1, %0" : "+v"(x[k]) : "v"(b));
                if (OP == 17) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[k]) : "v"(b) : "vcc");
                if (OP == 18) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(x[k]));
                if (OP == 19) asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_add_u32 %2, %2, %4\n\tv_and_b32 %3, %3, %4"
                                           : "+v"(acc[k]), "=s"(cy[k]), "+v"(x[k]), "+v"(y[k]) : "v"(b));
                if (OP == 20) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x[k]) : "v"(b) : "vcc");
                if (OP == 21) asm volatile("v_lshlrev_b64 %0, 7, %0" : "+v"(acc[k]));
                if (OP == 22) asm volatile("v_mov_b32 %0, %1" : "=v"(x[k]) : "v"(y[k]));
                if (OP == 23) asm volatile("v_bfe_u32 %0, %0, 3, 26" : "+v"(x[k]));
                if (OP == 24) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0\n\ts_nop 0"
                                           : "+v"(acc[k]), "=s"(cy[k]) : "v"(x[k]), "v"(b));
                if (OP == 25) asm volatile("s_nop 0\n\tv_add_u32 %0, %0, %1" : "+v"(x[k]) : "v"(b));
                if (OP == 26) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0\n\tv_mad_u64_u32 %0, %1, %2, %3, %0"
                                           : "+v"(acc[k]), "=s"(cy[k]) : "v"(x[k]), "v"(b));
                if (OP == 27) asm volatile("v_lshl_add_u64 %0, %0, 3, %1" : "+v"(acc[k]) : "v"(z64[k]));
                if (OP == 28) asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc"
                                           : "+v"(x[k]), "+v"(y[k]) : "v"(b) : "vcc");
                if (OP == 29) asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_lshl_add_u64 %2, %2, 3, %0"
                                           : "+v"(acc[k]), "=s"(cy[k]), "+v"(z64[k]) : "v"(x[k]), "v"(b));
            }
        }
    }
    uint64_t t1 = clock64(), w1 = wall_clock64();
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < CHAINS; k++)
        r ^= (uint32_t)cy[k] ^ (uint32_t)z64[k] ^ x[k] ^ y[k] ^ (uint32_t)acc[k] ^ (uint32_t)(acc[k] >> 32) ^ (uint32_t)f[k];
    if (r == 0x12345678u) out[0] = r;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = w1 - w0; }
}

static const char* NAMES[] = {"v_add_u32", "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_fma_f64",
                              "v_lshrrev_b64", "v_alignbit_b32", "v_mad_u32_u24", "v_mul_hi_u32_u24",
                              "v_dot4_u32_u8", "v_add_co+v_addc_co (2 instr)", "v_add3_u32", "v_and_b32",
                              "v_lshl_add_u32", "v_mul_u32_u24", "mad_u64 + add_u32 (2 instr)", "v_dot2_u32_u16",
                              "v_cndmask_b32", "v_lshrrev_b32", "mad_u64 + add + and (3 instr)", "v_add_co_u32",
                              "v_lshlrev_b64", "v_mov_b32", "v_bfe_u32", "mad + s_nop 0 (1 VALU)",
                              "s_nop 0 + v_add_u32 (1 VALU)", "mad -> dependent mad (2 instr)", "v_lshl_add_u64",
                              "add_co + addc (2 instr)", "mad + lshl_add_u64 (2 instr)"};
static const int NINSTR[] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 1, 1, 1, 1, 2, 1, 1, 1, 3, 1, 1, 1, 1, 1, 1, 2, 1, 2, 2};
#define NOPS 30

template <int OP>
static void run(int blocks, uint32_t iters, uint32_t* d, uint64_t* clk, int ncu) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_probe<OP><<<blocks, 256>>>(4, 7, d, clk);
    hipEventRecord(e0, 0);
    k_probe<OP><<<blocks, 256>>>(iters, 7, d, clk);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    uint64_t h[2];
    hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
    double ghz = (double)h[0] / ((double)h[1] / 100.0) / 1e3;  // wall_clock64 runs at 100 MHz
    double wave_instr = (double)blocks * 4.0 * iters * UNROLL * CHAINS * NINSTR[OP];
    double simd_cycles = (double)ncu * 4.0 * (ms * 1e-3) * ghz * 1e9;
    double lane_ops = wave_instr * 64.0 / (ms * 1e-3);
    printf("%-32s %7.3f ms  clk %.3f GHz  %6.2f cyc/wave-instr/SIMD  %7.2f T lane-instr/s\n", NAMES[OP], ms, ghz,
           simd_cycles / wave_instr,
           lane_ops / 1e12);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

template <int OP>
static void run_all(int blocks, uint32_t iters, uint32_t* d, uint64_t* clk, int ncu) {
    run<OP>(blocks, iters, d, clk, ncu);
    if constexpr (OP + 1 < NOPS) run_all<OP + 1>(blocks, iters, d, clk, ncu);
}

int main(int argc, char** argv) {
    int wps = argc > 1 ? atoi(argv[1]) : 8;
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    int ncu = prop.multiProcessorCount;
    int blocks = ncu * wps;  // 256 threads = 4 waves = one per SIMD
    uint32_t* d;
    uint64_t* clk;
    hipMalloc(&d, 4);
    hipMalloc(&clk, 16);
    printf("%s: %d CUs, %d waves/SIMD\n", prop.gcnArchName, ncu, wps);
    run_all<0>(blocks, 400, d, clk, ncu);
    return 0;
}
