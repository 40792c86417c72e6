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
#include "fe8_proto.h"
#include "kara_proto.h"

using namespace hd;

__device__ void seed_fe(fe& a, uint32_t s) {
    HD_UNROLL for (int i = 0; i < 9; i++) { s = s * 1664525u + 1013904223u; a.n[i] = s & HD_M29; }
    a.n[8] &= HD_M24;
}

// ---- FP64-FMA field product (round-4 prototype) --------
// 5 limbs of 52 bits held in doubles (exact integers, value < 2^260).  A limb
// product a b < 2^104 is split exactly with two FMAs under round-toward-zero
// (OCML's fma_rtz for the high part): ph = fma(a, b, 2^104) = 2^104 + H 2^52 with
// H = floor(a b / 2^52), pl = fma(a, b, (2^104 + 2^52) - ph) = 2^52 + L with
// L = a b mod 2^52 -- both in one binade, so their bit patterns are the
// offset integers H and L.  Columns accumulate the raw bit patterns as 64-bit
// integers (the offsets are subtracted once, folded into the initial column
// values); then carries at 52 bits, and the fold of the high half by
// 2^260 = 16 (2^32 + 977) mod p with the same FMA split.
struct f5 { double v[5]; };
#define F5_M52 ((1ull << 52) - 1)
__device__ __forceinline__ uint64_t dbits(double x) { return (uint64_t)__double_as_longlong(x); }
// acc[k] += a b's low part, acc[k+1] += its high part (raw bit patterns)
__device__ __forceinline__ void f5_prod(uint64_t& lo, uint64_t& hi, double a, double b) {
    const double C1 = 0x1p104, C2 = 0x1p104 + 0x1p52;
    const double ph = __ocml_fma_rtz_f64(a, b, C1);   // round toward zero: H = floor(a b / 2^52)
    const double pl = __builtin_fma(a, b, C2 - ph);
    lo += dbits(pl);
    hi += dbits(ph);
}
__device__ __forceinline__ double u2d(uint64_t x) { return (double)x; }   // x < 2^53: exact
__device__ void f5_mul(f5& r, const f5& a, const f5& b) {
    const uint64_t BH = dbits(0x1p104), BL = dbits(0x1p52);
    uint64_t col[11];
#pragma unroll
    for (int k = 0; k < 11; k++) {
        // products with i + j = k (low part) and i + j = k - 1 (high part)
        const uint64_t nl = k < 5 ? k + 1 : (k < 9 ? 9 - k : 0);
        const uint64_t nh = k == 0 ? 0 : (k - 1 < 5 ? k : (k - 1 < 9 ? 9 - (k - 1) : 0));
        col[k] = 0 - nl * BL - nh * BH;
    }
#pragma unroll
    for (int i = 0; i < 5; i++)
#pragma unroll
        for (int j = 0; j < 5; j++) f5_prod(col[i + j], col[i + j + 1], a.v[i], b.v[j]);
    // carries (columns < 2^56)
#pragma unroll
    for (int k = 0; k < 10; k++) {
        col[k + 1] += col[k] >> 52;
        col[k] &= F5_M52;
    }
    // fold: limbs 5..10 times K = 2^260 mod p = 0x1000003D10 (< 2^37)
    const double K = (double)0x1000003D10ull;
    uint64_t t[7];
    const uint64_t BK[7] = {0, 0, 0, 0, 0, 0, 0};
    (void)BK;
#pragma unroll
    for (int k = 0; k < 7; k++) t[k] = k < 5 ? col[k] : 0;
    // t[k] += low(col[5+k] K), t[k+1] += high(col[5+k] K); col[10] < 2^8 joins col[9]
    col[9] += col[10] << 52;   // < 2^61: split in two limbs of 52 below
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const uint64_t x = col[5 + k];
        const double xl = u2d(x & F5_M52), xh = u2d(x >> 52);
        uint64_t lo = 0 - BL, hi = 0 - BH;
        f5_prod(lo, hi, xl, K);
        t[k] += lo;
        t[k + 1] += hi;
        if (k == 4) {   // the part of col[9] above 52 bits: weight 2^(52 10)
            uint64_t lo2 = 0 - BL, hi2 = 0 - BH;
            f5_prod(lo2, hi2, xh, K);
            t[5] += lo2;
            t[6] += hi2;
        }
    }
#pragma unroll
    for (int k = 0; k < 6; k++) {
        t[k + 1] += t[k] >> 52;
        t[k] &= F5_M52;
    }
    // t[5], t[6] (< 2^46 at weight 2^260): once more times K, into limbs 0..2
    {
        const uint64_t x = t[5] + (t[6] << 52);   // < 2^99? no: t[6] is tiny (< 2^2); x < 2^54
        uint64_t lo = 0 - BL, hi = 0 - BH;
        f5_prod(lo, hi, u2d(x & F5_M52), K);
        uint64_t lo2 = 0 - BL, hi2 = 0 - BH;
        f5_prod(lo2, hi2, u2d(x >> 52), K);
        t[0] += lo;
        t[1] += hi + lo2;
        t[2] += hi2;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        t[k + 1] += t[k] >> 52;
        t[k] &= F5_M52;
    }
#pragma unroll
    for (int k = 0; k < 5; k++) r.v[k] = u2d(t[k]);   // t[4] < 2^53 (value < 2^260 + small)
}

__device__ void f5_from_fe(f5& r, const fe& a) {
    fe t = a;
    fe_normalize(t);
    uint32_t w[8];
    fe_to_le(w, t);
    uint64_t x[4];
    for (int k = 0; k < 4; k++) x[k] = (uint64_t)w[2 * k] | ((uint64_t)w[2 * k + 1] << 32);
    // 52-bit limbs of a 256-bit value
    for (int k = 0; k < 5; k++) {
        const int bit = 52 * k, word = bit >> 6, off = bit & 63;
        uint64_t v = x[word] >> off;
        if (off > 12 && word + 1 < 4) v |= x[word + 1] << (64 - off);
        r.v[k] = u2d(v & F5_M52);
    }
}
// f5 -> fe: t mod p as 8 LE words via fe_from_le on the low 256 bits plus the fold of bits >= 256
__device__ void fe_from_f5(fe& r, const f5& a) {
    uint64_t l[5];
    for (int k = 0; k < 5; k++) l[k] = (uint64_t)a.v[k];
    uint32_t w[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < 5; k++)
        for (int b = 0; b < 52; b++)
            if ((l[k] >> b) & 1) {
                const int bit = 52 * k + b;
                w[bit >> 5] |= 1u << (bit & 31);
            }
    fe lo, hi, k32;
    fe_from_le(lo, w);
    fe_set_u32(hi, w[8]);                  // bits 256..259
    fe_set_u32(k32, 977);
    k32.n[1] = 8;                          // 2^32 = 8 2^29: k32 = 2^32 + 977
    fe_mul(hi, hi, k32);
    fe_add(r, lo, hi);
    fe_normalize(r);
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
        if (OP == 10) fe_mul_kara(a, a, b);
    }
    if (OP == 8 || OP == 9) {   // 8 x 32-bit words with carry-out mads (hd_fe8.h)
        fe8 x, y;
        fe_normalize(a);
        fe_normalize(b);
        fe_to_le(x.w, a);
        fe_to_le(y.w, b);
        for (uint32_t it = 0; it < iters; it++) {
            if (OP == 8) fe8_mul(x, x, y);
            else fe8_sqr(x, x);
        }
        fe_from_fe8(a, x);
    }
    if (OP == 7) {   // the FP64 product chain (its own loop: f5 state)
        f5 x, y;
        f5_from_fe(x, a);
        f5_from_fe(y, b);
        for (uint32_t it = 0; it < iters; it++) f5_mul(x, x, y);
        fe_from_f5(a, x);
    }
    uint32_t r = 0;
    HD_UNROLL for (int i = 0; i < 9; i++) r ^= a.n[i] ^ p.x.n[i] ^ p.z.n[i];
    out[t] = r;
}

static const char* NAMES[] = {"fe_mul", "fe_sqr", "gej_dbl", "gej_add_ge", "gej_add", "fe_normalize", "fe_inv_divsteps",
                              "f5_mul (FP64 FMA)", "fe8_mul", "fe8_sqr", "fe_mul_kara"};
#define NOPS 11

// f5_mul against fe_mul: a chain of `iters` products from the same seeds,
// canonical results compared per lane (count of mismatching lanes)
__global__ __launch_bounds__(256) void k_f5_check(uint32_t iters, uint32_t* bad) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    fe a, b;
    seed_fe(a, t * 7 + 1);
    seed_fe(b, t * 13 + 5);
    if (t == 0) {   // extremes: p - 1 squared
        for (int i = 0; i < 9; i++) a.n[i] = b.n[i] = fe_p_limb(i);
        a.n[0] -= 1;
        b.n[0] -= 1;
    }
    f5 x, y;
    f5_from_fe(x, a);
    f5_from_fe(y, b);
    for (uint32_t it = 0; it < iters; it++) {
        fe_mul(a, a, b);
        f5_mul(x, x, y);
    }
    fe c;
    fe_from_f5(c, x);
    fe_normalize(a);
    uint32_t d = 0;
    for (int i = 0; i < 9; i++) d |= a.n[i] ^ c.n[i];
    if (d) atomicAdd(bad, 1u);
}

// fe8_mul / fe8_sqr against fe_mul / fe_sqr: chains of `iters` steps from the
// same seeds (extremes on lane 0: p - 1), canonical results compared per lane
__global__ __launch_bounds__(256) void k_fe8_check(uint32_t iters, uint32_t* bad) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    fe a, b;
    seed_fe(a, t * 7 + 1);
    seed_fe(b, t * 13 + 5);
    if (t == 0) {
        for (int i = 0; i < 9; i++) a.n[i] = b.n[i] = fe_p_limb(i);
        a.n[0] -= 1;
        b.n[0] -= 1;
    }
    fe_normalize(a);
    fe_normalize(b);
    fe8 x, y, z;
    fe_to_le(x.w, a);
    fe_to_le(y.w, b);
    z = x;
    fe c = a;
    for (uint32_t it = 0; it < iters; it++) {
        fe_mul(a, a, b);
        fe8_mul(x, x, y);
        fe_sqr(c, c);
        fe8_sqr(z, z);
        fe8 d;   // sums and differences along the way: (x - y) + y == x
        fe8_sub(d, x, y);
        fe8_add(d, d, y);
        fe8_sub(d, d, x);
        fe8_canon(d);
        uint32_t nz = 0;
        for (int i = 0; i < 8; i++) nz |= d.w[i];
        if (nz) atomicAdd(bad + 1, 1u);
    }
    fe u, v;
    fe_from_fe8(u, x);
    fe_from_fe8(v, z);
    fe_normalize(a);
    fe_normalize(c);
    uint32_t d = 0;
    for (int i = 0; i < 9; i++) d |= (a.n[i] ^ u.n[i]) | (c.n[i] ^ v.n[i]);
    if (d) atomicAdd(bad, 1u);
}

// fe_mul_kara against fe_mul: chains of `iters` products from the same seeds
// (extremes on lane 0: p - 1), canonical results compared per lane
__global__ __launch_bounds__(256) void k_kara_check(uint32_t iters, uint32_t* bad) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    fe a, b;
    seed_fe(a, t * 7 + 1);
    seed_fe(b, t * 13 + 5);
    if (t == 0) {
        for (int i = 0; i < 9; i++) a.n[i] = b.n[i] = fe_p_limb(i);
        a.n[0] -= 1;
        b.n[0] -= 1;
    }
    fe c = a;
    for (uint32_t it = 0; it < iters; it++) {
        fe_mul(a, a, b);
        fe_mul_kara(c, c, b);
    }
    fe_normalize(a);
    fe_normalize(c);
    uint32_t d = 0;
    for (int i = 0; i < 9; i++) d |= a.n[i] ^ c.n[i];
    if (d) atomicAdd(bad, 1u);
}

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
    run<OP>(blocks, OP == 6 ? 20 : 2000, d, ncu);   // (OP 7: the same 2000-product chain)
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
    uint32_t* bad;
    (void)hipMalloc(&bad, 8);
    (void)hipMemset(bad, 0, 4);
    k_f5_check<<<ncu * 4, 256>>>(64, bad);
    uint32_t hb = 0;
    (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("f5_mul vs fe_mul: %u of %d lanes differ after 64 chained products\n", hb, ncu * 4 * 256);
    (void)hipMemset(bad, 0, 8);
    k_fe8_check<<<ncu * 4, 256>>>(64, bad);
    uint32_t hb8[2] = {0, 0};
    (void)hipMemcpy(hb8, bad, 8, hipMemcpyDeviceToHost);
    printf("fe8 vs fe: %u of %d lanes differ after 64 chained products and squares; add/sub identity failures %u\n",
           hb8[0], ncu * 4 * 256, hb8[1]);
    (void)hipMemset(bad, 0, 4);
    k_kara_check<<<ncu * 4, 256>>>(64, bad);
    (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("fe_mul_kara vs fe_mul: %u of %d lanes differ after 64 chained products\n", hb, ncu * 4 * 256);
    run_all<0>(ncu * wps, d, ncu);
    return 0;
}
