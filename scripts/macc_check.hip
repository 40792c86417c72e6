// macc_check.hip -- device mul_256 / sc_mul (hd_field.h, v_mad_u64_u32 carry
// chain) against the same header's host build on random operands.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/macc_check.hip -o scripts/macc_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <random>
#include <vector>
#include "../hyperdrive_amd/csrc/hd_field.h"
using namespace hd;
__global__ void k(int n, const uint32_t* a, const uint32_t* b, uint32_t* t, uint32_t* s) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t x[8], y[8], o[16];
    for (int w = 0; w < 8; w++) { x[w] = a[8 * i + w]; y[w] = b[8 * i + w]; }
    mul_256(o, x, y);
    for (int w = 0; w < 16; w++) t[16 * i + w] = o[w];
    sc p, q, r;
    for (int w = 0; w < 8; w++) { p.v[w] = x[w]; q.v[w] = y[w]; }
    if (sc_ge_n(p.v)) sc_sub_n(p.v);
    if (sc_ge_n(q.v)) sc_sub_n(q.v);
    sc_mul(r, p, q);
    for (int w = 0; w < 8; w++) s[8 * i + w] = r.v[w];
}
int main() {
    const int n = 1 << 16;
    std::mt19937_64 g(7);
    std::vector<uint32_t> a(8 * n), b(8 * n), t(16 * n), s(8 * n);
    for (int i = 0; i < 8 * n; i++) {
        a[i] = (uint32_t)g(); b[i] = (uint32_t)g();
        if (i % 97 == 0) a[i] = 0xFFFFFFFFu;    // carry-heavy limbs
        if (i % 89 == 0) b[i] = 0xFFFFFFFFu;
    }
    for (int i = 0; i < 8; i++) a[i] = b[i] = 0xFFFFFFFFu;   // all-ones operands
    uint32_t *da, *db, *dt, *ds;
    hipMalloc(&da, 32 * n); hipMalloc(&db, 32 * n); hipMalloc(&dt, 64 * n); hipMalloc(&ds, 32 * n);
    hipMemcpy(da, a.data(), 32 * n, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), 32 * n, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(n, da, db, dt, ds);
    hipMemcpy(t.data(), dt, 64 * n, hipMemcpyDeviceToHost);
    hipMemcpy(s.data(), ds, 32 * n, hipMemcpyDeviceToHost);
    int bad_t = 0, bad_s = 0;
    for (int i = 0; i < n; i++) {
        uint32_t o[16];
        mul_256(o, &a[8 * i], &b[8 * i]);
        for (int w = 0; w < 16; w++) bad_t += o[w] != t[16 * i + w];
        sc p, q, r;
        for (int w = 0; w < 8; w++) { p.v[w] = a[8 * i + w]; q.v[w] = b[8 * i + w]; }
        if (sc_ge_n(p.v)) sc_sub_n(p.v);
        if (sc_ge_n(q.v)) sc_sub_n(q.v);
        sc_mul(r, p, q);
        for (int w = 0; w < 8; w++) bad_s += r.v[w] != s[8 * i + w];
    }
    printf("macc_check: %d products, mul_256 bad words %d, sc_mul bad words %d\n", n, bad_t, bad_s);
    return bad_t || bad_s;
}
