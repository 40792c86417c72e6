// fecheck.hip -- device vs host bit-exactness of the field primitives
// (debug aid: the host build of the same headers is the reference).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../hyperdrive_amd/csrc/hd_group.h"
using namespace hd;

__global__ void k_check(const fe* a, const fe* b, fe* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe r;
    fe_mul(r, a[i], b[i]); out[6 * i + 0] = r;
    fe_sqr(r, a[i]); out[6 * i + 1] = r;
    r = a[i]; fe_norm_weak(r); out[6 * i + 2] = r;
    r = a[i]; fe_normalize(r); out[6 * i + 3] = r;
    fe_sqr_n(r, a[i], 88); out[6 * i + 4] = r;
    { fe t; fe_sqr(t, a[i]); fe_mul(r, t, a[i]); } out[6 * i + 5] = r;
    { fe t; fe_sqr(t, a[i]); fe_mul(r, t, b[i]); } out[6 * i + 4] = r;
    { fe t = a[i]; fe_mul(t, t, b[i]); r = t; } out[6 * i + 3] = r;
    { fe t; fe_sqr(t, a[i]); fe_sqr(r, t); } out[6 * i + 2] = r;
}
int main() {
    const int n = 256;
    fe *ha = new fe[n], *hb = new fe[n], *ho = new fe[6 * n], *hr = new fe[6 * n];
    uint32_t s = 12345;
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 9; k++) {
            s = s * 1664525u + 1013904223u; ha[i].n[k] = (s >> 3) & (k == 8 ? HD_M24 : HD_M29);
            s = s * 1664525u + 1013904223u; hb[i].n[k] = (s >> 3) & (k == 8 ? HD_M24 : HD_M29);
        }
    for (int i = 0; i < n; i++) {
        fe r;
        fe_mul(r, ha[i], hb[i]); hr[6 * i + 0] = r;
        fe_sqr(r, ha[i]); hr[6 * i + 1] = r;
        r = ha[i]; fe_norm_weak(r); hr[6 * i + 2] = r;
        r = ha[i]; fe_normalize(r); hr[6 * i + 3] = r;
        fe_sqr_n(r, ha[i], 88); hr[6 * i + 4] = r;
        { fe t; fe_sqr(t, ha[i]); fe_mul(r, t, ha[i]); } hr[6 * i + 5] = r;
        { fe t; fe_sqr(t, ha[i]); fe_mul(r, t, hb[i]); } hr[6 * i + 4] = r;
        { fe t = ha[i]; fe_mul(t, t, hb[i]); r = t; } hr[6 * i + 3] = r;
        { fe t; fe_sqr(t, ha[i]); fe_sqr(r, t); } hr[6 * i + 2] = r;
    }
    fe *da, *db, *dout;
    (void)hipMalloc(&da, n * sizeof(fe)); (void)hipMalloc(&db, n * sizeof(fe)); (void)hipMalloc(&dout, 6 * n * sizeof(fe));
    (void)hipMemcpy(da, ha, n * sizeof(fe), hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb, n * sizeof(fe), hipMemcpyHostToDevice);
    k_check<<<n / 64, 64>>>(da, db, dout, n);
    (void)hipMemcpy(ho, dout, 6 * n * sizeof(fe), hipMemcpyDeviceToHost);
    int bad[6] = {0};
    for (int i = 0; i < n; i++)
        for (int op = 0; op < 6; op++)
            if (memcmp(&ho[6 * i + op], &hr[6 * i + op], sizeof(fe)) != 0) {
                if (bad[op]++ == 0) {
                    printf("op %d lane %d differs:\n dev:", op, i);
                    for (int k = 0; k < 9; k++) printf(" %08x", ho[6 * i + op].n[k]);
                    printf("\n hst:");
                    for (int k = 0; k < 9; k++) printf(" %08x", hr[6 * i + op].n[k]);
                    printf("\n");
                }
            }
    printf("mismatches per op (mul sqr sqrsqr mulalias sqrmul sqr*a): %d %d %d %d %d %d\n", bad[0], bad[1], bad[2], bad[3], bad[4], bad[5]);
    return 0;
}
