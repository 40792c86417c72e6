// swappc_repro.hip -- standalone reproducer (not product code) of the round-3
// 4-waves-per-SIMD mismatch: the full recovery's GLV ladder
// (hd_group.h ecmult_glv) returned wrong points in builds where the compiler
// emitted it as a CALLED device function (s_swappc, call frame and
// callee-saved spills beside the kernel's own spill slots), while every
// inlined build matched the host bit for bit.
//
// Four kernels run the same ladder over the same inputs:
//   inline_w3 / inline_w4    ecmult_glv inlined, 3 / 4 waves per SIMD (168 / 128 VGPRs)
//   call_w3 / call_w4        ecmult_glv behind a __noinline__ wrapper (s_swappc)
// Inputs: R = k G for 1024 seeded k (computed on the host with the same
// headers), u1, u2 seeded scalars.  Expected outputs: the host build of the
// same ecmult_glv (affine x, y canonical).  The program prints, per kernel,
// how many of the 1024 results differ from the host's.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o scripts/swappc_repro scripts/swappc_repro.hip
// ISA:   hipcc ... --offload-device-only -S -o - | grep -c s_swappc   (non-zero only in the call_* kernels)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "../hyperdrive_amd/csrc/hd_group.h"

using namespace hd;

struct Job {
    ge R;
    sc u1, u2;
};
struct Res {
    uint32_t x[8], y[8], inf;
};

static void seed_sc(sc& s, uint64_t& st) {
    for (int i = 0; i < 8; i++) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        s.v[i] = (uint32_t)(st >> 32);
    }
    s.v[7] &= 0x7FFFFFFFu;   // < n
}

template <typename T>
HD void finish(Res& o, const gej& q) {
    o.inf = gej_is_inf(q) ? 1u : 0u;
    if (o.inf) {
        for (int i = 0; i < 8; i++) o.x[i] = o.y[i] = 0;
        return;
    }
    fe x, y;
    gej_to_ge(x, y, q);
    fe_normalize(x);
    fe_normalize(y);
    fe_to_le(o.x, x);
    fe_to_le(o.y, y);
}

__device__ __noinline__ void ladder_call(gej& out, const ge& R, const sc& u1, const sc& u2, const ge* gtab) {
    ecmult_glv(out, R, u1, u2, gtab);
}

template <int WAVES, bool CALL>
__global__ __launch_bounds__(256, WAVES) void k_ladder(const Job* __restrict__ jobs, const ge* __restrict__ gtab,
                                                       Res* __restrict__ out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Job j = jobs[i];
    gej q;
    if (CALL) ladder_call(q, j.R, j.u1, j.u2, gtab);
    else ecmult_glv(q, j.R, j.u1, j.u2, gtab);
    Res o;
    finish<int>(o, q);
    out[i] = o;
}

template <int WAVES, bool CALL>
static int run(const char* name, const Job* dj, const ge* dg, Res* dout, const std::vector<Res>& want) {
    const uint32_t n = (uint32_t)want.size();
    (void)hipMemset(dout, 0xFF, sizeof(Res) * n);
    k_ladder<WAVES, CALL><<<(n + 255) / 256, 256>>>(dj, dg, dout, n);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("%-10s launch failed\n", name);
        return -1;
    }
    std::vector<Res> got(n);
    (void)hipMemcpy(got.data(), dout, sizeof(Res) * n, hipMemcpyDeviceToHost);
    int bad = 0;
    for (uint32_t i = 0; i < n; i++) bad += memcmp(&got[i], &want[i], sizeof(Res)) != 0;
    printf("%-10s %4d of %u ladder results differ from the host build\n", name, bad, n);
    return bad;
}

int main() {
    const uint32_t n = 1024;
    std::vector<ge> gtab(2 * HD_GLV_GTAB_N);
    build_gtab_glv(gtab.data());
    std::vector<Job> jobs(n);
    std::vector<Res> want(n);
    uint64_t st = 12345;
    for (uint32_t i = 0; i < n; i++) {
        sc k, zero;
        seed_sc(k, st);
        for (int w = 0; w < 8; w++) zero.v[w] = 0;
        gej R;
        ecmult_glv(R, gtab[0], zero, k, gtab.data());   // k G (u1 = 0, u2 = k, base G)
        fe x, y;
        gej_to_ge(x, y, R);
        fe_normalize(x);
        fe_normalize(y);
        jobs[i].R.x = x;
        jobs[i].R.y = y;
        seed_sc(jobs[i].u1, st);
        seed_sc(jobs[i].u2, st);
        gej q;
        ecmult_glv(q, jobs[i].R, jobs[i].u1, jobs[i].u2, gtab.data());
        finish<int>(want[i], q);
    }
    Job* dj;
    ge* dg;
    Res* dout;
    (void)hipMalloc(&dj, sizeof(Job) * n);
    (void)hipMalloc(&dg, sizeof(ge) * gtab.size());
    (void)hipMalloc(&dout, sizeof(Res) * n);
    (void)hipMemcpy(dj, jobs.data(), sizeof(Job) * n, hipMemcpyHostToDevice);
    (void)hipMemcpy(dg, gtab.data(), sizeof(ge) * gtab.size(), hipMemcpyHostToDevice);
    int rc = 0;
    rc |= run<3, false>("inline_w3", dj, dg, dout, want) != 0;
    rc |= run<4, false>("inline_w4", dj, dg, dout, want) != 0;
    rc |= run<3, true>("call_w3", dj, dg, dout, want) != 0;
    rc |= run<4, true>("call_w4", dj, dg, dout, want) != 0;
    (void)hipFree(dj);
    (void)hipFree(dg);
    (void)hipFree(dout);
    return rc ? 1 : 0;
}
