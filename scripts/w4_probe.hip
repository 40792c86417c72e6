// w4_probe.hip -- debug aid (not product code): bisects the full recovery of
// hd_verify_msg.h by phase, compiled for 3 and 4 waves per SIMD, so that the
// first phase whose output differs between register budgets (and from the
// host build of the same headers) can be named.
//
// Stage s of k_stage<W, S> runs the recovery from (digest, sig) up to phase S
// and writes that phase's output (16 words per message):
//   0  lift: R.y canonical (x = r[+n] is the input)
//   1  u1 = -m / r, u2 = s / r
//   2  the ladder's Jacobian Q = u1 G + u2 R, made affine (x, y)
//   3  the recovered signatory SHA-256(pubkey) and the verdict
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared
//        -I../include scripts/w4_probe.hip -o scripts/w4_probe.so
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "../hyperdrive_amd/csrc/hd_verify_msg.h"

using namespace hd;

struct PSrc {
    const uint32_t* dg;
    const uint8_t* sig;
    const uint8_t* frm;
    uint32_t i;
    HD_MEMBER uint32_t type() const { return 2; }
    HD_MEMBER int64_t h() const { return 0; }
    HD_MEMBER int64_t r() const { return 0; }
    HD_MEMBER int64_t vr() const { return -1; }
    HD_MEMBER uint32_t value(int) const { return 0; }
    HD_MEMBER uint32_t from(int w) const { return load_be32(frm + 32 * (size_t)i + 4 * w); }
    HD_MEMBER uint32_t sig_r(int w) const { return load_be32(sig + 65 * (size_t)i + 4 * w); }
    HD_MEMBER uint32_t sig_s(int w) const { return load_be32(sig + 65 * (size_t)i + 32 + 4 * w); }
    HD_MEMBER uint32_t sig_v() const { return sig[65 * (size_t)i + 64]; }
    HD_MEMBER bool has_digest() const { return true; }
    HD_MEMBER uint32_t digest(int w) const { return dg[8 * (size_t)i + w]; }
};

// ecmult_glv (hd_group.h) stopped after window jstop: the Jacobian
// accumulator (normalised x, y, z) -- to find the first window whose result
// differs between the device and the host build
template <typename GTab>
HD void ladder_until(gej& acc, const ge& R, const sc& u1, const sc& u2, GTab gtab, int jstop) {
    ge rt[HD_RTAB_N], lt[HD_RTAB_N];
    fe zg;
    build_rtab_iso(rt, lt, zg, R);
    int16_t dra[HD_GLV_NWIN_R], drb[HD_GLV_NWIN_R], dga[HD_GLV_NWIN_G], dgb[HD_GLV_NWIN_G];
    {
        sc k1, k2;
        uint32_t a[5];
        bool neg;
        sc_split_lambda(k1, k2, u2);
        neg = sc_signed_abs(a, k1);
        HD_UNROLL for (int j = 0; j < HD_GLV_NWIN_R; j++) dra[j] = (int16_t)booth_digit160<HD_WR>(a, j, neg);
        neg = sc_signed_abs(a, k2);
        HD_UNROLL for (int j = 0; j < HD_GLV_NWIN_R; j++) drb[j] = (int16_t)booth_digit160<HD_WR>(a, j, neg);
        sc_split_lambda(k1, k2, u1);
        neg = sc_signed_abs(a, k1);
        HD_UNROLL for (int j = 0; j < HD_GLV_NWIN_G; j++) dga[j] = (int16_t)booth_digit160<HD_WG_GLV>(a, j, neg);
        neg = sc_signed_abs(a, k2);
        HD_UNROLL for (int j = 0; j < HD_GLV_NWIN_G; j++) dgb[j] = (int16_t)booth_digit160<HD_WG_GLV>(a, j, neg);
    }
    gej_set_inf(acc);
    HD_NOUNROLL for (int j = HD_GLV_NWIN_R - 1; j >= jstop; j--) {
        if (j != HD_GLV_NWIN_R - 1) {
            HD_NOUNROLL for (int k = 0; k < HD_WR; k++) gej_dbl(acc, acc);
        }
        if (j % 3 == 0) {
            HD_NOUNROLL for (int half = 0; half < 2; half++) {
                const int d = half ? dgb[j / 3] : dga[j / 3];
                const int ad = d < 0 ? -d : d;
                ge t = gtab[half * HD_GLV_GTAB_N + (ad == 0 ? 0 : ad - 1)];
                if (d < 0) fe_neg(t.y, t.y);
                gej s;
                gej_add_ge_zinv(s, acc, t, zg);
                gej_cmov(acc, s, d != 0);
            }
        }
        HD_NOUNROLL for (int half = 0; half < 2; half++) {
            const int d = half ? drb[j] : dra[j];
            const int ad = d < 0 ? -d : d;
            ge t = half ? lt[ad == 0 ? 0 : ad - 1] : rt[ad == 0 ? 0 : ad - 1];
            if (d < 0) fe_neg(t.y, t.y);
            gej s;
            gej_add_ge(s, acc, t);
            gej_cmov(acc, s, d != 0);
        }
    }
}

template <int S>
__host__ __device__ __forceinline__ uint8_t stage_run(const PSrc& src, const ge* gtab, uint32_t out[48],
                                                     int arg = 0) {
    HD_UNROLL for (int k = 0; k < 48; k++) out[k] = 0;
    if (S == 3) {
        uint32_t rec[8];
        int32_t signer;
        const uint8_t v = verify_msg_src(src, gtab, (const uint32_t*)nullptr, 0u, 0, 1, rec, signer);
        HD_UNROLL for (int k = 0; k < 8; k++) out[k] = rec[k];
        return v;
    }
    uint32_t d[8], r_be[8], s_be[8];
    HD_UNROLL for (int w = 0; w < 8; w++) {
        d[w] = src.digest(w);
        r_be[w] = src.sig_r(w);
        s_be[w] = src.sig_s(w);
    }
    const uint32_t v = src.sig_v();
    sc r, s;
    HD_UNROLL for (int i = 0; i < 8; i++) { r.v[i] = r_be[7 - i]; s.v[i] = s_be[7 - i]; }
    uint32_t xw[8];
    HD_UNROLL for (int i = 0; i < 8; i++) xw[i] = r.v[i];
    if (v & 2) {
        const uint32_t N[8] = {HD_N0, HD_N1, HD_N2, HD_N3, HD_N4, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        uint64_t c = 0;
        HD_UNROLL for (int i = 0; i < 8; i++) { c += (uint64_t)xw[i] + N[i]; xw[i] = (uint32_t)c; c >>= 32; }
    }
    fe x;
    fe_from_le(x, xw);
    fe y2, y;
    fe_sqr(y2, x);
    fe_mul(y2, y2, x);
    fe seven;
    fe_set_u32(seven, 7);
    fe_add(y2, y2, seven);
    if (!fe_sqrt(y, y2)) return 3;
    fe_normalize(y);
    if ((uint32_t)(y.n[0] & 1u) != (v & 1u)) {
        fe_neg(y, y);
        fe_normalize(y);
    }
    if (S == 0) {
        fe_to_le(out, y);
        return 0;
    }
    ge R;
    R.x = x;
    R.y = y;
    sc m, rinv, u1, u2;
    sc_from_be_reduce(m, d);
    sc_inv_divsteps(rinv, r);
    sc_mul(u1, m, rinv);
    sc_neg(u1, u1);
    sc_mul(u2, s, rinv);
    if (S == 1) {
        HD_UNROLL for (int k = 0; k < 8; k++) { out[k] = u1.v[k]; out[8 + k] = u2.v[k]; }
        return 0;
    }
    if (S == 10) {   // build_rtab_iso
        ge rt[HD_RTAB_N], lt[HD_RTAB_N];
        fe zg;
        build_rtab_iso(rt, lt, zg, R);
        fe a = zg, b = rt[7].x, c = lt[3].x, d = rt[2].y, e = rt[0].x, f = lt[7].y;
        fe_normalize(a); fe_normalize(b); fe_normalize(c); fe_normalize(d); fe_normalize(e); fe_normalize(f);
        fe_to_le(out, a); fe_to_le(out + 8, b); fe_to_le(out + 16, c); fe_to_le(out + 24, d);
        fe_to_le(out + 32, e); fe_to_le(out + 40, f);
        return 0;
    }
    if (S == 11) {   // GLV splits
        sc k1, k2, k3, k4;
        sc_split_lambda(k1, k2, u1);
        sc_split_lambda(k3, k4, u2);
        HD_UNROLL for (int k = 0; k < 8; k++) {
            out[k] = k1.v[k]; out[8 + k] = k2.v[k]; out[16 + k] = k3.v[k]; out[24 + k] = k4.v[k];
        }
        return 0;
    }
    if (S == 12) {   // Booth digits of the four halves
        sc k1, k2;
        uint32_t a5[5];
        bool neg;
        int16_t dg[88];
        sc_split_lambda(k1, k2, u2);
        neg = sc_signed_abs(a5, k1);
        HD_UNROLL for (int j = 0; j < HD_GLV_NWIN_R; j++) dg[j] = (int16_t)booth_digit160<HD_WR>(a5, j, neg);
        neg = sc_signed_abs(a5, k2);
        HD_UNROLL for (int j = 0; j < HD_GLV_NWIN_R; j++) dg[33 + j] = (int16_t)booth_digit160<HD_WR>(a5, j, neg);
        sc_split_lambda(k1, k2, u1);
        neg = sc_signed_abs(a5, k1);
        HD_UNROLL for (int j = 0; j < HD_GLV_NWIN_G; j++) dg[66 + j] = (int16_t)booth_digit160<HD_WG_GLV>(a5, j, neg);
        neg = sc_signed_abs(a5, k2);
        HD_UNROLL for (int j = 0; j < HD_GLV_NWIN_G; j++) dg[77 + j] = (int16_t)booth_digit160<HD_WG_GLV>(a5, j, neg);
        HD_UNROLL for (int k = 0; k < 44; k++) out[k] = (uint32_t)(uint16_t)dg[2 * k] | ((uint32_t)(uint16_t)dg[2 * k + 1] << 16);
        return 0;
    }
    if (S == 13) {   // one G addition on E' (gej_add_ge_zinv) from a doubled R
        ge rt[HD_RTAB_N], lt[HD_RTAB_N];
        fe zg;
        build_rtab_iso(rt, lt, zg, R);
        gej a, o;
        gej_set_ge(a, rt[2]);
        gej_dbl(a, a);
        const ge t = gtab[5 + (d[0] & 1023u)];
        gej_add_ge_zinv(o, a, t, zg);
        fe x = o.x, y = o.y, z = o.z;
        fe_normalize(x); fe_normalize(y); fe_normalize(z);
        fe_to_le(out, x); fe_to_le(out + 8, y); fe_to_le(out + 16, z);
        gej_add_ge(o, a, rt[5]);
        x = o.x; y = o.y; z = o.z;
        fe_normalize(x); fe_normalize(y); fe_normalize(z);
        fe_to_le(out + 24, x); fe_to_le(out + 32, y); fe_to_le(out + 40, z);
        return 0;
    }
    if (S == 16 || S == 17) {   // the ladder stopped after window arg (17: G only)
        sc zero;
        HD_UNROLL for (int k = 0; k < 8; k++) zero.v[k] = 0;
        gej acc;
        ladder_until(acc, R, u1, S == 17 ? zero : u2, gtab, arg);
        fe x = acc.x, y = acc.y, z = acc.z;
        fe_normalize(x); fe_normalize(y); fe_normalize(z);
        fe_to_le(out, x); fe_to_le(out + 8, y); fe_to_le(out + 16, z);
        return 0;
    }
    gej Q;
    if (S == 14 || S == 15) {   // the ladder with one side only
        sc zero;
        HD_UNROLL for (int k = 0; k < 8; k++) zero.v[k] = 0;
        if (S == 14) ecmult_glv(Q, R, zero, u2, gtab);
        else ecmult_glv(Q, R, u1, zero, gtab);
    } else {
        ecmult_glv(Q, R, u1, u2, gtab);
    }
    if (gej_is_inf(Q)) return 4;
    fe qx, qy;
    gej_to_ge(qx, qy, Q);
    fe_to_le(out, qx);
    fe_to_le(out + 8, qy);
    return 0;
}

template <int W, int S>
__global__ __launch_bounds__(256, W) void k_stage(uint32_t n, const uint32_t* __restrict__ dg,
                                                  const uint8_t* __restrict__ sig, const uint8_t* __restrict__ from,
                                                  const ge* __restrict__ gtab, uint32_t* __restrict__ out,
                                                  uint8_t* __restrict__ verdict, int arg) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    PSrc src{dg, sig, from, i};
    uint32_t o[48];
    const uint8_t v = stage_run<S>(src, gtab, o, arg);
    HD_UNROLL for (int k = 0; k < 48; k++) out[48 * (size_t)i + k] = o[k];
    verdict[i] = v;
}

template <int W>
static void launch(int stage, uint32_t n, const uint32_t* dg, const uint8_t* sig, const uint8_t* from,
                   const ge* gtab, uint32_t* out, uint8_t* verdict, int arg) {
    const uint32_t b = (n + 255) / 256;
#define HD_ST(S) else if (stage == S) k_stage<W, S><<<b, 256>>>(n, dg, sig, from, gtab, out, verdict, arg)
    if (0) {}
    HD_ST(0); HD_ST(1); HD_ST(2); HD_ST(3); HD_ST(10); HD_ST(11); HD_ST(12); HD_ST(13); HD_ST(14); HD_ST(15);
    HD_ST(16); HD_ST(17);
#undef HD_ST
}

// host: digests (8 BE words per message), sigs (65 B), froms (32 B) -> out
// (16 words per message) and verdicts, for waves W (3 or 4) and stage 0..3
extern "C" int probe_run(int waves, int stage, int arg, uint32_t n, const uint32_t* dg, const uint8_t* sig,
                         const uint8_t* from, uint32_t* out, uint8_t* verdict) {
    static std::vector<ge> tab;
    if (tab.empty()) {
        tab.resize(2 * HD_GLV_GTAB_N);
        build_gtab_glv(tab.data());
    }
    ge* d_tab;
    uint32_t *d_dg, *d_out;
    uint8_t *d_sig, *d_from, *d_v;
    if (hipMalloc(&d_tab, sizeof(ge) * tab.size()) || hipMalloc(&d_dg, 32 * (size_t)n) ||
        hipMalloc(&d_out, 192 * (size_t)n) || hipMalloc(&d_sig, 65 * (size_t)n) ||
        hipMalloc(&d_from, 32 * (size_t)n) || hipMalloc(&d_v, n))
        return -2;
    hipMemcpy(d_tab, tab.data(), sizeof(ge) * tab.size(), hipMemcpyHostToDevice);
    hipMemcpy(d_dg, dg, 32 * (size_t)n, hipMemcpyHostToDevice);
    hipMemcpy(d_sig, sig, 65 * (size_t)n, hipMemcpyHostToDevice);
    hipMemcpy(d_from, from, 32 * (size_t)n, hipMemcpyHostToDevice);
    if (waves == 4) launch<4>(stage, n, d_dg, d_sig, d_from, d_tab, d_out, d_v, arg);
    else launch<3>(stage, n, d_dg, d_sig, d_from, d_tab, d_out, d_v, arg);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, d_out, 192 * (size_t)n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(verdict, d_v, n, hipMemcpyDeviceToHost);
    hipFree(d_tab);
    hipFree(d_dg);
    hipFree(d_out);
    hipFree(d_sig);
    hipFree(d_from);
    hipFree(d_v);
    return e == hipSuccess ? 0 : -3;
}

// the same stages on the host (g++-equivalent host build of the headers)
extern "C" int probe_host(int stage, int arg, uint32_t n, const uint32_t* dg, const uint8_t* sig,
                          const uint8_t* from, uint32_t* out, uint8_t* verdict) {
    static std::vector<ge> tab;
    if (tab.empty()) {
        tab.resize(2 * HD_GLV_GTAB_N);
        build_gtab_glv(tab.data());
    }
    for (uint32_t i = 0; i < n; i++) {
        PSrc src{dg, sig, from, i};
        uint32_t o[48];
        uint8_t v = 0;
#define HD_ST(S) else if (stage == S) v = stage_run<S>(src, tab.data(), o, arg)
        if (0) {}
        HD_ST(0); HD_ST(1); HD_ST(2); HD_ST(3); HD_ST(10); HD_ST(11); HD_ST(12); HD_ST(13); HD_ST(14); HD_ST(15);
        HD_ST(16); HD_ST(17);
#undef HD_ST
        for (int k = 0; k < 48; k++) out[48 * (size_t)i + k] = o[k];
        verdict[i] = v;
    }
    return 0;
}
