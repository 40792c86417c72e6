// Host (g++) build of the device math headers -- TEST HARNESS ONLY.
// Lets the CPU-only test suite exercise, bit for bit, the arithmetic the
// gfx950 kernels run (hyperdrive_amd/csrc/*.h), against the oracle.
#include <stdio.h>
#include <string.h>
#include <vector>
#include "../../hyperdrive_amd/csrc/hd_gen.h"
#include "../../hyperdrive_amd/csrc/hd_fixedbase.h"
#include "../../hyperdrive_amd/csrc/hd_scmont.h"
#include "../../hyperdrive_amd/csrc/hd_keccak.h"
#include "../../hyperdrive_amd/csrc/hd_modinv.h"

using namespace hd;

static ge g_tab[2 * HD_GLV_GTAB_N];
static bool g_init = false;
static const ge* gtab() {
    if (!g_init) { build_gtab_glv(g_tab); g_init = true; }
    return g_tab;
}
static void le_in(uint32_t* o, const uint8_t* b) { for (int i = 0; i < 8; i++) o[i] = load_be32(b + 4 * (7 - i)); }
static void le_out(uint8_t* b, const uint32_t* o) { for (int i = 0; i < 8; i++) store_be32(b + 4 * (7 - i), o[i]); }
static void fe_in(fe& r, const uint8_t* b) { uint32_t w[8]; le_in(w, b); fe_from_le(r, w); }
static void fe_out(uint8_t* b, const fe& a) { fe t = a; fe_normalize(t); uint32_t w[8]; fe_to_le(w, t); le_out(b, w); }

extern "C" {
// all 32-byte operands big-endian
void hdh_fe_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
    fe x, y, r;
    fe_in(x, a);
    fe_in(y, b);
    int ok = 1;
    switch (op) {
        case 0: fe_mul(r, x, y); break;
        case 1: fe_sqr(r, x); break;
        case 2: fe_add(r, x, y); break;
        case 3: fe_sub(r, x, y); break;
        case 4: fe_neg(r, x); break;
        case 5: fe_inv(r, x); break;
        case 6: ok = fe_sqrt(r, x); break;
        case 7: fe_inv_divsteps(r, x); break;
        default: fe_clear(r);
    }
    fe_out(out, r);
    out[32] = (uint8_t)ok;
}
void hdh_sc_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
    sc x, y, r;
    le_in(x.v, a);
    le_in(y.v, b);
    switch (op) {
        case 0: sc_mul(r, x, y); break;
        case 1: sc_sqr(r, x); break;
        case 2: sc_neg(r, x); break;
        case 3: sc_inv(r, x); break;
        case 4: { uint32_t w[8]; for (int i = 0; i < 8; i++) w[i] = load_be32(a + 4 * i); sc_from_be_reduce(r, w); break; }
        case 5: sc_inv_divsteps(r, x); break;
        default: for (int i = 0; i < 8; i++) r.v[i] = 0;
    }
    le_out(out, r.v);
}
void hdh_gtab(uint8_t* out /* 128 x 64 */) {
    const ge* t = gtab();
    for (int k = 0; k < 2 * HD_GTAB_N; k++) {  // 1G..128G, then lambda 1G..128G
        const ge& e = t[k < HD_GTAB_N ? k : HD_GLV_GTAB_N + (k - HD_GTAB_N)];
        fe_out(out + 64 * k, e.x);
        fe_out(out + 64 * k + 32, e.y);
    }
}
int hdh_booth(const uint8_t* k32, int w, int j) {
    sc k;
    le_in(k.v, k32);
    return w == 4 ? booth_digit<4>(k, j) : booth_digit<8>(k, j);
}
// Q = u1 G + u2 R (R affine given); returns 1 if inf; out = x||y
int hdh_ecmult(const uint8_t* rx, const uint8_t* ry, const uint8_t* u1b, const uint8_t* u2b, uint8_t* out) {
    ge R;
    fe_in(R.x, rx);
    fe_in(R.y, ry);
    sc u1, u2;
    le_in(u1.v, u1b);
    le_in(u2.v, u2b);
    gej Q;
    ecmult(Q, R, u1, u2, gtab());
    if (gej_is_inf(Q)) return 1;
    fe x, y;
    gej_to_ge(x, y, Q);
    fe_out(out, x);
    fe_out(out + 32, y);
    return 0;
}
int hdh_recover(const uint8_t* digest, const uint8_t* sig, uint8_t* pub64) {
    uint32_t d[8], rb[8], sb[8];
    for (int i = 0; i < 8; i++) { d[i] = load_be32(digest + 4 * i); rb[i] = load_be32(sig + 4 * i); sb[i] = load_be32(sig + 32 + 4 * i); }
    fe qx, qy;
    int v = recover(qx, qy, d, rb, sb, sig[64], gtab());
    if (v == V_VALID) { fe_out(pub64, qx); fe_out(pub64 + 32, qy); }
    return v;
}
void hdh_sign(const uint8_t* sk32, const uint8_t* digest, uint8_t* sig65) {
    sc sk;
    le_in(sk.v, sk32);
    uint32_t d[8], rb[8], sb[8], rid;
    for (int i = 0; i < 8; i++) d[i] = load_be32(digest + 4 * i);
    ecdsa_sign(rb, sb, rid, sk, d, gtab());
    for (int i = 0; i < 8; i++) { store_be32(sig65 + 4 * i, rb[i]); store_be32(sig65 + 32 + 4 * i, sb[i]); }
    sig65[64] = (uint8_t)rid;
}
void hdh_signer_sk(uint32_t idx, uint8_t* out) {
    sc sk;
    signer_sk(sk, idx);
    le_out(out, sk.v);
}
void hdh_keys(uint32_t S, int compressed, uint8_t* sigs32, uint8_t* foreign32) {
    for (uint32_t j = 0; j < S + HD_NONADMITTED_KEYS; j++) {
        uint32_t idx = j < S ? j : HD_NONADMITTED_BASE + (j - S);
        sc sk;
        signer_sk(sk, idx);
        uint32_t o[8];
        pubkey_signatory(o, sk, compressed, gtab());
        uint8_t* dst = j < S ? sigs32 + 32 * j : foreign32 + 32 * (j - S);
        for (int i = 0; i < 8; i++) store_be32(dst + 4 * i, o[i]);
    }
}
static std::vector<uint32_t> words_of(const uint8_t* b, uint32_t n) {
    std::vector<uint32_t> w(8 * (size_t)n);
    for (size_t i = 0; i < 8 * (size_t)n; i++) w[i] = load_be32(b + 4 * i);
    return w;
}
int hdh_gen(uint32_t kind, uint64_t start, uint32_t n, uint32_t S, uint32_t adv_pct, const uint8_t* sigs32,
            const uint8_t* foreign32, uint8_t* type, int64_t* h, int64_t* r, int64_t* vr, uint8_t* value32,
            uint8_t* from32, uint8_t* sig65, int8_t* cls) {
    std::vector<uint32_t> sw = words_of(sigs32, S), fw = words_of(foreign32, HD_NONADMITTED_KEYS);
    for (uint32_t k = 0; k < n; k++) {
        cls[k] = (int8_t)gen_message(kind, start + k, S, adv_pct, gtab(), sw.data(), fw.data(), type[k], h[k], r[k],
                                     vr[k], value32 + 32 * (size_t)k, from32 + 32 * (size_t)k, sig65 + 65 * (size_t)k);
    }
    return 0;
}
// host run of verify_msg over a batch (admitted must be sorted ascending)
int hdh_verify(uint32_t n, const uint8_t* type, const int64_t* h, const int64_t* r, const int64_t* vr,
               const uint8_t* value32, const uint8_t* from32, const uint8_t* sig65, const uint8_t* adm32,
               uint32_t n_adm, int compressed, uint8_t* verdict, uint8_t* rec32, int32_t* signer) {
    std::vector<uint32_t> aw = words_of(adm32, n_adm);
    int steps = 0;
    while ((1u << steps) < n_adm) steps++;
    for (uint32_t i = 0; i < n; i++) {
        MsgIn m;
        m.type = type[i];
        m.h = h[i];
        m.r = r[i];
        m.vr = vr ? vr[i] : -1;
        for (int w = 0; w < 8; w++) {
            m.value_be[w] = load_be32(value32 + 32 * (size_t)i + 4 * w);
            m.from_be[w] = load_be32(from32 + 32 * (size_t)i + 4 * w);
            m.r_be[w] = load_be32(sig65 + 65 * (size_t)i + 4 * w);
            m.s_be[w] = load_be32(sig65 + 65 * (size_t)i + 32 + 4 * w);
        }
        m.v = sig65[65 * (size_t)i + 64];
        uint32_t rec[8];
        int32_t s;
        verdict[i] = verify_msg(m, gtab(), aw.data(), n_adm, steps, compressed, rec, s);
        signer[i] = s;
        for (int w = 0; w < 8; w++) store_be32(rec32 + 32 * (size_t)i + 4 * w, rec[w]);
    }
    return 0;
}
}
extern "C" int hdh_ecmult_trace(const uint8_t* rx, const uint8_t* ry, const uint8_t* u1b, const uint8_t* u2b, uint8_t* out, uint8_t* infs) {
    ge R; fe_in(R.x, rx); fe_in(R.y, ry);
    sc u1, u2; le_in(u1.v, u1b); le_in(u2.v, u2b);
    const ge* gt = gtab();
    gej rt[HD_RTAB_N];
    gej_set_ge(rt[0], R);
    gej_dbl(rt[1], rt[0]);
    for (int k = 2; k < HD_RTAB_N; k++) gej_add_ge(rt[k], rt[k - 1], R);
    gej acc; gej_set_inf(acc);
    for (int j = HD_NWIN_R - 1; j >= 0; j--) {
        if (j != HD_NWIN_R - 1) for (int k = 0; k < HD_WR; k++) gej_dbl(acc, acc);
        if ((j & 1) == 0) {
            int d = booth_digit<HD_WG>(u1, j >> 1); int ad = d < 0 ? -d : d;
            ge t = gt[ad == 0 ? 0 : ad - 1]; if (d < 0) fe_neg(t.y, t.y);
            gej s; gej_add_ge(s, acc, t); gej_cmov(acc, s, d != 0);
        }
        { int d = booth_digit<HD_WR>(u2, j); int ad = d < 0 ? -d : d;
          gej t = rt[ad == 0 ? 0 : ad - 1]; if (d < 0) fe_neg(t.y, t.y);
          gej s; gej_add(s, acc, t); gej_cmov(acc, s, d != 0); }
        infs[j] = gej_is_inf(acc);
        if (!infs[j]) { fe x, y; gej_to_ge(x, y, acc); fe_out(out + 64 * j, x); fe_out(out + 64 * j + 32, y); }
    }
    return 0;
}
// raw-limb access for the lazy-reduction bound tests (9 limbs of 29 bits)
extern "C" void hdh_fe_raw(int op, const uint32_t* a9, const uint32_t* b9, uint32_t* out9) {
    fe a, b, r;
    for (int i = 0; i < 9; i++) { a.n[i] = a9[i]; b.n[i] = b9[i]; }
#ifdef HD_BOUND_CHECKS
    fe_bound_exact(a);
    fe_bound_exact(b);
#endif
    switch (op) {
        case 0: fe_mul(r, a, b); break;
        case 1: fe_sqr(r, a); break;
        case 2: r = a; fe_norm_weak(r); break;
        case 3: r = a; fe_normalize(r); break;
        default: fe_clear(r);
    }
    for (int i = 0; i < 9; i++) out9[i] = r.n[i];
}

#ifdef HD_BOUND_CHECKS
// ---- bound certification (built with -DHD_BOUNDS) -------------------------
static int g_bound_fails = 0;
static char g_bound_first[256] = "";
extern "C" void hd_bound_fail(const char* what, int line) {
    if (g_bound_fails++ == 0) {
        snprintf(g_bound_first, sizeof g_bound_first, "%s (hd_field.h/hd_group.h line %d)", what, line);
        fprintf(stderr, "bound violation: %s\n", g_bound_first);
    }
}
extern "C" int hdh_bound_failures(char* first, int cap) {
    snprintf(first, cap, "%s", g_bound_first);
    int n = g_bound_fails;
    g_bound_fails = 0;
    g_bound_first[0] = 0;
    return n;
}
static void set_class(fe& a, int k) {  // bound = k * T (k = 1 tight, 2 = fresh negation)
    for (int i = 0; i < 9; i++) a.b[i] = (uint64_t)k * fe_t_limb(i);
}
static void point_T(gej& p, int yk = 1) { set_class(p.x, 1); set_class(p.y, yk); set_class(p.z, 1); }
// Runs every point formula (main and exceptional paths) with operand bounds
// at their class maxima; returns the number of violated preconditions.
extern "C" int hdh_bound_certify(const uint8_t* px, const uint8_t* py, const uint8_t* qx, const uint8_t* qy) {
    ge P, Q;
    fe_in(P.x, px); fe_in(P.y, py); fe_in(Q.x, qx); fe_in(Q.y, qy);
    gej a, b, r;
    gej_set_ge(a, P);
    gej_dbl(a, a);                      // a: Jacobian with z != 1
    gej_set_ge(b, Q);
    gej_dbl(b, b);
    point_T(a);
    point_T(b);
    // doubling
    gej_dbl(r, a);
    // mixed addition, b.y tight and negated (2T)
    ge qn = Q;
    set_class(qn.x, 1); set_class(qn.y, 1);
    gej_add_ge(r, a, qn);
    fe_neg(qn.y, Q.y); set_class(qn.y, 2);
    gej_add_ge(r, a, qn);
    // full addition, b.y tight and negated
    gej bn = b;
    gej_add(r, a, bn);
    fe_neg(bn.y, b.y); set_class(bn.y, 2);
    gej_add(r, a, bn);
    // exceptional paths: a = inf; a = b (doubling); a = -b (cancel)
    gej inf; gej_set_inf(inf);
    gej_add_ge(r, inf, qn);
    gej_add(r, inf, bn);
    gej aq; gej_set_ge(aq, Q); point_T(aq);
    ge qq = Q; set_class(qq.x, 1); set_class(qq.y, 1);
    gej_add_ge(r, aq, qq);              // a == b
    fe_neg(qq.y, Q.y); set_class(qq.y, 2);
    gej_add_ge(r, aq, qq);              // a == -b
    gej_add(r, b, b);
    gej bneg = b; fe_neg(bneg.y, b.y); set_class(bneg.y, 2);
    gej_add(r, b, bneg);
    // the known-key check's addition (no exceptional branches), b.y 2T and T,
    // and its first-digit start (an affine point, y weakly normalised)
    fe_neg(qn.y, Q.y); set_class(qn.y, 2);
    gej_add_ge_nx(r, a, qn);
    qn.y = Q.y; set_class(qn.y, 1);
    gej_add_ge_nx(r, a, qn);
    gej_add_ge_nx(r, aq, qq);           // a == -b: Z3 = 0, still in bounds
    // the first addition of a fixed-base sum (two affine points), b.y T and 2T
    {
        ge pa = P; set_class(pa.x, 1); set_class(pa.y, 1);
        ge qb = Q; set_class(qb.x, 1); set_class(qb.y, 1);
        gej_add_ge_z1(r, pa, qb);
        fe_neg(qb.y, Q.y); set_class(qb.y, 2);
        gej_add_ge_z1(r, pa, qb);
    }
    // the XYZZ sums of k_fast_sums: the loop invariant (X 5T, Y 3T, ZZ and
    // ZZZ tight in; the same classes out) for a table point y of T and 2T,
    // the affine first addition, the zero-digit select, the stored form
    {
        gxz xa;
        xa.x = a.x; xa.y = a.y; xa.zz = a.z; xa.zzz = a.z;
        set_class(xa.x, 5); set_class(xa.y, 3); set_class(xa.zz, 1); set_class(xa.zzz, 1);
        ge pb = Q; set_class(pb.x, 1); set_class(pb.y, 1);
        ge nb = Q; fe_neg(nb.y, Q.y); set_class(nb.y, 2);
        gxz o;
        auto in_class = [](const gxz& g) {
            for (int i = 0; i < 9; i++) {
                HD_BREQ(g.x.b[i] <= 5ull * fe_t_limb(i), "gxz: X out of its 5T class");
                HD_BREQ(g.y.b[i] <= 3ull * fe_t_limb(i), "gxz: Y out of its 3T class");
                HD_BREQ(g.zz.b[i] <= fe_t_limb(i) && g.zzz.b[i] <= fe_t_limb(i), "gxz: ZZ / ZZZ not tight");
            }
        };
        gxz_add_ge_nx(o, xa, pb); in_class(o);
        gxz_add_ge_nx(o, xa, nb); in_class(o);
        ge pa = P; set_class(pa.x, 1); set_class(pa.y, 1);
        gxz_add_ge_z1(o, pa, pb); in_class(o);
        gxz_add_ge_z1(o, pa, nb); in_class(o);
        gxz first;
        gxz_set_ge(first, nb);
        fe_norm_weak(first.y);
        gxz s = o;
        gxz_cmov(s, first, true);
        gxz_cmov(xa, s, true); in_class(xa);
        fe xn, yn, t;
        gxz_finish(xn, yn, t, xa);
        fe w = t;
        fe xr = P.x; set_class(xr, 1);
        (void)fast_final_xz(xn, yn, w, xr, 0);
    }
    // isomorphic-curve additions (G side of the ladder) and the R table build
    fe zg = b.z; set_class(zg, 1);
    gej_add_ge_zinv(r, a, qn, zg);
    qn.y = Q.y; set_class(qn.y, 1);
    gej_add_ge_zinv(r, a, qn, zg);
    gej_add_ge_zinv(r, inf, qn, zg);
    ge rt[HD_RTAB_N], lt[HD_RTAB_N];
    build_rtab_iso(rt, lt, zg, P);
    for (int k = 0; k < HD_RTAB_N; k++) { fe_require_T(rt[k].x, "rtab x"); fe_require_T(rt[k].y, "rtab y"); }
    // field chains on a T input
    fe t = P.x, o;
    set_class(t, 1);
    fe_inv(o, t);
    fe_sqrt(o, t);
    char buf[256];
    return hdh_bound_failures(buf, sizeof buf);
}
#endif

extern "C" int hdh_ecmult_glv(const uint8_t* rx, const uint8_t* ry, const uint8_t* u1b, const uint8_t* u2b, uint8_t* out) {
    ge R;
    fe_in(R.x, rx);
    fe_in(R.y, ry);
    sc u1, u2;
    le_in(u1.v, u1b);
    le_in(u2.v, u2b);
    gej Q;
    ecmult_glv(Q, R, u1, u2, gtab());
    if (gej_is_inf(Q)) return 1;
    fe x, y;
    gej_to_ge(x, y, Q);
    fe_out(out, x);
    fe_out(out + 32, y);
    return 0;
}
extern "C" void hdh_split(const uint8_t* kb, uint8_t* k1b, uint8_t* k2b) {
    sc k, k1, k2;
    le_in(k.v, kb);
    sc_split_lambda(k1, k2, k);
    le_out(k1b, k1.v);
    le_out(k2b, k2.v);
}

// signatory hash of hd_sha256.h's sha256_pubkey for arbitrary coordinates
// (not necessarily on the curve: exercises every encoding length)
extern "C" void hdh_pubkey_hash(int fmt, const uint8_t* x32, const uint8_t* y32, uint8_t* out32) {
    uint32_t xb[8], yb[8], d[8];
    for (int w = 0; w < 8; w++) { xb[w] = load_be32(x32 + 4 * w); yb[w] = load_be32(y32 + 4 * w); }
    sha256_pubkey(d, fmt, xb, yb, yb[7] & 1u);
    for (int w = 0; w < 8; w++) store_be32(out32 + 4 * w, d[w]);
}

// Keccak sponge of hd_keccak.h over a host byte string (pad 0x01 Keccak-256,
// 0x06 SHA3-256)
extern "C" void hdh_keccak_bytes(int pad, const uint8_t* data, uint64_t len, uint8_t* out32) {
    uint32_t d[8];
    keccak256_bytes(d, len, (uint8_t)pad, [&](uint64_t off) {
        uint64_t lane = 0;
        for (int k = 0; k < 8; k++)
            if (off + k < len) lane |= (uint64_t)data[off + k] << (8 * k);
        return lane;
    });
    for (int w = 0; w < 8; w++) store_be32(out32 + 4 * w, d[w]);
}
// preimage digest of one message with the fixed-size Keccak paths
extern "C" void hdh_keccak_msg(int pad, int type, int64_t h, int64_t r, int64_t vr, const uint8_t* value32,
                               uint8_t* out32) {
    uint32_t v[8], d[8];
    for (int w = 0; w < 8; w++) v[w] = load_be32(value32 + 4 * w);
    if (type == T_PROPOSE) keccak256_propose(d, h, r, vr, v, (uint8_t)pad);
    else keccak256_vote(d, h, r, v, (uint8_t)pad);
    for (int w = 0; w < 8; w++) store_be32(out32 + 4 * w, d[w]);
}

// Known-key fast path of hd_fixedbase.h on the host: tables of G and of the
// key (x, y big-endian) are built with fb_window_base / fb_entry exactly as
// the device builds them (cached for the last key), then verify_fast.
template <int W>
static std::vector<ge> fb_tables(const ge& B) {
    std::vector<ge> t(FbL<W>::TAB);
    ge bj;
    int jprev = -1;
    for (uint32_t e = 0; e < FbL<W>::TAB; e++) {
        int j;
        uint32_t d;
        fb_entry_pos<W>(e, j, d);
        if (j != jprev) fb_window_base(bj, B, W, j);
        jprev = j;
        fb_entry(t[e], bj, d);
    }
    return t;
}
static std::vector<ge> fb_gt, fb_pt;
std::vector<ge>* hdh_fb_cache(int which) { return which == 0 ? &fb_gt : &fb_pt; }
extern "C" int hdh_fb_verify(const uint8_t* pub64, const uint8_t* digest, const uint8_t* sig65) {
    std::vector<ge>& gt = fb_gt;
    std::vector<ge>& pt = fb_pt;
    static uint8_t last[64];
    static bool have = false;
    if (gt.empty()) {
        ge g;
        g.x = gtab()[0].x;
        g.y = gtab()[0].y;
        gt = fb_tables<HD_FB_WG>(g);
    }
    if (!have || memcmp(last, pub64, 64) != 0) {
        ge P;
        fe_in(P.x, pub64);
        fe_in(P.y, pub64 + 32);
        pt = fb_tables<HD_FB_W>(P);
        memcpy(last, pub64, 64);
        have = true;
    }
    uint32_t d[8], r[8], sw[8];
    for (int w = 0; w < 8; w++) {
        d[w] = load_be32(digest + 4 * w);
        r[w] = load_be32(sig65 + 4 * w);
        sw[w] = load_be32(sig65 + 32 + 4 * w);
    }
    return verify_fast(d, r, sw, sig65[64], gt.data(), pt.data());
}
// one table entry d 2^(12 j) B (x || y big-endian), for the table-layout test
// scalar Montgomery product (hd_scmont.h): out = a b R^-1 mod n, canonical
// (operands 32-byte big-endian);
// raw9 != NULL also returns the 9 radix-2^29 limbs before the final reduction
extern "C" void hdh_sm_mul(const uint8_t* a_le, const uint8_t* b_le, uint8_t* out_le, uint32_t* raw9) {
    sc a, b, o;
    le_in(a.v, a_le);
    le_in(b.v, b_le);
    sm x, y, r;
    sm_from_sc(x, a);
    sm_from_sc(y, b);
    sm_mul(r, x, y);
    if (raw9) for (int i = 0; i < 9; i++) raw9[i] = r.n[i];
    sm_to_sc(o, r);
    le_out(out_le, o.v);
}
// a chain of Montgomery products on radix-2^29 values kept below 2n:
// x <- x * y_k for k steps (inputs canonical), result canonical
extern "C" void hdh_sm_chain(const uint8_t* x_le, const uint8_t* ys_le, int k, uint8_t* out_le) {
    sc a, o;
    le_in(a.v, x_le);
    sm x;
    sm_from_sc(x, a);
    for (int t = 0; t < k; t++) {
        sc b;
        le_in(b.v, ys_le + 32 * t);
        sm y;
        sm_from_sc(y, b);
        sm_mul(x, x, y);
    }
    sm_to_sc(o, x);
    le_out(out_le, o.v);
}

// two affine points added with the first-step formula of the fixed-base sum
// (gej_add_ge_z1); returns 1 when Z3 = 0 (a = +-b), else out = affine x || y
extern "C" int hdh_add_affine(const uint8_t* ax, const uint8_t* ay, const uint8_t* bx, const uint8_t* by,
                              uint8_t* out64) {
    ge a, b;
    fe_in(a.x, ax); fe_in(a.y, ay); fe_in(b.x, bx); fe_in(b.y, by);
    gej r;
    gej_add_ge_z1(r, a, b);
    if (gej_is_inf(r)) return 1;
    fe x, y;
    gej_to_ge(x, y, r);
    fe_out(out64, x);
    fe_out(out64 + 32, y);
    return 0;
}

// k_fast_sums' XYZZ accumulation on the host: n affine points (x || y
// big-endian, 64 B each), point k negated when neg[k] and skipped when
// skip[k] (a zero digit), summed by the kernel's own window step
// (gxz_sum_step: the first window's point starts the sum, the affine first
// addition, then the general one, each into the other accumulator and
// followed by the repair branch when `rare`).  force_rare runs the repair branch at every step (the kernel runs
// it whenever any lane of the wavefront needs it), else only where this
// lane needs it.  The result goes through gxz_finish, one inversion and
// fast_final_xz's products.  Returns 1 for a degenerate sum (ZZ = 0 or
// nothing started), else out = affine x || y.
extern "C" int hdh_xyzz_sum(const uint8_t* pts, const int* neg, const int* skip, int n, uint8_t* out64,
                            int force_rare) {
    gxz acc;
    ge p0;
    bool started = false;
    for (int k = 0; k < n; k++) {
        ge g;
        fe_in(g.x, pts + 64 * k);
        fe_in(g.y, pts + 64 * k + 32);
        const bool nz = !skip[k];
        if (k == 0) {
            p0 = g;
            if (neg[k]) fe_neg(p0.y, p0.y);
            fe_norm_weak(p0.y);
            gxz_set_ge(acc, p0);
            started = nz;
            continue;
        }
        const bool rare = force_rare || !(started && nz);
        gxz next;   // the kernel's two accumulators in turn
        if (k == 1) gxz_sum_step<true>(next, acc, started, p0, g, neg[k] != 0, nz, rare);
        else gxz_sum_step<false>(next, acc, started, p0, g, neg[k] != 0, nz, rare);
        acc = next;
    }
    if (!started || gxz_is_inf(acc)) return 1;
    fe xn, yn, t, w, ax, ay;
    gxz_finish(xn, yn, t, acc);
    fe_inv(w, t);
    fe_mul(ax, xn, w);
    fe_mul(ay, yn, w);
    fe_out(out64, ax);
    fe_out(out64 + 32, ay);
    return 0;
}

extern "C" void hdh_fb_entry(const uint8_t* b64, int j, uint32_t d, uint8_t* out64) {
    ge B, bj, e;
    fe_in(B.x, b64);
    fe_in(B.y, b64 + 32);
    fb_window_base(bj, B, HD_FB_W, j);
    fb_entry(e, bj, d);
    fe_out(out64, e.x);
    fe_out(out64 + 32, e.y);
}
// fb_digit (the known-key check's window digits) for a 256-bit scalar (BE)
extern "C" int hdh_fb_digits(const uint8_t* k32, int* out) {
    sc k;
    le_in(k.v, k32);
    for (int j = 0; j < HD_FB_NWIN; j++) out[j] = fb_digit<HD_FB_W>(k, j);
    return HD_FB_NWIN;
}

// verify_fast2 on the host: two messages against two keys' tables (the
// caches of hdh_fb_verify are reused: both messages use the same key)
extern "C" void hdh_fb_verify2(const uint8_t* pub64, const uint8_t* digests, const uint8_t* sigs, const int* ready,
                               uint8_t* out) {
    uint8_t dummy[65] = {0};
    hdh_fb_verify(pub64, dummy, dummy);  // builds / refreshes the table caches
    FastIn in[2];
    for (int k = 0; k < 2; k++) {
        for (int w = 0; w < 8; w++) {
            in[k].digest_be[w] = load_be32(digests + 32 * k + 4 * w);
            in[k].r_be[w] = load_be32(sigs + 65 * k + 4 * w);
            in[k].s_be[w] = load_be32(sigs + 65 * k + 32 + 4 * w);
        }
        in[k].v = sigs[65 * k + 64];
        in[k].ready = ready[k] != 0;
    }
    FastPark park;
    verify_fast2(out, in, hdh_fb_cache(0)->data(), hdh_fb_cache(1)->data(), hdh_fb_cache(1)->data(), &park);
}

// ecmult_glv_fbg (hd_fixedbase.h: the full recovery's u1 G from a fixed-base
// G table) over an 8-bit-window host table of G (32 windows: 11 interleaved
// with the ladder, 21 after it), against ecmult_glv; returns 1 for infinity.
static const ge* fbg8_table() {
    static std::vector<ge> tab;
    if (tab.empty()) {
        tab.resize(FbL<8>::TAB);
        const ge& G = gtab()[0];
        for (int j = 0; j < FbL<8>::NWIN; j++) {
            ge bj;
            fb_window_base(bj, G, 8, j);
            const uint32_t nd = j == FbL<8>::NWIN - 1 ? FbL<8>::NTOP : FbL<8>::N;
            for (uint32_t d = 1; d <= nd; d++) fb_entry(tab[(size_t)j * FbL<8>::N + d - 1], bj, d);
        }
    }
    return tab.data();
}
extern "C" int hdh_ecmult_glv_fbg8(const uint8_t* rx, const uint8_t* ry, const uint8_t* u1b, const uint8_t* u2b,
                                   uint8_t* out) {
    ge R;
    sc u1, u2;
    fe_in(R.x, rx);
    fe_in(R.y, ry);
    le_in(u1.v, u1b);
    le_in(u2.v, u2b);
    gej Q;
    ecmult_glv_fbg<8>(Q, R, u1, u2, fbg8_table());
    if (gej_is_inf(Q)) return 1;
    fe x, y;
    gej_to_ge(x, y, Q);
    fe_out(out, x);
    fe_out(out + 32, y);
    return 0;
}

// fb_is_infinity (hd_fixedbase.h) over the host's 12-bit G table: R and the
// scalars m, s as 32-byte big-endian values; 1 iff R == (m / s) G
extern "C" int hdh_fb_is_infinity(const uint8_t* rx, const uint8_t* ry, const uint8_t* m32, const uint8_t* s32) {
    if (fb_gt.empty()) {   // the G table cache hdh_fb_verify uses
        ge g;
        g.x = gtab()[0].x;
        g.y = gtab()[0].y;
        fb_gt = fb_tables<HD_FB_WG>(g);
    }
    ge R;
    fe_in(R.x, rx);
    fe_in(R.y, ry);
    sc m, s;
    le_in(m.v, m32);
    le_in(s.v, s32);
    return fb_is_infinity<HD_FB_WG>(m, s, R, fb_gt.data()) ? 1 : 0;
}

// the admitted table's hashed index (hd_verify_msg.h AdmIndex) against the
// binary search, for n sorted 32-byte entries and q query keys: out[k] = the
// index lookup, out[q + k] = the binary search
extern "C" void hdh_adm_lookup(const uint8_t* sorted32, uint32_t n, const uint8_t* keys32, uint32_t q, int32_t* out) {
    std::vector<uint32_t> words(8 * (size_t)n);
    for (size_t k = 0; k < words.size(); k++) words[k] = hd::load_be32(sorted32 + 4 * k);
    const uint32_t slots = hd::adm_index_slots(n);
    std::vector<uint32_t> ix(slots);
    hd::adm_index_build(words.data(), n, ix.data(), slots);
    int steps = 0;
    while ((1u << steps) < n) steps++;
    for (uint32_t k = 0; k < q; k++) {
        uint32_t key[8];
        for (int w = 0; w < 8; w++) key[w] = hd::load_be32(keys32 + 32 * (size_t)k + 4 * w);
        out[k] = n ? hd::adm_index_find(words.data(), ix.data(), slots - 1, key) : -1;
        out[q + k] = hd::admitted_find(words.data(), n, steps, key);
    }
}

// the foreign-key dictionary's bucket and its host rebuild (fb_evict)
extern "C" uint32_t hdh_fdict_bucket(const uint32_t* from_be) { return hd::fdict_bucket(from_be); }
extern "C" int hdh_fdict_rebuild(const uint32_t* from_be, const uint32_t* slot, uint32_t n, uint32_t* nd,
                                 int32_t* where) {
    return hd::fdict_rebuild(nd, where, from_be, slot, n) ? 1 : 0;
}
extern "C" int32_t hdh_fdict_find(const uint32_t* nd, const uint32_t* from_be) { return hd::fdict_find(nd, from_be); }
