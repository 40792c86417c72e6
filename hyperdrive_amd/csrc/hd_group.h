// hd_group.h -- secp256k1 points (a = 0), the double-scalar multiplication
// used by recovery, and the recovery itself with libsecp256k1 semantics
// (go-ethereum v1.9.5 crypto/secp256k1 -> secp256k1_ext_ecdsa_recover).
//
// SIMD design note: per-lane wNAF sparsity buys nothing on a 64-wide
// wavefront -- some lane always has a non-zero digit, so every lane would pay
// every addition.  The ladder therefore uses *uniform* Booth-recoded fixed
// windows over the GLV halves: 4-bit windows for the variable point R and
// lambda R (tables 1R..8R, per lane, made affine on an isomorphic curve, in
// scratch) and 12-bit windows for G and lambda G (1G..2048G, affine, 288 KiB
// read through L2 -- it does not fit the 160 KiB LDS next to the kernel's
// occupancy, and L2 hits measured as fast).  Every lane runs
// the identical sequence of doublings/additions; a zero digit is a per-lane
// select, and the exceptional cases of the addition law (P = inf, P = +-T)
// are rare branches.
//
// Jacobian infinity is Z == 0 (mod p), tested on the normalised value.
#pragma once
#include "hd_field.h"
#include "hd_modinv.h"

namespace hd {

struct ge { fe x, y; };          // affine
struct gej { fe x, y, z; };      // Jacobian, Z == 0 <=> infinity

HD bool gej_is_inf(const gej& a) { return fe_is_zero(a.z); }
HD void gej_set_inf(gej& r) { fe_clear(r.x); fe_set_u32(r.y, 1); fe_clear(r.z); }
HD void gej_set_ge(gej& r, const ge& a) { r.x = a.x; r.y = a.y; fe_set_u32(r.z, 1); }
HD void gej_cmov(gej& r, const gej& a, bool flag) {
    fe_cmov(r.x, a.x, flag);
    fe_cmov(r.y, a.y, flag);
    fe_cmov(r.z, a.z, flag);
}

// Bounds (hd_field.h): every point coordinate is T, except that the y of a
// table entry may be a fresh negation 2p - y (2T).  Outputs are T.  The
// formulas are certified by the host bound tracker (HD_BOUNDS) for all inputs
// of those classes (tests/test_field_bounds.py).

// Doubling (a = 0), 4S + 3M (dbl-2009-l shape with D = (2X)(2Y^2) and
// 8Y^4 = 2 (2Y^2)^2 so that no limb-wise multiple exceeds 32 bits).
// inf -> inf (Z3 = 2 Y Z = 0).  r may alias a.
HD void gej_dbl(gej& r, const gej& a) {
    HD_REQUIRE_T(a.x, "gej_dbl: x");
    HD_REQUIRE_T(a.y, "gej_dbl: y");
    HD_REQUIRE_T(a.z, "gej_dbl: z");
    fe A, D, C4, E, t, u;
    fe_sqr(A, a.x);            // X^2               T
    fe_sqr(u, a.y);            // B = Y^2           T
    fe_add(u, u, u);           // 2B                2T
    fe_add(t, a.x, a.x);       // 2X                2T
    fe_mul(D, t, u);           // D = 4 X Y^2       T
    fe_sqr(C4, u);             // 4 Y^4             T
    fe_add(u, a.y, a.y);       // 2Y                2T
    fe_mul(r.z, u, a.z);       // Z3 = 2 Y Z        T   (a.z, a.y dead from here)
    fe_mul_int(E, A, 3);
    fe_norm_weak(E);           // E = 3 X^2         T
    fe_sqr(t, E);              // E^2               T
    fe_add(u, D, D);           // 2D                2T
    fe_sub_k<3>(r.x, t, u);
    fe_norm_weak(r.x);         // X3 = E^2 - 2D     T
    fe_sub_k<2>(t, D, r.x);    // D - X3            3T
    fe_mul(t, E, t);           // E (D - X3)        T
    fe_add(u, C4, C4);         // 8 Y^4             2T
    fe_sub_k<3>(r.y, t, u);
    fe_norm_weak(r.y);         // Y3                T
}

// the doubling of the rare a == b case of the additions, inlined like everything
// else: a kernel with no device calls has no call frames next to its spill
// slots (a called ladder miscompiled on gfx950, scripts/w4_probe.hip, DESIGN.md
// §4 "Known issue, resolved")
HD void gej_dbl_slow(gej& r, const gej& a) { gej_dbl(r, a); }

// r = a + b, b affine and finite (madd-2007-bl shape, 8M + 3S with
// Z3 = 2 Z1 H).  Handles a = inf (up front, so b is dead after the first
// products) and a = +-b.  b.y may be 2T.
HD void gej_add_ge(gej& r, const gej& a, const ge& b) {
    HD_REQUIRE_T(a.x, "gej_add_ge: x");
    HD_REQUIRE_T(a.y, "gej_add_ge: y");
    HD_REQUIRE_T(a.z, "gej_add_ge: z");
    HD_REQUIRE_T(b.x, "gej_add_ge: b.x");
    if (fe_is_zero(a.z)) {
        gej o;
        gej_set_ge(o, b);
        fe_norm_weak(o.y);
        r = o;
        return;
    }
    fe z1z1, u2, s2, h, R, t;
    fe_sqr(z1z1, a.z);         // T
    fe_mul(u2, b.x, z1z1);     // T
    fe_mul(s2, b.y, a.z);      // T (2T x T)
    fe_mul(s2, s2, z1z1);      // T
    fe_sub_k<2>(h, u2, a.x);
    fe_norm_weak(h);           // H = U2 - X1       T
    fe_sub_k<2>(R, s2, a.y);   // r = S2 - Y1       3T
    if (fe_is_zero(h)) {
        // a == +-b (rare): double or cancel
        gej o;
        if (fe_is_zero(R)) {
            gej bj;
            gej_set_ge(bj, b);
            fe_norm_weak(bj.y);
            gej_dbl_slow(o, bj);
        } else {
            gej_set_inf(o);
        }
        r = o;
        return;
    }
    gej o;
    fe_add(t, a.z, a.z);
    fe_mul(o.z, t, h);         // Z3 = 2 Z1 H       T
    fe hh, i4, j, v;
    fe_norm_weak(R);
    fe_add(R, R, R);           // 2r                2T
    fe_sqr(hh, h);             // T
    fe_mul_int(i4, hh, 4);     // I = 4 H^2         4T
    fe_mul(j, h, i4);          // J = H I           T
    fe_mul(v, a.x, i4);        // V = X1 I          T
    fe_sqr(o.x, R);            // T
    fe_add(t, v, v);
    fe_add(t, t, j);           // 2V + J            3T
    fe_sub_k<4>(o.x, o.x, t);
    fe_norm_weak(o.x);         // X3                T
    fe_sub_k<2>(t, v, o.x);    // V - X3            3T
    fe_mul(t, R, t);           // r (V - X3)        T (2T x 3T)
    fe_mul(j, a.y, j);
    fe_add(j, j, j);           // 2 Y1 J            2T
    fe_sub_k<3>(o.y, t, j);
    fe_norm_weak(o.y);         // Y3                T
    r = o;
}

// Mixed addition on an isomorphic curve ("effective affine", as in
// libsecp256k1's ecmult): b is affine on E: y^2 = x^3 + 7 while a lives on
// E': y^2 = x^3 + 7 zg^6, where a point (x, y) of E is (x zg^2, y zg^3).
// Substituting az = a.z zg for a.z in U2 = b.x az^2, S2 = b.y az^3 adds the
// image of b without computing it; Z3 = 2 a.z H as usual.  One multiply more
// than gej_add_ge.  The rare paths (a = inf, a = +-b) build the image
// explicitly.
HD void gej_add_ge_zinv(gej& r, const gej& a, const ge& b, const fe& zg) {
    HD_REQUIRE_T(a.x, "gej_add_ge_zinv: x");
    HD_REQUIRE_T(a.y, "gej_add_ge_zinv: y");
    HD_REQUIRE_T(a.z, "gej_add_ge_zinv: z");
    HD_REQUIRE_T(b.x, "gej_add_ge_zinv: b.x");
    HD_REQUIRE_T(zg, "gej_add_ge_zinv: zg");
    if (fe_is_zero(a.z)) {
        gej o;
        fe z2;
        fe_sqr(z2, zg);
        fe_mul(o.x, b.x, z2);
        fe_mul(z2, z2, zg);
        fe_mul(o.y, b.y, z2);
        fe_set_u32(o.z, 1);
        r = o;
        return;
    }
    fe az, z1z1, u2, s2, h, R, t;
    fe_mul(az, a.z, zg);       // T
    fe_sqr(z1z1, az);          // T
    fe_mul(u2, b.x, z1z1);     // T
    fe_mul(s2, b.y, az);       // T (2T x T)
    fe_mul(s2, s2, z1z1);      // T
    fe_sub_k<2>(h, u2, a.x);
    fe_norm_weak(h);           // H = U2 - X1       T
    fe_sub_k<2>(R, s2, a.y);   // r = S2 - Y1       3T
    if (fe_is_zero(h)) {
        gej o;
        if (fe_is_zero(R)) {
            gej bj;
            fe z2;
            fe_sqr(z2, zg);
            fe_mul(bj.x, b.x, z2);
            fe_mul(z2, z2, zg);
            fe_mul(bj.y, b.y, z2);
            fe_set_u32(bj.z, 1);
            gej_dbl_slow(o, bj);
        } else {
            gej_set_inf(o);
        }
        r = o;
        return;
    }
    gej o;
    fe_add(t, a.z, a.z);
    fe_mul(o.z, t, h);         // Z3 = 2 Z1 H       T
    fe hh, i4, j, v;
    fe_norm_weak(R);
    fe_add(R, R, R);           // 2r                2T
    fe_sqr(hh, h);
    fe_mul_int(i4, hh, 4);     // I = 4 H^2         4T
    fe_mul(j, h, i4);          // J = H I           T
    fe_mul(v, a.x, i4);        // V = X1 I          T
    fe_sqr(o.x, R);
    fe_add(t, v, v);
    fe_add(t, t, j);           // 2V + J            3T
    fe_sub_k<4>(o.x, o.x, t);
    fe_norm_weak(o.x);         // X3                T
    fe_sub_k<2>(t, v, o.x);    // V - X3            3T
    fe_mul(t, R, t);           // r (V - X3)        T
    fe_mul(j, a.y, j);
    fe_add(j, j, j);           // 2 Y1 J            2T
    fe_sub_k<3>(o.y, t, j);
    fe_norm_weak(o.y);         // Y3                T
    r = o;
}

// r = a + b (b affine) for the table build, also returning the z ratio
// zr = Z3 / Z1 = 2 H.  a != inf, a != +-b (multiples 2R..7R of a point of
// prime order n never hit those).
HD void gej_add_ge_zr(gej& r, const gej& a, const ge& b, fe& zr) {
    fe z1z1, u2, s2, h, R, t;
    fe_sqr(z1z1, a.z);
    fe_mul(u2, b.x, z1z1);
    fe_mul(s2, b.y, a.z);
    fe_mul(s2, s2, z1z1);
    fe_sub_k<2>(h, u2, a.x);
    fe_norm_weak(h);
    fe_sub_k<2>(R, s2, a.y);
    gej o;
    fe_add(zr, h, h);          // 2H                2T
    fe_mul(o.z, a.z, zr);      // Z3 = 2 Z1 H       T
    fe hh, i4, j, v;
    fe_norm_weak(R);
    fe_add(R, R, R);
    fe_sqr(hh, h);
    fe_mul_int(i4, hh, 4);
    fe_mul(j, h, i4);
    fe_mul(v, a.x, i4);
    fe_sqr(o.x, R);
    fe_add(t, v, v);
    fe_add(t, t, j);
    fe_sub_k<4>(o.x, o.x, t);
    fe_norm_weak(o.x);
    fe_sub_k<2>(t, v, o.x);
    fe_mul(t, R, t);
    fe_mul(j, a.y, j);
    fe_add(j, j, j);
    fe_sub_k<3>(o.y, t, j);
    fe_norm_weak(o.y);
    r = o;
}

// r = a + b, both Jacobian, b finite (add-2007-bl shape, 12M + 4S with
// Z3 = 2 Z1 Z2 H).  Handles a = inf (up front) and a = +-b.  b.y may be 2T.
HD void gej_add(gej& r, const gej& a, const gej& b) {
    HD_REQUIRE_T(a.x, "gej_add: x");
    HD_REQUIRE_T(a.y, "gej_add: y");
    HD_REQUIRE_T(a.z, "gej_add: z");
    HD_REQUIRE_T(b.x, "gej_add: b.x");
    HD_REQUIRE_T(b.z, "gej_add: b.z");
    if (fe_is_zero(a.z)) {
        gej o = b;
        fe_norm_weak(o.y);
        r = o;
        return;
    }
    fe z1z1, z2z2, u1, u2, s1, s2, h, R, t, z12;
    fe_sqr(z1z1, a.z);
    fe_sqr(z2z2, b.z);
    fe_mul(u1, a.x, z2z2);
    fe_mul(u2, b.x, z1z1);
    fe_mul(s1, a.y, b.z);
    fe_mul(s1, s1, z2z2);
    fe_mul(s2, b.y, a.z);      // 2T x T
    fe_mul(s2, s2, z1z1);
    fe_mul(z12, a.z, b.z);
    fe_sub_k<2>(h, u2, u1);
    fe_norm_weak(h);           // H                 T
    fe_sub_k<2>(R, s2, s1);    // r                 3T
    if (fe_is_zero(h)) {
        gej o;
        if (fe_is_zero(R)) gej_dbl_slow(o, a);
        else gej_set_inf(o);
        r = o;
        return;
    }
    gej o;
    fe_norm_weak(R);
    fe_add(R, R, R);           // 2r                2T
    fe_add(t, h, h);           // 2H                2T
    fe_mul(o.z, z12, t);       // Z3 = 2 Z1 Z2 H    T
    fe i, j, v;
    fe_sqr(i, t);              // I = (2H)^2        T
    fe_mul(j, h, i);           // J = H I           T
    fe_mul(v, u1, i);          // V = U1 I          T
    fe_sqr(o.x, R);
    fe_add(t, v, v);
    fe_add(t, t, j);           // 2V + J            3T
    fe_sub_k<4>(o.x, o.x, t);
    fe_norm_weak(o.x);         // X3 = r^2 - J - 2V T
    fe_sub_k<2>(t, v, o.x);    // V - X3            3T
    fe_mul(t, R, t);           // T
    fe_add(s1, s1, s1);
    fe_mul(s1, s1, j);         // 2 S1 J            T
    fe_sub_k<2>(o.y, t, s1);
    fe_norm_weak(o.y);         // Y3 = r (V - X3) - 2 S1 J
    r = o;
}

// ------------------------------------------------------------ recoding
// Booth digit of window j (width W) of a 256-bit scalar k:
//   d = b[Wj-1] + sum_{t<W-1} 2^t b[Wj+t] - 2^(W-1) b[Wj+W-1],  |d| <= 2^(W-1)
HD uint32_t sc_bits(const sc& k, int pos, int len) {
    // bits [pos, pos+len) of k, bits outside [0,256) read as 0; len <= 17
    uint32_t out = 0;
    HD_UNROLL for (int t = 0; t < 17; t++) {
        if (t < len) {
            int b = pos + t;
            uint32_t bit = (b >= 0 && b < 256) ? ((k.v[b >> 5] >> (b & 31)) & 1u) : 0u;
            out |= bit << t;
        }
    }
    return out;
}
template <int W>
HD int booth_digit(const sc& k, int j) {
    uint32_t x = sc_bits(k, W * j - 1, W + 1);
    return (int)((x >> 1) + (x & 1)) - (int)((x >> W) << W);
}

#define HD_WR 4                       // R window
#define HD_WG 8                       // G window
#define HD_NWIN_R (256 / HD_WR + 1)   // 65 windows
#define HD_NWIN_G (256 / HD_WG + 1)   // 33 windows
#define HD_GTAB_N (1 << (HD_WG - 1))  // 128 affine multiples 1G..128G
#define HD_RTAB_N (1 << (HD_WR - 1))  // 8 Jacobian multiples 1R..8R

// Q = u1*G + u2*R.  gtab[k] = (k+1) G affine (k < 128).
template <typename GTab>
HD void ecmult(gej& out, const ge& R, const sc& u1, const sc& u2, GTab gtab) {
    gej rt[HD_RTAB_N];
    gej_set_ge(rt[0], R);
    gej_dbl(rt[1], rt[0]);
    HD_NOUNROLL for (int k = 2; k < HD_RTAB_N; k++) gej_add_ge(rt[k], rt[k - 1], R);

    int16_t dr[HD_NWIN_R], dg[HD_NWIN_G];  // |digit| <= 128: int8 would overflow
    HD_UNROLL for (int j = 0; j < HD_NWIN_R; j++) dr[j] = (int16_t)booth_digit<HD_WR>(u2, j);
    HD_UNROLL for (int j = 0; j < HD_NWIN_G; j++) dg[j] = (int16_t)booth_digit<HD_WG>(u1, j);

    gej acc;
    gej_set_inf(acc);
    HD_NOUNROLL for (int j = HD_NWIN_R - 1; j >= 0; j--) {
        if (j != HD_NWIN_R - 1) {
            HD_NOUNROLL for (int k = 0; k < HD_WR; k++) gej_dbl(acc, acc);
        }
        if ((j & 1) == 0) {
            int d = dg[j >> 1];
            int ad = d < 0 ? -d : d;
            ge t = gtab[ad == 0 ? 0 : ad - 1];
            if (d < 0) fe_neg(t.y, t.y);
            gej s;
            gej_add_ge(s, acc, t);
            gej_cmov(acc, s, d != 0);
        }
        {
            int d = dr[j];
            int ad = d < 0 ? -d : d;
            gej t = rt[ad == 0 ? 0 : ad - 1];
            if (d < 0) fe_neg(t.y, t.y);
            gej s;
            gej_add(s, acc, t);
            gej_cmov(acc, s, d != 0);
        }
    }
    out = acc;
}

// ------------------------------------------------------------ GLV
// secp256k1 endomorphism: lambda * (x, y) = (beta * x, y), lambda^3 = 1 mod n,
// beta^3 = 1 mod p.  A scalar k splits as k = k1 + k2 lambda (mod n) with
// |k1|, |k2| < 2^128 (lattice basis from the extended Euclid on (n, lambda);
// constants derived and checked in tests/test_glv.py), so u1 G + u2 R becomes
// a 4-scalar ladder of 132 doublings instead of 256.
HD void sc_add(sc& r, const sc& a, const sc& b) {
    uint32_t o[8];
    uint64_t c = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) { c += (uint64_t)a.v[i] + b.v[i]; o[i] = (uint32_t)c; c >>= 32; }
    if (c || sc_ge_n(o)) sc_sub_n(o);
    HD_UNROLL for (int i = 0; i < 8; i++) r.v[i] = o[i];
}
// round(k * g / 2^384) for a 256-bit constant g
HD void sc_mul_shift384(sc& r, const sc& k, const uint32_t g[8]) {
    uint32_t t[16];
    mul_256(t, k.v, g);
    uint64_t c = (t[11] >> 31);
    HD_UNROLL for (int i = 0; i < 4; i++) { c += t[12 + i]; r.v[i] = (uint32_t)c; c >>= 32; }
    r.v[4] = (uint32_t)c;
    HD_UNROLL for (int i = 5; i < 8; i++) r.v[i] = 0;
}
HD void sc_split_lambda(sc& k1, sc& k2, const sc& k) {
    const uint32_t G1[8] = {0x45DBB031u, 0xE893209Au, 0x71E8CA7Fu, 0x3DAA8A14u,
                            0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u};
    const uint32_t G2[8] = {0x8AC47F71u, 0x1571B4AEu, 0x9DF506C6u, 0x221208ACu,
                            0x0ABFE4C4u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u};
    sc mb1, mb2, mlam, c1, c2, t;
    const uint32_t MB1[8] = {0x0ABFE4C3u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u, 0u, 0u, 0u, 0u};
    const uint32_t MB2[8] = {0x3DB1562Cu, 0xD765CDA8u, 0x0774346Du, 0x8A280AC5u,
                             0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    const uint32_t MLAM[8] = {0xB51283CFu, 0xE0CFC810u, 0x8EC739C2u, 0xA880B9FCu,
                              0x77ED9BA4u, 0x5AD9E3FDu, 0x3FA3CF1Fu, 0xAC9C52B3u};
    HD_UNROLL for (int i = 0; i < 8; i++) { mb1.v[i] = MB1[i]; mb2.v[i] = MB2[i]; mlam.v[i] = MLAM[i]; }
    sc_mul_shift384(c1, k, G1);
    sc_mul_shift384(c2, k, G2);
    sc_mul(c1, c1, mb1);
    sc_mul(c2, c2, mb2);
    sc_add(k2, c1, c2);          // k2 = -c1 b1 - c2 b2
    sc_mul(t, k2, mlam);
    sc_add(k1, k, t);            // k1 = k - k2 lambda
}
// |k| as a 5-word (160-bit) magnitude and its sign (k > n/2 means negative)
HD bool sc_signed_abs(uint32_t a[5], const sc& k) {
    const uint32_t NH[8] = {0x681B20A0u, 0xDFE92F46u, 0x57A4501Du, 0x5D576E73u,
                            0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};
    bool lt = false, gt = false;
    HD_UNROLL for (int i = 7; i >= 0; i--) {
        bool g = !lt && !gt && k.v[i] > NH[i];
        bool l = !lt && !gt && k.v[i] < NH[i];
        gt = gt || g;
        lt = lt || l;
    }
    sc m = k;
    if (gt) sc_neg(m, k);
    HD_UNROLL for (int i = 0; i < 5; i++) a[i] = m.v[i];
    return gt;
}
// Booth digit of window j (width W) of a 160-bit magnitude, sign applied
template <int W>
HD int booth_digit160(const uint32_t a[5], int j, bool neg) {
    uint32_t x = 0;
    HD_UNROLL for (int t = 0; t <= W; t++) {
        const int b = W * j - 1 + t;
        const uint32_t bit = (b >= 0 && b < 160) ? ((a[b >> 5] >> (b & 31)) & 1u) : 0u;
        x |= bit << t;
    }
    const int d = (int)((x >> 1) + (x & 1)) - (int)((x >> W) << W);
    return neg ? -d : d;
}

#define HD_GLV_NWIN_R 33   // 4-bit windows over 132 bits
#define HD_WG_GLV 12       // G window of the GLV ladder (= 3 R windows)
#define HD_GLV_NWIN_G 11   // 12-bit windows over 132 bits
#define HD_GLV_GTAB_N (1 << (HD_WG_GLV - 1))  // 2048 affine multiples per base

HD void fe_beta(fe& b) {
    const uint32_t BETA[8] = {0x719501EEu, 0xC1396C28u, 0x12F58995u, 0x9CF04975u,
                              0xAC3434E9u, 0x6E64479Eu, 0x657C0710u, 0x7AE96A2Bu};
    fe_from_le(b, BETA);
}

// Per-lane table of 1R..8R, all brought to one Jacobian Z (zg), so they are
// affine points of the isomorphic curve E' (gej_add_ge_zinv): the R-side
// ladder additions become mixed additions.  z ratios of the building chain
// (dbl, then madd) give the rescale factors walking back from 8R.
// Returns zg (T); tab[k] = (k+1) R on E', lam[k] = lambda (k+1) R on E'.
HD void build_rtab_iso(ge tab[HD_RTAB_N], ge lam[HD_RTAB_N], fe& zg, const ge& R) {
    gej p[HD_RTAB_N];
    fe zr[HD_RTAB_N];          // zr[k] = Z_k / Z_{k-1}
    gej_set_ge(p[0], R);
    gej_dbl(p[1], p[0]);
    fe_add(zr[1], R.y, R.y);   // Z_1 = 2 Y Z_0, Z_0 = 1
    HD_NOUNROLL for (int k = 2; k < HD_RTAB_N; k++) gej_add_ge_zr(p[k], p[k - 1], R, zr[k]);
    zg = p[HD_RTAB_N - 1].z;
    tab[HD_RTAB_N - 1].x = p[HD_RTAB_N - 1].x;
    tab[HD_RTAB_N - 1].y = p[HD_RTAB_N - 1].y;
    fe f = zr[HD_RTAB_N - 1];  // Z_7 / Z_6
    fe_norm_weak(f);
    HD_NOUNROLL for (int k = HD_RTAB_N - 2; k >= 0; k--) {
        // f = Z_7 / Z_k
        fe f2, f3;
        fe_sqr(f2, f);
        fe_mul(f3, f2, f);
        fe_mul(tab[k].x, p[k].x, f2);
        fe_mul(tab[k].y, p[k].y, f3);
        if (k > 0) fe_mul(f, f, zr[k]);
    }
    fe beta;
    fe_beta(beta);
    HD_NOUNROLL for (int k = 0; k < HD_RTAB_N; k++) {
        fe_mul(lam[k].x, tab[k].x, beta);
        lam[k].y = tab[k].y;
    }
}

// Q = u1 G + u2 R with the endomorphism.  gtab[0..2047] = (k+1) G,
// gtab[2048..4095] = (k+1) lambda G (affine on E, 288 KiB: read through the
// L2, 72 bytes per G addition).  The accumulator runs on the
// isomorphic curve E' of the R table (build_rtab_iso); the G additions map
// their point on the fly (gej_add_ge_zinv) and Q is mapped back at the end
// (Z *= zg).
template <typename GTab>
HD void ecmult_glv(gej& out, const ge& R, const sc& u1, const sc& u2, GTab gtab) {
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
    gej acc;
    gej_set_inf(acc);
    HD_NOUNROLL for (int j = HD_GLV_NWIN_R - 1; j >= 0; j--) {
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
    fe_mul(acc.z, acc.z, zg);  // back from E' to E
    out = acc;
}

// Multiples 1G..nG in affine form (canonical), by one chain of additions and
// a Montgomery batch inversion of the Z coordinates (one modular inversion
// for the whole table).  Host-side precomputation.
HD_HOSTONLY void build_gmultiples(ge* tab, int n) {
    ge g;
    const uint32_t GX[8] = {0x79BE667Eu, 0xF9DCBBACu, 0x55A06295u, 0xCE870B07u,
                            0x029BFCDBu, 0x2DCE28D9u, 0x59F2815Bu, 0x16F81798u};
    const uint32_t GY[8] = {0x483ADA77u, 0x26A3C465u, 0x5DA4FBFCu, 0x0E1108A8u,
                            0xFD17B448u, 0xA6855419u, 0x9C47D08Fu, 0xFB10D4B8u};
    fe_from_be(g.x, GX);
    fe_from_be(g.y, GY);
    tab[0] = g;
    if (n < 2) return;
    fe* z = new fe[n];
    fe* pre = new fe[n];
    gej acc;
    gej_set_ge(acc, g);
    for (int k = 1; k < n; k++) {
        if (k == 1) gej_dbl(acc, acc);
        else gej_add_ge(acc, acc, g);
        tab[k].x = acc.x;  // Jacobian X, Y until the pass below
        tab[k].y = acc.y;
        z[k] = acc.z;
        if (k == 1) pre[1] = z[1];
        else fe_mul(pre[k], pre[k - 1], z[k]);
    }
    fe inv;
    fe_inv_divsteps(inv, pre[n - 1]);  // (Z_1 ... Z_{n-1})^-1
    for (int k = n - 1; k >= 1; k--) {
        fe zi, zi2, zi3;
        if (k > 1) {
            fe_mul(zi, inv, pre[k - 1]);
            fe_mul(inv, inv, z[k]);    // (Z_1 ... Z_{k-1})^-1
        } else {
            zi = inv;
        }
        fe_sqr(zi2, zi);
        fe_mul(zi3, zi2, zi);
        fe_mul(tab[k].x, tab[k].x, zi2);
        fe_mul(tab[k].y, tab[k].y, zi3);
        fe_normalize(tab[k].x);
        fe_normalize(tab[k].y);
    }
    delete[] z;
    delete[] pre;
}
// [1G .. HD_GLV_GTAB_N G] followed by lambda times those = (beta x, y).  The
// first HD_GTAB_N entries double as the 8-bit-window table of ecmult_gen.
HD_HOSTONLY void build_gtab_glv(ge* tab) {
    build_gmultiples(tab, HD_GLV_GTAB_N);
    fe beta;
    fe_beta(beta);
    for (int k = 0; k < HD_GLV_GTAB_N; k++) {
        fe_mul(tab[HD_GLV_GTAB_N + k].x, tab[k].x, beta);
        fe_normalize(tab[HD_GLV_GTAB_N + k].x);
        tab[HD_GLV_GTAB_N + k].y = tab[k].y;
    }
}

// affine, canonical (a finite)
HD void gej_to_ge(fe& x, fe& y, const gej& a) {
    fe zi, zi2;
    fe_inv_divsteps(zi, a.z);
    fe_sqr(zi2, zi);
    fe_mul(x, a.x, zi2);
    fe_mul(zi2, zi2, zi);
    fe_mul(y, a.y, zi2);
    fe_normalize(x);
    fe_normalize(y);
}

// ------------------------------------------------------------ recovery
// libsecp256k1 recover semantics:
//   V >= 4 -> BAD_RECID (go-ethereum checkSignature); r or s >= n -> BAD_RS
//   (parse_compact overflow); r or s == 0 -> BAD_RS (sig_recover);
//   V&2 and r >= p - n -> NO_POINT; x^3+7 non-residue -> NO_POINT;
//   Q = inf -> INFINITY.  High-S accepted.  m = digest mod n.
// On VALID writes the affine Q (x, y), canonical.
// gtab: 2 * HD_GLV_GTAB_N entries (build_gtab_glv).
// the multiplication Q = u1 G + u2 R of the recovery (ecmult_glv over the
// small GLV G table; hd_fixedbase.h has a form over the fixed-base G table)
template <typename GTab>
struct GlvMult {
    GTab gtab;
    HD_MEMBER void operator()(gej& out, const ge& R, const sc& u1, const sc& u2) const {
        ecmult_glv(out, R, u1, u2, gtab);
    }
};

template <typename Mult>
HD uint8_t recover_m(fe& qx, fe& qy, const uint32_t digest_be[8], const uint32_t r_be[8],
                     const uint32_t s_be[8], uint32_t v, Mult mult) {
    if (v >= 4) return V_BAD_RECID;
    sc r, s;
    HD_UNROLL for (int i = 0; i < 8; i++) { r.v[i] = r_be[7 - i]; s.v[i] = s_be[7 - i]; }
    if (sc_ge_n(r.v) || sc_ge_n(s.v)) return V_BAD_RS;
    if (sc_is_zero(r) || sc_is_zero(s)) return V_BAD_RS;
    uint32_t xw[8];
    HD_UNROLL for (int i = 0; i < 8; i++) xw[i] = r.v[i];
    if (v & 2) {
        // x = r + n must stay < p  <=>  r < p - n
        // p - n = 0x14551231950B75FC4402DA1722FC9BAEE (129 bits, LE limbs below)
        const uint32_t PMN[8] = {0x2FC9BAEEu, 0x402DA172u, 0x50B75FC4u, 0x45512319u, 1u, 0u, 0u, 0u};
        bool lt = false, gt = false;
        HD_UNROLL for (int i = 7; i >= 0; i--) {
            bool g = !lt && !gt && r.v[i] > PMN[i];
            bool l = !lt && !gt && r.v[i] < PMN[i];
            gt = gt || g;
            lt = lt || l;
        }
        if (!lt) return V_NO_POINT;
        const uint32_t N[8] = {HD_N0, HD_N1, HD_N2, HD_N3, HD_N4, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        uint64_t c = 0;
        HD_UNROLL for (int i = 0; i < 8; i++) { c += (uint64_t)xw[i] + N[i]; xw[i] = (uint32_t)c; c >>= 32; }
    }
    fe x;
    fe_from_le(x, xw);                // x < p: canonical
    fe y2, y;
    fe_sqr(y2, x);
    fe_mul(y2, y2, x);
    fe seven;
    fe_set_u32(seven, 7);
    fe_add(y2, y2, seven);
    if (!fe_sqrt(y, y2)) return V_NO_POINT;
    fe_normalize(y);
    if ((uint32_t)(y.n[0] & 1u) != (v & 1u)) {
        fe_neg(y, y);
        fe_normalize(y);
    }
    ge R;
    R.x = x;
    R.y = y;

    sc m, rinv, u1, u2;
    sc_from_be_reduce(m, digest_be);
    sc_inv_divsteps(rinv, r);
    sc_mul(u1, m, rinv);
    sc_neg(u1, u1);
    sc_mul(u2, s, rinv);

    gej Q;
    mult(Q, R, u1, u2);
    if (gej_is_inf(Q)) return V_INFINITY;
    fe zi, zi2;
    fe_inv_divsteps(zi, Q.z);
    fe_sqr(zi2, zi);
    fe_mul(qx, Q.x, zi2);
    fe_mul(zi2, zi2, zi);
    fe_mul(qy, Q.y, zi2);
    fe_normalize(qx);
    fe_normalize(qy);
    return V_VALID;
}
template <typename GTab>
HD uint8_t recover(fe& qx, fe& qy, const uint32_t digest_be[8], const uint32_t r_be[8],
                   const uint32_t s_be[8], uint32_t v, GTab gtab) {
    return recover_m(qx, qy, digest_be, r_be, s_be, v, GlvMult<GTab>{gtab});
}

}  // namespace hd
