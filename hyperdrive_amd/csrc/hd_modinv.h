// hd_modinv.h -- modular inversion by Bernstein-Yang divsteps ("safegcd",
// https://gcd.cr.yp.to/safegcd-20190413.pdf), constant-time form with
// 30-divstep jumps on signed 30-bit limbs.
//
// Why this shape on a 64-wide SIMD: every lane runs the same 20 x 30 divsteps
// with branch-free masks (no divergence), all arithmetic is native 32-bit
// (signed 32x32->64 products are single v_mad_i64_i32), and it replaces a
// ~320-multiplication Fermat chain (x^(m-2)) with ~14k simple instructions.
//
// Representation: value = sum v[i] 2^(30 i), 9 limbs; limbs 0..7 in [0, 2^30)
// when normalised, limb 8 carries the sign.  Inputs of 256 bits need at most
// 590 divsteps (the paper's bound); 20 x 30 = 600 are performed.
#pragma once
#include "hd_field.h"

namespace hd {

struct s30 { int32_t v[9]; };
struct ModInfo30 {
    s30 m;              // modulus (odd)
    uint32_t m_inv30;   // m^-1 mod 2^30
};

struct Trans2x2 { int32_t u, v, q, r; };


// 30 divsteps on the low 30 bits of f, g.  zeta = -(delta + 1/2).
// Returns the new zeta; t gets the transition matrix scaled by 2^30:
//   2^30 f' = u f + v g,   2^30 g' = q f + r g.
HD int32_t divsteps30(int32_t zeta, uint32_t f0, uint32_t g0, Trans2x2& t) {
    uint32_t u = 1, v = 0, q = 0, r = 1;
    uint32_t f = f0, g = g0;
    HD_UNROLL for (int i = 0; i < 30; i++) {
        // c1: zeta < 0 (delta > 0); c2: g odd
        uint32_t c1 = (uint32_t)(zeta >> 31);
        uint32_t c2 = 0u - (g & 1u);
        // x, y, z: f, u, v negated when delta > 0
        uint32_t x = (f ^ c1) - c1;
        uint32_t y = (u ^ c1) - c1;
        uint32_t z = (v ^ c1) - c1;
        // g odd: g += x (g - f or g + f), likewise for the matrix row
        g += x & c2;
        q += y & c2;
        r += z & c2;
        // delta > 0 and g odd: swap roles (f takes the old g)
        c1 &= c2;
        zeta = (int32_t)(((uint32_t)zeta ^ c1) - 1u);
        f += g & c1;
        u += q & c1;
        v += r & c1;
        g >>= 1;
        u <<= 1;
        v <<= 1;
    }
    t.u = (int32_t)u;
    t.v = (int32_t)v;
    t.q = (int32_t)q;
    t.r = (int32_t)r;
    return zeta;
}

// (d, e) <- t (d, e) / 2^30  (mod m), keeping d, e in (-2m, m)
HD void update_de30(s30& d, s30& e, const Trans2x2& t, const ModInfo30& mi) {
    const int32_t M30 = (int32_t)0x3FFFFFFF;
    const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
    // add m * [md, me] so that the low 30 bits of t [d, e] + m [md, me] vanish;
    // start md, me with corrections for negative d / e
    const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
    int32_t md = (u & sd) + (v & se);
    int32_t me = (q & sd) + (r & se);
    int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0];
    int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
    md -= (int32_t)((mi.m_inv30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)M30);
    me -= (int32_t)((mi.m_inv30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)M30);
    cd += (int64_t)mi.m.v[0] * md;
    ce += (int64_t)mi.m.v[0] * me;
    cd >>= 30;
    ce >>= 30;
    HD_UNROLL for (int i = 1; i < 9; i++) {
        const int32_t di = d.v[i], ei = e.v[i];
        cd += (int64_t)u * di + (int64_t)v * ei + (int64_t)mi.m.v[i] * md;
        ce += (int64_t)q * di + (int64_t)r * ei + (int64_t)mi.m.v[i] * me;
        d.v[i - 1] = (int32_t)cd & M30;
        cd >>= 30;
        e.v[i - 1] = (int32_t)ce & M30;
        ce >>= 30;
    }
    d.v[8] = (int32_t)cd;
    e.v[8] = (int32_t)ce;
}

// (f, g) <- t (f, g) / 2^30 (exact)
HD void update_fg30(s30& f, s30& g, const Trans2x2& t) {
    const int32_t M30 = (int32_t)0x3FFFFFFF;
    const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
    int64_t cf = (int64_t)u * f.v[0] + (int64_t)v * g.v[0];
    int64_t cg = (int64_t)q * f.v[0] + (int64_t)r * g.v[0];
    cf >>= 30;
    cg >>= 30;
    HD_UNROLL for (int i = 1; i < 9; i++) {
        const int32_t fi = f.v[i], gi = g.v[i];
        cf += (int64_t)u * fi + (int64_t)v * gi;
        cg += (int64_t)q * fi + (int64_t)r * gi;
        f.v[i - 1] = (int32_t)cf & M30;
        cf >>= 30;
        g.v[i - 1] = (int32_t)cg & M30;
        cg >>= 30;
    }
    f.v[8] = (int32_t)cf;
    g.v[8] = (int32_t)cg;
}

// d in (-2m, m), sign < 0 means negate: result in [0, m)
HD void normalize30(s30& d, int32_t sign, const ModInfo30& mi) {
    const int32_t M30 = (int32_t)0x3FFFFFFF;
    int32_t cond_add = d.v[8] >> 31;
    HD_UNROLL for (int i = 0; i < 9; i++) d.v[i] += mi.m.v[i] & cond_add;
    const int32_t cond_neg = sign >> 31;
    HD_UNROLL for (int i = 0; i < 9; i++) d.v[i] = (d.v[i] ^ cond_neg) - cond_neg;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        d.v[i + 1] += d.v[i] >> 30;
        d.v[i] &= M30;
    }
    cond_add = d.v[8] >> 31;
    HD_UNROLL for (int i = 0; i < 9; i++) d.v[i] += mi.m.v[i] & cond_add;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        d.v[i + 1] += d.v[i] >> 30;
        d.v[i] &= M30;
    }
}

// x <- x^-1 mod m (x in [0, m); 0 maps to 0)
HD void modinv30(s30& x, const ModInfo30& mi) {
    s30 d, e, f = mi.m, g = x;
    HD_UNROLL for (int i = 0; i < 9; i++) { d.v[i] = 0; e.v[i] = 0; }
    e.v[0] = 1;
    int32_t zeta = -1;
    HD_NOUNROLL for (int it = 0; it < 20; it++) {
        Trans2x2 t;
        zeta = divsteps30(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
        update_de30(d, e, t, mi);
        update_fg30(f, g, t);
#ifdef __HIP_DEVICE_COMPILE__
        // Once g = 0 further divsteps only halve g = 0 and leave d fixed
        // (their matrix is diag(2^30, 1) / 2^30), so a wavefront whose lanes
        // all reached g = 0 stops: random 256-bit inputs need ~531 divsteps
        // (the worst of 64 lanes ~550, 19 batches) of the 590 bound.
        if (it >= 16) {
            uint32_t nz = 0;
            HD_UNROLL for (int i = 0; i < 9; i++) nz |= (uint32_t)g.v[i];
            if (__ballot(nz != 0) == 0ull) break;
        }
#endif
    }
    normalize30(d, f.v[8], mi);
    x = d;
}

// 8 little-endian 32-bit words (value < 2^256) <-> signed-30 limbs
HD void s30_from_le(s30& r, const uint32_t w[8]) {
    HD_UNROLL for (int i = 0; i < 9; i++) {
        const int bit = 30 * i, word = bit >> 5, off = bit & 31;
        uint32_t v = word < 8 ? (w[word] >> off) : 0u;
        if (off > 2 && word + 1 < 8) v |= w[word + 1] << (32 - off);
        r.v[i] = (int32_t)(v & 0x3FFFFFFFu);
    }
}
HD void s30_to_le(uint32_t w[8], const s30& a) {  // a in [0, 2^256), limbs normalised
    HD_UNROLL for (int k = 0; k < 8; k++) w[k] = 0;
    HD_UNROLL for (int i = 0; i < 9; i++) {
        const int bit = 30 * i, word = bit >> 5, off = bit & 31;
        const uint32_t v = (uint32_t)a.v[i];
        if (word < 8) w[word] |= v << off;
        if (off > 2 && word + 1 < 8) w[word + 1] |= v >> (32 - off);
    }
}

// secp256k1 group order n and field prime p in signed-30 form
HD void modinfo_n(ModInfo30& mi) {
    const int32_t N30[9] = {0x10364141, 0x3F497A33, 0x348A03BB, 0x2BB739AB, -0x146, 0, 0, 0, 65536};
    HD_UNROLL for (int i = 0; i < 9; i++) mi.m.v[i] = N30[i];
    mi.m_inv30 = 0x2A774EC1u;
}
HD void modinfo_p(ModInfo30& mi) {
    const int32_t P30[9] = {-0x3D1, -4, 0, 0, 0, 0, 0, 0, 65536};
    HD_UNROLL for (int i = 0; i < 9; i++) mi.m.v[i] = P30[i];
    mi.m_inv30 = 0x2DDACACFu;
}

// scalar inverse mod n
HD void sc_inv_divsteps(sc& r, const sc& a) {
    ModInfo30 mi;
    modinfo_n(mi);
    s30 x;
    s30_from_le(x, a.v);
    modinv30(x, mi);
    s30_to_le(r.v, x);
}

// field inverse mod p (result canonical)
HD void fe_inv_divsteps(fe& r, const fe& a) {
    fe t = a;
    fe_normalize(t);
    uint32_t w[8];
    fe_to_le(w, t);
    ModInfo30 mi;
    modinfo_p(mi);
    s30 x;
    s30_from_le(x, w);
    modinv30(x, mi);
    s30_to_le(w, x);
    fe_from_le(r, w);
}

}  // namespace hd
