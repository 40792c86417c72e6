// hd_field.h -- secp256k1 base-field (mod p) and scalar-field (mod n)
// arithmetic for one message per 64-wide-wavefront lane.
//
// Representation: 8 x 32-bit little-endian limbs, always fully reduced
// (value in [0, p) or [0, n)).  The 256x256 products are operand-scanning
// schoolbook on v_mad_u64_u32 (each step is mad + 64-bit carry add); the
// reduction mod p uses 2^256 = 2^32 + 977 (mod p); the reduction mod n folds
// with c = 2^256 - n (129 bits) three times.  Rare carries / final subtractions
// are branches (taken with probability ~2^-220 on honest data), so the common
// path is straight-line VALU with no divergence.
//
// Inversion mod p and sqrt use the 255-squaring addition chains (p = 3 mod 4,
// sqrt = a^((p+1)/4)); inversion mod n uses a fixed 4-bit window over n-2
// (tests/test_devmath.py checks the chains' exponents and every operation
// against Python integers).
#pragma once
#include "hd_common.h"

namespace hd {

struct fe { uint32_t v[8]; };  // mod p
struct sc { uint32_t v[8]; };  // mod n

// p = 2^256 - 2^32 - 977
#define HD_P0 0xFFFFFC2Fu
#define HD_P1 0xFFFFFFFEu
// n (LE limbs)
#define HD_N0 0xD0364141u
#define HD_N1 0xBFD25E8Cu
#define HD_N2 0xAF48A03Bu
#define HD_N3 0xBAAEDCE6u
#define HD_N4 0xFFFFFFFEu
// c = 2^256 - n (LE limbs; c4 = 1)
#define HD_C0 0x2FC9BEBFu
#define HD_C1 0x402DA173u
#define HD_C2 0x50B75FC4u
#define HD_C3 0x45512319u

// ------------------------------------------------------------ 256-bit core
HD void mul_256(uint32_t t[16], const uint32_t a[8], const uint32_t b[8]) {
    // row 0
    {
        uint64_t c = 0;
        HD_UNROLL for (int j = 0; j < 8; j++) {
            uint64_t p = (uint64_t)a[0] * b[j] + c;
            t[j] = (uint32_t)p;
            c = p >> 32;
        }
        t[8] = (uint32_t)c;
    }
    HD_UNROLL for (int i = 1; i < 8; i++) {
        uint64_t c = 0;
        HD_UNROLL for (int j = 0; j < 8; j++) {
            uint64_t p = (uint64_t)a[i] * b[j] + t[i + j] + c;
            t[i + j] = (uint32_t)p;
            c = p >> 32;
        }
        t[i + 8] = (uint32_t)c;
    }
}

HD void sqr_256(uint32_t t[16], const uint32_t a[8]) {
    // off-diagonal products a_i a_j (i < j)
    t[0] = 0;
    {
        uint64_t c = 0;
        HD_UNROLL for (int j = 1; j < 8; j++) {
            uint64_t p = (uint64_t)a[0] * a[j] + c;
            t[j] = (uint32_t)p;
            c = p >> 32;
        }
        t[8] = (uint32_t)c;
    }
    HD_UNROLL for (int i = 1; i < 7; i++) {
        uint64_t c = 0;
        HD_UNROLL for (int j = i + 1; j < 8; j++) {
            uint64_t p = (uint64_t)a[i] * a[j] + t[i + j] + c;
            t[i + j] = (uint32_t)p;
            c = p >> 32;
        }
        t[i + 8] = (uint32_t)c;
    }
    t[15] = 0;
    // double
    t[15] = t[14] >> 31;
    HD_UNROLL for (int k = 14; k > 0; k--) t[k] = (t[k] << 1) | (t[k - 1] >> 31);
    t[0] = 0;  // t[0] was 0 before doubling
    // add the diagonal a_i^2
    uint64_t c = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        uint64_t p = (uint64_t)a[i] * a[i];
        c += (uint64_t)t[2 * i] + (uint32_t)p;
        t[2 * i] = (uint32_t)c;
        c >>= 32;
        c += (uint64_t)t[2 * i + 1] + (p >> 32);
        t[2 * i + 1] = (uint32_t)c;
        c >>= 32;
    }
}

// ------------------------------------------------------------- field mod p
HD void fe_clear(fe& r) { HD_UNROLL for (int i = 0; i < 8; i++) r.v[i] = 0; }
HD void fe_set_u32(fe& r, uint32_t x) { fe_clear(r); r.v[0] = x; }
HD bool fe_is_zero(const fe& a) {
    uint32_t o = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) o |= a.v[i];
    return o == 0;
}
HD bool fe_eq(const fe& a, const fe& b) {
    uint32_t o = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) o |= a.v[i] ^ b.v[i];
    return o == 0;
}
// big-endian word array (w[0] most significant) <-> limbs
HD void fe_from_be(fe& r, const uint32_t w[8]) { HD_UNROLL for (int i = 0; i < 8; i++) r.v[i] = w[7 - i]; }
HD void fe_to_be(uint32_t w[8], const fe& a) { HD_UNROLL for (int i = 0; i < 8; i++) w[i] = a.v[7 - i]; }

// a >= p ?
HD bool fe_ge_p(const uint32_t m[8]) {
    uint32_t hi = m[7] & m[6] & m[5] & m[4] & m[3] & m[2];
    return hi == 0xFFFFFFFFu && (m[1] == 0xFFFFFFFFu || (m[1] == HD_P1 && m[0] >= HD_P0));
}
// m -= p (as m + 0x1000003D1 mod 2^256); caller guarantees p <= m < 2^256
HD void fe_sub_p(uint32_t m[8]) {
    uint64_t c = (uint64_t)m[0] + 0x3D1u;
    m[0] = (uint32_t)c; c >>= 32;
    c += (uint64_t)m[1] + 1u;
    m[1] = (uint32_t)c; c >>= 32;
    HD_UNROLL for (int i = 2; i < 8; i++) { c += m[i]; m[i] = (uint32_t)c; c >>= 32; }
}

// r = t mod p for a 512-bit t
HD void fe_reduce(fe& r, const uint32_t t[16]) {
    uint32_t m[8];
    uint64_t c = (uint64_t)t[8] * 977u + t[0];
    m[0] = (uint32_t)c;
    c >>= 32;
    HD_UNROLL for (int i = 1; i < 8; i++) {
        c += (uint64_t)t[8 + i] * 977u + t[i];
        c += t[8 + i - 1];
        m[i] = (uint32_t)c;
        c >>= 32;
    }
    uint64_t top = c + t[15];  // < 2^34
    uint64_t x = top * 977u;
    c = (uint64_t)m[0] + (uint32_t)x;
    m[0] = (uint32_t)c; c >>= 32;
    c += (uint64_t)m[1] + (x >> 32) + (uint32_t)top;
    m[1] = (uint32_t)c; c >>= 32;
    c += (uint64_t)m[2] + (top >> 32);
    m[2] = (uint32_t)c; c >>= 32;
    HD_UNROLL for (int i = 3; i < 8; i++) { c += m[i]; m[i] = (uint32_t)c; c >>= 32; }
    if (c) {
        // value was >= 2^256: m is small (< 2^66); add 2^256 mod p
        uint64_t d = (uint64_t)m[0] + 0x3D1u;
        m[0] = (uint32_t)d; d >>= 32;
        d += (uint64_t)m[1] + 1u;
        m[1] = (uint32_t)d; d >>= 32;
        HD_UNROLL for (int i = 2; i < 8; i++) { d += m[i]; m[i] = (uint32_t)d; d >>= 32; }
    }
    if (fe_ge_p(m)) fe_sub_p(m);
    HD_UNROLL for (int i = 0; i < 8; i++) r.v[i] = m[i];
}

HD void fe_mul(fe& r, const fe& a, const fe& b) {
    uint32_t t[16];
    mul_256(t, a.v, b.v);
    fe_reduce(r, t);
}
HD void fe_sqr(fe& r, const fe& a) {
    uint32_t t[16];
    sqr_256(t, a.v);
    fe_reduce(r, t);
}
HD void fe_add(fe& r, const fe& a, const fe& b) {
    uint32_t s[8], d[8];
    uint64_t c = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) { c += (uint64_t)a.v[i] + b.v[i]; s[i] = (uint32_t)c; c >>= 32; }
    uint64_t e = (uint64_t)s[0] + 0x3D1u;
    d[0] = (uint32_t)e; e >>= 32;
    e += (uint64_t)s[1] + 1u;
    d[1] = (uint32_t)e; e >>= 32;
    HD_UNROLL for (int i = 2; i < 8; i++) { e += s[i]; d[i] = (uint32_t)e; e >>= 32; }
    bool sub = (c | e) != 0;  // a + b >= p
    HD_UNROLL for (int i = 0; i < 8; i++) r.v[i] = sub ? d[i] : s[i];
}
HD void fe_sub(fe& r, const fe& a, const fe& b) {
    uint32_t d[8];
    uint64_t br = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        uint64_t t = (uint64_t)a.v[i] - b.v[i] - br;
        d[i] = (uint32_t)t;
        br = t >> 63;
    }
    // if borrow: d += p  <=>  d -= 0x1000003D1 (mod 2^256)
    uint32_t k0 = br ? 0x3D1u : 0u, k1 = br ? 1u : 0u;
    uint64_t t = (uint64_t)d[0] - k0;
    r.v[0] = (uint32_t)t;
    uint64_t b2 = t >> 63;
    t = (uint64_t)d[1] - k1 - b2;
    r.v[1] = (uint32_t)t;
    b2 = t >> 63;
    HD_UNROLL for (int i = 2; i < 8; i++) {
        t = (uint64_t)d[i] - b2;
        r.v[i] = (uint32_t)t;
        b2 = t >> 63;
    }
}
HD void fe_neg(fe& r, const fe& a) {
    fe z;
    fe_clear(z);
    fe_sub(r, z, a);
}
HD void fe_cmov(fe& r, const fe& a, bool flag) {
    HD_UNROLL for (int i = 0; i < 8; i++) r.v[i] = flag ? a.v[i] : r.v[i];
}
HD void fe_sqr_n(fe& r, const fe& a, int n) {
    r = a;
    HD_NOUNROLL for (int i = 0; i < n; i++) fe_sqr(r, r);
}

// x^(2^223 - 1) and the shared prefix of the inversion / sqrt chains
// (the libsecp256k1 chain shape; exponents verified in tests).
struct FeChain { fe x2, x3, x22, x223; };
HD void fe_chain223(FeChain& c, const fe& a) {
    fe t, x6, x11, x44;
    fe_sqr(c.x2, a);
    fe_mul(c.x2, c.x2, a);            // 2^2 - 1
    fe_sqr(c.x3, c.x2);
    fe_mul(c.x3, c.x3, a);            // 2^3 - 1
    fe_sqr_n(t, c.x3, 3);
    fe_mul(x6, t, c.x3);              // 2^6 - 1
    fe_sqr_n(t, x6, 3);
    fe_mul(t, t, c.x3);               // 2^9 - 1
    fe_sqr_n(t, t, 2);
    fe_mul(x11, t, c.x2);             // 2^11 - 1
    fe_sqr_n(t, x11, 11);
    fe_mul(c.x22, t, x11);            // 2^22 - 1
    fe_sqr_n(t, c.x22, 22);
    fe_mul(x44, t, c.x22);            // 2^44 - 1
    fe_sqr_n(t, x44, 44);
    fe_mul(t, t, x44);                // 2^88 - 1
    fe_sqr_n(c.x223, t, 88);
    fe_mul(c.x223, c.x223, t);        // 2^176 - 1
    fe_sqr_n(c.x223, c.x223, 44);
    fe_mul(c.x223, c.x223, x44);      // 2^220 - 1
    fe_sqr_n(c.x223, c.x223, 3);
    fe_mul(c.x223, c.x223, c.x3);     // 2^223 - 1
}
// r = a^(p-2)
HD void fe_inv(fe& r, const fe& a) {
    FeChain c;
    fe_chain223(c, a);
    fe t;
    fe_sqr_n(t, c.x223, 23);
    fe_mul(t, t, c.x22);
    fe_sqr_n(t, t, 5);
    fe_mul(t, t, a);
    fe_sqr_n(t, t, 3);
    fe_mul(t, t, c.x2);
    fe_sqr_n(t, t, 2);
    fe_mul(r, t, a);
}
// r = a^((p+1)/4); returns true iff r^2 == a
HD bool fe_sqrt(fe& r, const fe& a) {
    FeChain c;
    fe_chain223(c, a);
    fe t;
    fe_sqr_n(t, c.x223, 23);
    fe_mul(t, t, c.x22);
    fe_sqr_n(t, t, 6);
    fe_mul(t, t, c.x2);
    fe_sqr(t, t);
    fe_sqr(r, t);
    fe_sqr(t, r);
    return fe_eq(t, a);
}

// ------------------------------------------------------------ scalar mod n
HD bool sc_is_zero(const sc& a) {
    uint32_t o = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) o |= a.v[i];
    return o == 0;
}
// m >= n ?  (m as 8 limbs)
HD bool sc_ge_n(const uint32_t m[8]) {
    const uint32_t N[8] = {HD_N0, HD_N1, HD_N2, HD_N3, HD_N4, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    // lexicographic compare from the top
    bool gt = false, lt = false;
    HD_UNROLL for (int i = 7; i >= 0; i--) {
        bool g = !lt && !gt && m[i] > N[i];
        bool l = !lt && !gt && m[i] < N[i];
        gt = gt || g;
        lt = lt || l;
    }
    return !lt;  // gt or equal
}
HD void sc_sub_n(uint32_t m[8]) {
    // m -= n  <=>  m += c (mod 2^256)
    const uint32_t C[8] = {HD_C0, HD_C1, HD_C2, HD_C3, 1u, 0u, 0u, 0u};
    uint64_t c = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) { c += (uint64_t)m[i] + C[i]; m[i] = (uint32_t)c; c >>= 32; }
}
// from big-endian words, reduced mod n (digest -> message scalar; the
// libsecp256k1 secp256k1_scalar_set_b32 with overflow ignored)
HD void sc_from_be_reduce(sc& r, const uint32_t w[8]) {
    uint32_t m[8];
    HD_UNROLL for (int i = 0; i < 8; i++) m[i] = w[7 - i];
    if (sc_ge_n(m)) sc_sub_n(m);
    HD_UNROLL for (int i = 0; i < 8; i++) r.v[i] = m[i];
}

// P[0 .. na+4] = a[0..na-1] * c  (c = 2^256 - n: 4 limbs + implicit c4 = 1)
template <int NA>
HD void mul_by_c(uint32_t* P, const uint32_t* a) {
    const uint32_t C[4] = {HD_C0, HD_C1, HD_C2, HD_C3};
    HD_UNROLL for (int k = 0; k < 5; k++) P[k] = 0;
    HD_UNROLL for (int i = 0; i < NA; i++) {
        uint64_t cy = 0;
        HD_UNROLL for (int j = 0; j < 4; j++) {
            uint64_t p = (uint64_t)a[i] * C[j] + P[i + j] + cy;
            P[i + j] = (uint32_t)p;
            cy = p >> 32;
        }
        uint64_t p = (uint64_t)a[i] + P[i + 4] + cy;  // c4 = 1
        P[i + 4] = (uint32_t)p;
        P[i + 5] = (uint32_t)(p >> 32);
    }
}

// r = t mod n for a 512-bit t (three folds with c, libsecp256k1
// scalar_reduce_512 shape)
HD void sc_reduce(sc& r, const uint32_t t[16]) {
    // stage 1: m (13 limbs) = t_lo + t_hi * c   (< 2^386)
    uint32_t P[13], m[13];
    mul_by_c<8>(P, t + 8);
    uint64_t cy = 0;
    HD_UNROLL for (int i = 0; i < 13; i++) {
        cy += (uint64_t)P[i] + (i < 8 ? t[i] : 0u);
        m[i] = (uint32_t)cy;
        cy >>= 32;
    }
    // stage 2: m2 (9 limbs) = m_lo + m_hi * c   (m_hi < 2^130 -> m2 < 2^260)
    uint32_t Q[10], m2[9];
    mul_by_c<5>(Q, m + 8);
    cy = 0;
    HD_UNROLL for (int i = 0; i < 9; i++) {
        cy += (uint64_t)Q[i] + (i < 8 ? m[i] : 0u);
        m2[i] = (uint32_t)cy;
        cy >>= 32;
    }
    // stage 3: r = m2_lo + m2[8] * c   (< 2^256 + 2^133)
    const uint32_t C5[5] = {HD_C0, HD_C1, HD_C2, HD_C3, 1u};
    uint32_t o[8];
    cy = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        uint64_t p = (uint64_t)m2[i] + cy;
        if (i < 5) p += (uint64_t)m2[8] * C5[i];
        o[i] = (uint32_t)p;
        cy = p >> 32;
    }
    if (cy) sc_sub_n(o);          // wrapped past 2^256: add c (o is small)
    if (sc_ge_n(o)) sc_sub_n(o);
    HD_UNROLL for (int i = 0; i < 8; i++) r.v[i] = o[i];
}

HD void sc_mul(sc& r, const sc& a, const sc& b) {
    uint32_t t[16];
    mul_256(t, a.v, b.v);
    sc_reduce(r, t);
}
HD void sc_sqr(sc& r, const sc& a) {
    uint32_t t[16];
    sqr_256(t, a.v);
    sc_reduce(r, t);
}
// r = n - a (0 -> 0)
HD void sc_neg(sc& r, const sc& a) {
    const uint32_t N[8] = {HD_N0, HD_N1, HD_N2, HD_N3, HD_N4, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    bool z = sc_is_zero(a);
    uint64_t br = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        uint64_t t = (uint64_t)N[i] - a.v[i] - br;
        r.v[i] = z ? 0u : (uint32_t)t;
        br = t >> 63;
    }
}

// r = a^(n-2) mod n: fixed 4-bit windows over the constant exponent; the
// 16-entry power table is indexed at run time (lives in scratch on device).
HD void sc_inv(sc& r, const sc& a) {
    // n - 2, little-endian 32-bit words
    const uint32_t E[8] = {0xD036413Fu, HD_N1, HD_N2, HD_N3, HD_N4, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    sc tab[16];
    HD_UNROLL for (int i = 0; i < 8; i++) tab[0].v[i] = 0;
    tab[0].v[0] = 1;
    tab[1] = a;
    HD_NOUNROLL for (int i = 2; i < 16; i++) sc_mul(tab[i], tab[i - 1], a);
    sc acc = tab[(E[7] >> 28) & 15];
    HD_NOUNROLL for (int j = 62; j >= 0; j--) {
        HD_NOUNROLL for (int k = 0; k < 4; k++) sc_sqr(acc, acc);
        uint32_t d = (E[j >> 3] >> ((j & 7) * 4)) & 15u;
        if (d) sc_mul(acc, acc, tab[d]);
    }
    r = acc;
}

}  // namespace hd
