// hd_field.h -- secp256k1 base-field (mod p) and scalar-field (mod n)
// arithmetic for one message per 64-wide-wavefront lane.
//
// Base field: radix 2^26 x 10 limbs, lazily reduced (see the field section):
// a product column is a chain of v_mad_u64_u32 into one 64-bit accumulator, so
// the multiply needs no carry flags (a VCC carry chain costs s_nop hazards on
// gfx950) and no operand moves; additions are 10 plain v_add_u32.
// Scalar field: 8 x 32-bit limbs, fully reduced, operand-scanning schoolbook;
// the reduction mod n folds with c = 2^256 - n (129 bits) three times.  Rare
// carries / final subtractions are branches (taken with probability ~2^-220
// on honest data), so the common path has no divergence.
//
// Inversion mod p and sqrt use the 255-squaring addition chains (p = 3 mod 4,
// sqrt = a^((p+1)/4)); inversion mod n uses a fixed 4-bit window over n-2
// (tests/test_devmath.py checks the chains' exponents and every operation
// against Python integers).
#pragma once
#include "hd_common.h"

namespace hd {

struct fe { uint32_t n[10]; };  // mod p, radix 2^26 (see below)
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
// Radix 2^26, 10 limbs, lazily reduced.  Value = sum n[i] 2^(26 i).
// Bounds (checked in tests/test_devmath.py and asserted by construction):
//   T  "tight" (output of mul / sqr / norm_weak): n[0..8] < 2^26 + 2^24,
//      n[9] < 2^22 + 1 -- value < 2^256 + 2^230, NOT necessarily < p.
//   L  "loose" (valid mul / sqr input):            n[0..8] < 2^30, n[9] < 2^25.5.
// With L inputs every 64-bit product column sum stays < 2^63.3, so a column is
// a chain of v_mad_u64_u32 into one 64-bit accumulator (no carry flags, no
// moves).  fe_sub(a, b) = a + K p - b limb-wise needs b <= K p limb-wise; the
// caller picks K (4 for a T subtrahend).  Exact tests (zero, equality, parity,
// serialisation) go through fe_normalize (canonical, < p).
#define HD_M26 0x3FFFFFFu
#define HD_M22 0x3FFFFFu
// p limbs: 0x3FFFC2F, 0x3FFFFBF, 7 x 0x3FFFFFF, 0x3FFFFF
#define HD_FP0 0x3FFFC2Fu
#define HD_FP1 0x3FFFFBFu

HD void fe_clear(fe& r) { HD_UNROLL for (int i = 0; i < 10; i++) r.n[i] = 0; }
HD void fe_set_u32(fe& r, uint32_t x) { fe_clear(r); r.n[0] = x & HD_M26; r.n[1] = x >> 26; }

// 8 little-endian 32-bit words (value < 2^256) -> limbs (T, not reduced)
HD void fe_from_le(fe& r, const uint32_t w[8]) {
    HD_UNROLL for (int i = 0; i < 10; i++) {
        const int bit = 26 * i, word = bit >> 5, off = bit & 31;
        uint32_t v = w[word] >> off;
        if (off > 6 && word + 1 < 8) v |= w[word + 1] << (32 - off);
        r.n[i] = v & (i == 9 ? HD_M22 : HD_M26);
    }
}
HD void fe_from_be(fe& r, const uint32_t be[8]) {
    uint32_t w[8];
    HD_UNROLL for (int i = 0; i < 8; i++) w[i] = be[7 - i];
    fe_from_le(r, w);
}

// a + K p - b, limb-wise (no carries).  Requires b[i] <= K p[i].
template <int K>
HD void fe_sub_k(fe& r, const fe& a, const fe& b) {
    r.n[0] = a.n[0] + (uint32_t)K * HD_FP0 - b.n[0];
    r.n[1] = a.n[1] + (uint32_t)K * HD_FP1 - b.n[1];
    HD_UNROLL for (int i = 2; i < 9; i++) r.n[i] = a.n[i] + (uint32_t)K * HD_M26 - b.n[i];
    r.n[9] = a.n[9] + (uint32_t)K * HD_M22 - b.n[9];
}
HD void fe_sub(fe& r, const fe& a, const fe& b) { fe_sub_k<4>(r, a, b); }
HD void fe_neg(fe& r, const fe& a) { fe z; fe_clear(z); fe_sub_k<4>(r, z, a); }
HD void fe_add(fe& r, const fe& a, const fe& b) { HD_UNROLL for (int i = 0; i < 10; i++) r.n[i] = a.n[i] + b.n[i]; }
HD void fe_mul_int(fe& r, const fe& a, uint32_t k) { HD_UNROLL for (int i = 0; i < 10; i++) r.n[i] = a.n[i] * k; }
HD void fe_cmov(fe& r, const fe& a, bool flag) {
    HD_UNROLL for (int i = 0; i < 10; i++) r.n[i] = flag ? a.n[i] : r.n[i];
}

// Weak normalisation: any limbs < 2^32 (top < 2^31) -> T.
HD void fe_norm_weak(fe& r) {
    uint32_t c = 0;
    HD_UNROLL for (int i = 0; i < 9; i++) {
        uint32_t t = r.n[i] + c;  // < 2^32: limbs < 2^32 - 2^6 in every caller
        r.n[i] = t & HD_M26;
        c = t >> 26;
    }
    uint32_t t9 = r.n[9] + c;
    r.n[9] = t9 & HD_M22;
    uint32_t u = t9 >> 22;  // weight 2^256 == 0x1000003D1 (mod p)
    uint64_t x = (uint64_t)u * 0x3D1u + r.n[0];
    r.n[0] = (uint32_t)x & HD_M26;
    uint64_t y = (x >> 26) + ((uint64_t)u << 6) + r.n[1];
    r.n[1] = (uint32_t)y & HD_M26;
    r.n[2] += (uint32_t)(y >> 26);
}

// Canonical form: every limb < 2^26, value < p.  Input: L (or anything
// norm_weak accepts).
HD void fe_normalize(fe& r) {
    fe_norm_weak(r);
    uint32_t c = 0;
    HD_UNROLL for (int i = 0; i < 9; i++) {
        uint32_t t = r.n[i] + c;
        r.n[i] = t & HD_M26;
        c = t >> 26;
    }
    r.n[9] += c;
    // value >= 2^256 (top > 22 bits) or p <= value < 2^256: subtract p once
    uint32_t mid = r.n[2] & r.n[3] & r.n[4] & r.n[5] & r.n[6] & r.n[7] & r.n[8];
    bool ge = (r.n[9] >> 22) != 0 ||
              (r.n[9] == HD_M22 && mid == HD_M26 &&
               (r.n[1] > HD_FP1 || (r.n[1] == HD_FP1 && r.n[0] >= HD_FP0)));
    if (ge) {
        // r - p == r + 0x1000003D1 - 2^256
        uint32_t t = r.n[0] + 0x3D1u;
        r.n[0] = t & HD_M26;
        t = r.n[1] + 0x40u + (t >> 26);  // 2^32 = 2^6 * 2^26
        r.n[1] = t & HD_M26;
        c = t >> 26;
        HD_UNROLL for (int i = 2; i < 9; i++) {
            t = r.n[i] + c;
            r.n[i] = t & HD_M26;
            c = t >> 26;
        }
        r.n[9] = (r.n[9] + c) & HD_M22;
    }
}
HD void fe_to_le(uint32_t w[8], const fe& a) {  // a canonical
    HD_UNROLL for (int k = 0; k < 8; k++) w[k] = 0;
    HD_UNROLL for (int i = 0; i < 10; i++) {
        const int bit = 26 * i, word = bit >> 5, off = bit & 31;
        w[word] |= a.n[i] << off;
        if (off > 6 && word + 1 < 8) w[word + 1] |= a.n[i] >> (32 - off);
    }
}
HD void fe_to_be(uint32_t be[8], const fe& a) {  // a canonical
    uint32_t w[8];
    fe_to_le(w, a);
    HD_UNROLL for (int i = 0; i < 8; i++) be[i] = w[7 - i];
}
HD bool fe_is_zero(const fe& a) {
    fe t = a;
    fe_normalize(t);
    uint32_t o = 0;
    HD_UNROLL for (int i = 0; i < 10; i++) o |= t.n[i];
    return o == 0;
}
HD bool fe_is_odd(const fe& a) {
    fe t = a;
    fe_normalize(t);
    return t.n[0] & 1u;
}
HD bool fe_eq(const fe& a, const fe& b) {  // b must be T
    fe d;
    fe_sub_k<4>(d, a, b);
    return fe_is_zero(d);
}

// Product scanning with the high column folded in as it is produced: column
// k (weight 2^(26k)) and column k+10 (weight 2^(26k) * 2^260, 2^260 ==
// 0x400 * 2^26 + 0x3D10 mod p) are accumulated together, so only three
// 64-bit accumulators are live (low register pressure -> more waves/SIMD).
// Inputs L (limbs < 2^30, top limb < 2^25.5); output T.
template <bool SQR>
HD void fe_mul_impl(fe& out, const fe& a, const fe& b) {
    fe r;               // out may alias a or b
    uint64_t chi = 0;   // carry of the high columns
    uint64_t clo = 0;   // carry of the low columns
    uint64_t pend = 0;  // h_{k-1} * 0x400 (< 2^36), owed to column k
    HD_UNROLL for (int k = 0; k < 10; k++) {
        uint64_t d = chi;
        HD_UNROLL for (int i = k + 1; i < 10; i++) {
            const int j = k + 10 - i;
            if (SQR) {
                if (i < j) d += (uint64_t)(a.n[i] << 1) * a.n[j];
                else if (i == j) d += (uint64_t)a.n[i] * a.n[i];
            } else {
                d += (uint64_t)a.n[i] * b.n[j];
            }
        }
        const uint32_t hk = (uint32_t)d & HD_M26;
        chi = d >> 26;
        uint64_t c = clo + pend + (uint64_t)hk * 0x3D10u;
        HD_UNROLL for (int i = 0; i <= k; i++) {
            const int j = k - i;
            if (SQR) {
                if (i < j) c += (uint64_t)(a.n[i] << 1) * a.n[j];
                else if (i == j) c += (uint64_t)a.n[i] * a.n[i];
            } else {
                c += (uint64_t)a.n[i] * b.n[j];
            }
        }
        pend = (uint64_t)hk << 10;
        r.n[k] = (uint32_t)c & HD_M26;
        clo = c >> 26;
    }
    // bits >= 2^256: r9's top 4 bits, the low carry and the last fold at 2^260
    // (chi is 0: top limbs < 2^25.5 keep the highest column < 2^52)
    uint64_t u = ((clo + pend) << 4) + (r.n[9] >> 22);
    r.n[9] &= HD_M22;
    uint64_t x = u * 0x3D1u + r.n[0];
    r.n[0] = (uint32_t)x & HD_M26;
    uint64_t y = (x >> 26) + (u << 6) + r.n[1];
    r.n[1] = (uint32_t)y & HD_M26;
    r.n[2] += (uint32_t)(y >> 26);
    out = r;
}
HD void fe_mul(fe& r, const fe& a, const fe& b) { fe_mul_impl<false>(r, a, b); }
HD void fe_sqr(fe& r, const fe& a) { fe_mul_impl<true>(r, a, a); }
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
// r = a^(p-2) (T)
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
// r = a^((p+1)/4) (T); returns true iff r^2 == a (mod p)
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
    fe an = a;
    fe_norm_weak(an);
    return fe_eq(t, an);
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
