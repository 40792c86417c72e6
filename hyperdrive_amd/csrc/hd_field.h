// hd_field.h -- secp256k1 base-field (mod p) and scalar-field (mod n)
// arithmetic for one message per 64-wide-wavefront lane.
//
// Base field: radix 2^29 x 9 limbs, lazily reduced (see the field section):
// a product column is a chain of v_mad_u64_u32 into one 64-bit accumulator, so
// the multiply needs no carry flags and no operand moves; additions are 9
// plain v_add_u32.
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
// 96-bit column accumulator (acc, hi) += a * b.  On the device this is one
// v_mad_u64_u32 whose carry-out lands in VCC plus one v_addc_co_u32 that adds
// it to the third word: the C formulation (a 64-bit product plus two 32-bit
// addends) compiles to a mad, a 64-bit add and register moves to build
// {x, 0} operand pairs, about twice the cycles per product.
HD void macc96(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(HD_NO_MACC_ASM)
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+v"(acc), "+v"(hi)
        : "v"(a), "v"(b)
        : "vcc");
#else
    const uint64_t p = (uint64_t)a * b;
    const uint64_t s = acc + p;
    hi += s < p ? 1u : 0u;
    acc = s;
#endif
}
// next column: (acc, hi) >>= 32
HD void col96_shift(uint64_t& acc, uint32_t& hi) {
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
}

// t = a b, product scanning (one 96-bit accumulator per column)
HD void mul_256(uint32_t t[16], const uint32_t a[8], const uint32_t b[8]) {
    uint64_t acc = 0;
    uint32_t hi = 0;
    HD_UNROLL for (int k = 0; k < 15; k++) {
        HD_UNROLL for (int i = 0; i < 8; i++) {
            const int j = k - i;
            if (j >= 0 && j < 8) macc96(acc, hi, a[i], b[j]);
        }
        t[k] = (uint32_t)acc;
        col96_shift(acc, hi);
    }
    t[15] = (uint32_t)acc;
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
// Radix 2^29, 9 limbs, lazily reduced.  Value = sum n[i] 2^(29 i) (261 bits
// of room for a 256-bit field).
//
// Why 2^29 x 9 on gfx950: a 26x26..29x29-bit partial product plus a 64-bit
// accumulate is ONE v_mad_u64_u32 (measured 4.3 cycles per wave-instruction,
// scripts/valu_probe.hip), the most expensive instruction of the kernel, and
// 9 limbs need 81 of them per product where 10 x 26-bit limbs need 100.  A
// column of at most 8 full products of < 2^61 each still fits the 64-bit
// accumulator, so no carry flags are ever needed (VCC carry chains cost
// VOP3 issue + s_nop hazards on gfx950).
//
// Limb classes (inclusive per-limb maxima; M = 2^29 - 1, M24 = 2^24 - 1):
//   T  "tight": n[0..7] <= M except n[2] <= M + 2^17, n[8] <= M24.  Every
//      fe_mul / fe_sqr / fe_norm_weak output is T; value < 2^256 + 2^75.
//   kT: the limb-wise sum of k tight values (fe_add, fe_mul_int, fe_sub_k).
// fe_mul(a, b) is exact for max(a) * max(b) <= 7.9 T^2 limb-wise (e.g. T x 7T,
// 2T x 3T); fe_sub_k<K>(a, b) = a + K p - b needs b <= K p limb-wise (K = 2
// for a T subtrahend).  Exact tests (zero, equality, parity, serialisation)
// go through fe_normalize (canonical, < p).
//
// Host test builds define HD_BOUNDS: every fe then carries per-limb upper
// bounds (b[]) that each operation propagates by interval arithmetic and
// checks against its precondition, so one run of a formula on the host
// certifies its limb bounds for ALL inputs of the declared classes
// (tests/test_field_bounds.py).  Device builds carry no bounds.
#define HD_M29 0x1FFFFFFFu
#define HD_M24 0xFFFFFFu
// p limbs: 0x1FFFFC2F, 0x1FFFFFF7, 6 x 0x1FFFFFFF, 0xFFFFFF
#define HD_FP0 0x1FFFFC2Fu
#define HD_FP1 0x1FFFFFF7u
#define HD_FE_T2 (HD_M29 + (1u << 17))   // T bound of limb 2

#if defined(HD_BOUNDS) && !defined(__HIP_DEVICE_COMPILE__)
#define HD_BOUND_CHECKS 1
#define HD_B(...) __VA_ARGS__
extern "C" void hd_bound_fail(const char* what, int line);
#define HD_BREQ(cond, what)                              \
    do {                                                 \
        if (!(cond)) hd_bound_fail(what, __LINE__);      \
    } while (0)
#else
#define HD_B(...)
#define HD_BREQ(cond, what) \
    do {                    \
    } while (0)
#endif

struct fe {
    uint32_t n[9];
    HD_B(uint64_t b[9];)
};

HD uint32_t fe_p_limb(int i) { return i == 0 ? HD_FP0 : i == 1 ? HD_FP1 : i == 8 ? HD_M24 : HD_M29; }
HD uint32_t fe_t_limb(int i) { return i == 2 ? HD_FE_T2 : i == 8 ? HD_M24 : HD_M29; }

#ifdef HD_BOUND_CHECKS
HD void fe_bound_exact(fe& r) { for (int i = 0; i < 9; i++) r.b[i] = r.n[i]; }
HD void fe_bound_T(fe& r) { for (int i = 0; i < 9; i++) r.b[i] = fe_t_limb(i); }
HD void fe_bound_check_values(const fe& a) {
    for (int i = 0; i < 9; i++) HD_BREQ(a.n[i] <= a.b[i], "limb exceeds its tracked bound");
}
HD void fe_require_T(const fe& a, const char* what) {
    for (int i = 0; i < 9; i++) HD_BREQ(a.b[i] <= fe_t_limb(i), what);
}
#define HD_REQUIRE_T(a, what) fe_require_T(a, what)
#else
#define HD_REQUIRE_T(a, what) \
    do {                      \
    } while (0)
#endif

// One v_mad_u64_u32: a * b + c.  The empty asm makes the result opaque, so
// the compiler keeps the accumulation chain exactly as written (left alone,
// it re-associates product scanning into operand scanning plus a 64-bit add
// per column -- 30 % more cycles, measured).
HD uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
    uint64_t r = (uint64_t)a * b + c;
#if defined(__HIP_DEVICE_COMPILE__) && !defined(HD_NO_LAUNDER)
    asm("" : "+v"(r));
#endif
    return r;
}
// a register copy the compiler cannot see through (keeps a constant multiplier
// in a VGPR instead of strength-reducing a * 256 into a 64-bit shift + add)
HD uint32_t opaque_u32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(HD_NO_LAUNDER)
    asm("" : "+v"(x));
#endif
    return x;
}

HD void fe_clear(fe& r) {
    HD_UNROLL for (int i = 0; i < 9; i++) r.n[i] = 0;
    HD_B(fe_bound_exact(r);)
}
HD void fe_set_u32(fe& r, uint32_t x) {  // x < 2^29
    fe_clear(r);
    r.n[0] = x;
    HD_B(fe_bound_exact(r);)
}

// 8 little-endian 32-bit words (value < 2^256) -> limbs (canonical layout, T)
HD void fe_from_le(fe& r, const uint32_t w[8]) {
    HD_UNROLL for (int i = 0; i < 9; i++) {
        const int bit = 29 * i, word = bit >> 5, off = bit & 31;
        uint32_t v = w[word] >> off;
        if (off > 3 && word + 1 < 8) v |= w[word + 1] << (32 - off);
        r.n[i] = v & (i == 8 ? HD_M24 : HD_M29);
    }
    HD_B(for (int i = 0; i < 9; i++) r.b[i] = i == 8 ? HD_M24 : HD_M29;)
}
HD void fe_from_be(fe& r, const uint32_t be[8]) {
    uint32_t w[8];
    HD_UNROLL for (int i = 0; i < 8; i++) w[i] = be[7 - i];
    fe_from_le(r, w);
}

// a + K p - b, limb-wise (no carries).  Requires b[i] <= K p[i].
template <int K>
HD void fe_sub_k(fe& r, const fe& a, const fe& b) {
#ifdef HD_BOUND_CHECKS
    fe_bound_check_values(a);
    fe_bound_check_values(b);
    uint64_t nb[9];
    for (int i = 0; i < 9; i++) {
        HD_BREQ(b.b[i] <= (uint64_t)K * fe_p_limb(i), "fe_sub_k: subtrahend exceeds K p");
        nb[i] = a.b[i] + (uint64_t)K * fe_p_limb(i);
        HD_BREQ(nb[i] < (1ull << 32), "fe_sub_k: limb overflow");
    }
#endif
    HD_UNROLL for (int i = 0; i < 9; i++) r.n[i] = a.n[i] + (uint32_t)K * fe_p_limb(i) - b.n[i];
    HD_B(for (int i = 0; i < 9; i++) r.b[i] = nb[i];)
}
HD void fe_sub(fe& r, const fe& a, const fe& b) { fe_sub_k<2>(r, a, b); }
// 2p - a (a tight): the result is 2T
HD void fe_neg(fe& r, const fe& a) {
    fe z;
    fe_clear(z);
    fe_sub_k<2>(r, z, a);
}
HD void fe_add(fe& r, const fe& a, const fe& b) {
#ifdef HD_BOUND_CHECKS
    fe_bound_check_values(a);
    fe_bound_check_values(b);
    uint64_t nb[9];
    for (int i = 0; i < 9; i++) {
        nb[i] = a.b[i] + b.b[i];
        HD_BREQ(nb[i] < (1ull << 32), "fe_add: limb overflow");
    }
#endif
    HD_UNROLL for (int i = 0; i < 9; i++) r.n[i] = a.n[i] + b.n[i];
    HD_B(for (int i = 0; i < 9; i++) r.b[i] = nb[i];)
}
HD void fe_mul_int(fe& r, const fe& a, uint32_t k) {
#ifdef HD_BOUND_CHECKS
    fe_bound_check_values(a);
    uint64_t nb[9];
    for (int i = 0; i < 9; i++) {
        nb[i] = a.b[i] * k;
        HD_BREQ(nb[i] < (1ull << 32), "fe_mul_int: limb overflow");
    }
#endif
    HD_UNROLL for (int i = 0; i < 9; i++) r.n[i] = a.n[i] * k;
    HD_B(for (int i = 0; i < 9; i++) r.b[i] = nb[i];)
}
HD void fe_cmov(fe& r, const fe& a, bool flag) {
    HD_UNROLL for (int i = 0; i < 9; i++) r.n[i] = flag ? a.n[i] : r.n[i];
    HD_B(for (int i = 0; i < 9; i++) r.b[i] = r.b[i] > a.b[i] ? r.b[i] : a.b[i];)
}

// Weak normalisation: limbs <= 2^32 - 9 -> T.  All 32-bit arithmetic.
HD void fe_norm_weak(fe& r) {
#ifdef HD_BOUND_CHECKS
    fe_bound_check_values(r);
    for (int i = 0; i < 9; i++) HD_BREQ(r.b[i] <= 0xFFFFFFF7ull, "fe_norm_weak: input limb too large");
#endif
    uint32_t c = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        const uint32_t t = r.n[i] + c;
        r.n[i] = t & HD_M29;
        c = t >> 29;
    }
    const uint32_t t8 = r.n[8] + c;
    r.n[8] = t8 & HD_M24;
    const uint32_t u = t8 >> 24;  // weight 2^256 == 0x1000003D1 (mod p); u < 2^8 + 1
    const uint32_t x = u * 977u + r.n[0];
    r.n[0] = x & HD_M29;
    const uint32_t y = (x >> 29) + (u << 3) + r.n[1];  // 2^32 = 8 * 2^29
    r.n[1] = y & HD_M29;
    r.n[2] += y >> 29;  // <= 1
    HD_B(fe_bound_T(r); r.b[2] = HD_M29 + 1;)
}

// Canonical form: every limb <= M29 (top <= M24), value < p.
HD void fe_normalize(fe& r) {
    fe_norm_weak(r);
    uint32_t c = 0;
    HD_UNROLL for (int i = 2; i < 8; i++) {
        const uint32_t t = r.n[i] + c;
        r.n[i] = t & HD_M29;
        c = t >> 29;
    }
    r.n[8] += c;  // <= 2^24: value < 2^256 + 2^233
    // value >= p  <=>  (top > M24) or (limbs 2..8 at their maxima and (n1, n0) >= (p1, p0))
    uint32_t mid = r.n[2] & r.n[3] & r.n[4] & r.n[5] & r.n[6] & r.n[7];
    bool ge = (r.n[8] >> 24) != 0 ||
              (r.n[8] == HD_M24 && mid == HD_M29 &&
               (r.n[1] > HD_FP1 || (r.n[1] == HD_FP1 && r.n[0] >= HD_FP0)));
    if (ge) {
        // r - p == r + 0x1000003D1 - 2^256
        uint32_t t = r.n[0] + 977u;
        r.n[0] = t & HD_M29;
        t = r.n[1] + 8u + (t >> 29);
        r.n[1] = t & HD_M29;
        c = t >> 29;
        HD_UNROLL for (int i = 2; i < 8; i++) {
            t = r.n[i] + c;
            r.n[i] = t & HD_M29;
            c = t >> 29;
        }
        r.n[8] = (r.n[8] + c) & HD_M24;
    }
    HD_B(for (int i = 0; i < 9; i++) r.b[i] = i == 8 ? HD_M24 : HD_M29;)
}
HD void fe_to_le(uint32_t w[8], const fe& a) {  // a canonical
    HD_UNROLL for (int k = 0; k < 8; k++) w[k] = 0;
    HD_UNROLL for (int i = 0; i < 9; i++) {
        const int bit = 29 * i, word = bit >> 5, off = bit & 31;
        w[word] |= a.n[i] << off;
        if (off > 3 && word + 1 < 8) w[word + 1] |= a.n[i] >> (32 - off);
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
    HD_UNROLL for (int i = 0; i < 9; i++) o |= t.n[i];
    return o == 0;
}
HD bool fe_is_odd(const fe& a) {
    fe t = a;
    fe_normalize(t);
    return t.n[0] & 1u;
}
HD bool fe_eq(const fe& a, const fe& b) {  // b <= 2p limb-wise (T)
    fe d;
    fe_sub_k<2>(d, a, b);
    return fe_is_zero(d);
}

#ifdef HD_BOUND_CHECKS
// Interval image of fe_mul_impl: per-limb maxima of the output, and a check
// that no 64-bit column accumulator can overflow for ANY inputs within the
// input bounds.  Mirrors the device algorithm step by step (every step is
// monotone in its inputs, so upper bounds propagate).
static void fe_mul_bounds(uint64_t* ob, const uint64_t* A, const uint64_t* B) {
    typedef unsigned __int128 u128;
    const u128 LIM = (u128)1 << 64, W32 = ((u128)1 << 32) - 1;
    u128 dhi = 0, clo = 0, c = 0, hprev = 0;
    uint64_t r[9];
    for (int k = 0; k < 9; k++) {
        u128 d = k > 0 ? dhi * 8u : 0;
        for (int i = k + 1; i < 9; i++) d += (u128)A[i] * B[k + 9 - i];
        HD_BREQ(d < LIM, "fe_mul: high column overflow");
        const u128 hk = d < W32 ? d : W32;
        dhi = d >> 32;
        c = clo + hk * 0x7A20u + (k > 0 ? hprev * 256u : 0);
        for (int i = 0; i <= k; i++) c += (u128)A[i] * B[k - i];
        HD_BREQ(c < LIM, "fe_mul: low column overflow");
        r[k] = c > HD_M29 ? HD_M29 : (uint64_t)c;
        clo = c >> 29;
        hprev = hk;
    }
    HD_BREQ(dhi == 0, "fe_mul: carry out of the top column");
    const u128 u = (c >> 24) + (hprev << 13);
    HD_BREQ(u < ((u128)1 << 48), "fe_mul: final fold too large");
    const u128 ulo = u < W32 ? u : W32, uhi = u >> 32;
    const u128 f0 = ulo * 977u + r[0];
    HD_BREQ(f0 < LIM, "fe_mul: fold overflow");
    const u128 f1 = (f0 >> 29) + r[1] + uhi * 7816u + (u << 3);
    HD_BREQ(f1 < LIM && (f1 >> 29) < ((u128)1 << 32), "fe_mul: fold overflow");
    for (int i = 0; i < 9; i++) ob[i] = r[i];
    ob[0] = HD_M29;
    ob[1] = HD_M29;
    ob[2] = r[2] + (uint64_t)(f1 >> 29);
    ob[8] = HD_M24;
    for (int i = 0; i < 9; i++) HD_BREQ(ob[i] <= fe_t_limb(i), "fe_mul: output not tight");
}
#endif

// A constant multiplier in an SGPR (the VOP3 mad reads one scalar operand):
// no per-product v_mov to materialise it in a VGPR.
HD uint32_t opaque_s32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(HD_NO_LAUNDER)
    asm("" : "+s"(x));
#endif
    return x;
}

// Product scanning with the high half folded in as it is produced: column k
// (weight 2^(29k)) and column k+9 (weight 2^(29k) 2^261, 2^261 == 2^8 2^29 +
// 0x7A20 mod p) are accumulated side by side, so only two 64-bit accumulator
// chains are live.
//  * A high column d is split at its register boundary, not at 29 bits:
//    hk = d mod 2^32 adds hk * 0x7A20 to column k and hk * 2^8 to column
//    k+1, and d >> 32 (weight 2^32 2^(29(k+9)) = 2^3 2^(29(k+10))) enters the
//    next high column as one mad by 8.  The split costs no instruction
//    (mask + 64-bit shift before).
//  * A low column c leaves c mod 2^29 as the output limb and c >> 29 as the
//    next column's carry.
//  * Column 8's accumulator and the top high part fold at weight 2^256:
//    u = (c8 >> 24) + h8 2^13, then u (2^32 + 977) into limbs 0..2.
// Output T.
#ifdef HD_FE_NOINLINE
#define HD_FEMUL __host__ __device__ __noinline__
#else
#define HD_FEMUL HD
#endif
template <bool SQR>
HD_FEMUL void fe_mul_impl(fe& out, const fe& a, const fe& b) {
#ifdef HD_BOUND_CHECKS
    fe_bound_check_values(a);
    fe_bound_check_values(b);
    uint64_t ob[9];
    fe_mul_bounds(ob, a.b, SQR ? a.b : b.b);
#endif
    fe r;  // out may alias a or b
    // Inputs pass through opaque copies: the AMDGPU backend otherwise carries
    // known-bits facts (e.g. the 24-bit top limb masked by the producing
    // multiply) into this one and mis-selects the 64-bit column products when
    // two multiplies are inlined back to back (wrong results at -O1..-O3,
    // correct at -O0 and with fe_mul_impl out of line; scripts/fecheck.hip).
    uint32_t x[9], y[9];
    HD_UNROLL for (int i = 0; i < 9; i++) x[i] = i == 8 ? opaque_u32(a.n[i]) : a.n[i];
    if (!SQR) {
        HD_UNROLL for (int i = 0; i < 9; i++) y[i] = i == 8 ? opaque_u32(b.n[i]) : b.n[i];
    }
    uint32_t a2[8];
    if (SQR) {
        HD_UNROLL for (int i = 0; i < 8; i++) a2[i] = x[i] << 1;
    }
    // (K8 and K13 are opaque too: a known power of two turns the one mad
    // into a 64-bit shift, two masks and an add)
    const uint32_t K1 = opaque_s32(0x7A20u), K2 = opaque_s32(256u), K8 = opaque_s32(8u), K13 = opaque_s32(1u << 13);
    uint64_t clo = 0, c = 0;
    uint32_t dhi = 0, hprev = 0;
    HD_UNROLL for (int k = 0; k < 9; k++) {
        uint64_t d = 0;
        HD_UNROLL for (int i = k + 1; i < 9; i++) {
            const int j = k + 9 - i;
            if (SQR) {
                if (i < j) d = mad64(a2[i], x[j], d);
                else if (i == j) d = mad64(x[i], x[i], d);
            } else {
                d = mad64(x[i], y[j], d);
            }
        }
        if (k > 0) d = mad64(dhi, K8, d);
        const uint32_t hk = (uint32_t)d;
        dhi = (uint32_t)(d >> 32);
        c = mad64(hk, K1, clo);
        if (k > 0) c = mad64(hprev, K2, c);
        HD_UNROLL for (int i = 0; i <= k; i++) {
            const int j = k - i;
            if (SQR) {
                if (i < j) c = mad64(a2[i], x[j], c);
                else if (i == j) c = mad64(x[i], x[i], c);
            } else {
                c = mad64(x[i], y[j], c);
            }
        }
        if (k < 8) {
            r.n[k] = (uint32_t)c & HD_M29;
            clo = c >> 29;
        }
        hprev = hk;
    }
    // weight 2^256: u = (c8 >> 24) + h8 2^13 (< 2^48); limb 8 keeps c8's low 24 bits
    r.n[8] = (uint32_t)c & HD_M24;
    const uint64_t u = mad64(hprev, K13, c >> 24);
    // u (2^32 + 977): u 977 into limb 0, u 2^32 = 8 u 2^29 into limb 1
    const uint64_t f0 = mad64((uint32_t)u, 977u, r.n[0]);
    const uint64_t g = mad64((uint32_t)(u >> 32), 977u * 8u, (f0 >> 29) + r.n[1]);
    const uint64_t f1 = g + (u << 3);
    r.n[0] = (uint32_t)f0 & HD_M29;
    r.n[1] = (uint32_t)f1 & HD_M29;
    // laundered: left alone the backend keeps limb 2 as the 64-bit sum and
    // multiplies both of its halves in the next product
    r.n[2] = opaque_u32(r.n[2] + (uint32_t)(f1 >> 29));
    HD_B(for (int i = 0; i < 9; i++) r.b[i] = ob[i];)
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
// (product scanning; the c4 = 1 term is a multiply by 1 into the same column)
template <int NA>
HD void mul_by_c(uint32_t* P, const uint32_t* a) {
    const uint32_t C[5] = {HD_C0, HD_C1, HD_C2, HD_C3, 1u};
    uint64_t acc = 0;
    uint32_t hi = 0;
    HD_UNROLL for (int k = 0; k < NA + 4; k++) {
        HD_UNROLL for (int j = 0; j < 5; j++) {
            const int i = k - j;
            if (i >= 0 && i < NA) macc96(acc, hi, a[i], C[j]);
        }
        P[k] = (uint32_t)acc;
        col96_shift(acc, hi);
    }
    P[NA + 4] = (uint32_t)acc;
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
