// fe8_proto.h (prototype, scripts/fieldbench.hip; measured slower, not used by the library) -- secp256k1 field elements as 8 x 32-bit words, for the
// known-key check's fixed-base sums (k_fast_sums).
//
// hd_field.h's fe keeps 9 limbs of 29 bits so that product columns never
// overflow 64 bits: 81 limb products plus ~28 multiply-adds of folding per
// product.  With full 32-bit words a product has 64 limb products, and the
// column sums outgrow 64 bits: each v_mad_u64_u32 here also writes its
// carry-out (the 64-bit add's overflow, a lane mask in an SGPR pair), and one
// full-rate v_addc_co_u32 counts it into a third accumulator word.  The
// pseudo-Mersenne fold (2^256 == 2^32 + 977 mod p) then costs 8 + 2
// multiply-adds instead of ~28.
//
// Values are any residue in [0, 2^256) (not necessarily below p): products,
// sums and differences all return such a value; fe8_canon gives the
// canonical one.  Table points (hd_fixedbase.h gp) are canonical 8-word
// little-endian values already, so they are read without conversion.
//
// Like the rest of csrc/, this header compiles for gfx950 and as host C++
// (tests/native: the same formulas with __int128 in place of the carry-out
// instruction, checked against Python integers).
#pragma once
#include "../hyperdrive_amd/csrc/hd_field.h"

namespace hd {

struct fe8 {
    uint32_t w[8];
};

#define HD_FE8_C0 977u   // 2^256 mod p = 2^32 + 977: word 0
// acc : hi (96 bits) += a b: v_mad_u64_u32 with its carry-out, then
// v_addc_co_u32 of the carry into hi
HD void madc(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint64_t r, cc, cc2;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(a), "v"(b), "v"(acc));
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(hi), "=s"(cc2) : "v"(hi), "s"(cc));
    (void)cc2;
    acc = r;
#else
    const unsigned __int128 s = (unsigned __int128)a * b + acc;
    acc = (uint64_t)s;
    hi += (uint32_t)(s >> 64);
#endif
}

// the 512-bit t (16 words) mod p into [0, 2^256): t = L + H 2^256 ==
// L + H 977 + H 2^32, then the part above 2^256 (< 2^33) once more, then a
// last carry (possible only when the value is then below 2^66)
HD void fe8_reduce512(fe8& r, const uint32_t t[16]) {
    uint64_t acc = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        acc += t[i];
        if (i > 0) acc += t[8 + i - 1];
        acc = mad64(t[8 + i], HD_FE8_C0, acc);   // < 2^42
        r.w[i] = (uint32_t)acc;
        acc >>= 32;
    }
    const uint64_t top = acc + t[15];   // < 2^33
    const uint32_t tl = (uint32_t)top, th = (uint32_t)(top >> 32);
    acc = mad64(tl, HD_FE8_C0, r.w[0]);
    r.w[0] = (uint32_t)acc;
    acc = (acc >> 32) + r.w[1] + tl + (uint64_t)th * HD_FE8_C0;
    r.w[1] = (uint32_t)acc;
    acc = (acc >> 32) + r.w[2] + th;
    r.w[2] = (uint32_t)acc;
    HD_UNROLL for (int i = 3; i < 8; i++) {
        acc = (acc >> 32) + r.w[i];
        r.w[i] = (uint32_t)acc;
    }
    // a carry out of 2^256 leaves r < top (2^32 + 977) < 2^66: adding
    // 2^32 + 977 once more cannot carry past word 2
    const uint32_t c = (uint32_t)(acc >> 32);
    acc = (uint64_t)r.w[0] + c * HD_FE8_C0;
    r.w[0] = (uint32_t)acc;
    acc = (acc >> 32) + r.w[1] + c;
    r.w[1] = (uint32_t)acc;
    r.w[2] += (uint32_t)(acc >> 32);
}

// product scanning: column k collects a_i b_j (i + j = k) in 96 bits
HD void fe8_mul(fe8& r, const fe8& a, const fe8& b) {
    uint32_t t[16];
    uint64_t acc = 0;
    HD_UNROLL for (int k = 0; k < 15; k++) {
        uint32_t hi = 0;
        HD_UNROLL for (int i = (k > 7 ? k - 7 : 0); i <= (k < 7 ? k : 7); i++) madc(acc, hi, a.w[i], b.w[k - i]);
        t[k] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)hi << 32);
    }
    t[15] = (uint32_t)acc;
    fe8_reduce512(r, t);
}

// the cross products a_i a_j (i < j) by product scanning, doubled, plus the
// squares: 28 + 8 multiply-adds
HD void fe8_sqr(fe8& r, const fe8& a) {
    uint32_t x[16];
    x[0] = 0;
    uint64_t acc = 0;
    HD_UNROLL for (int k = 1; k < 14; k++) {
        uint32_t hi = 0;
        HD_UNROLL for (int i = (k > 7 ? k - 7 : 0); 2 * i < k; i++) madc(acc, hi, a.w[i], a.w[k - i]);
        x[k] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)hi << 32);
    }
    x[14] = (uint32_t)acc;
    x[15] = (uint32_t)(acc >> 32);
    uint32_t t[16];
    uint32_t c = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        const uint32_t lo = (x[2 * i] << 1) | (i > 0 ? x[2 * i - 1] >> 31 : 0u);
        const uint32_t hw = (x[2 * i + 1] << 1) | (x[2 * i] >> 31);
        const uint64_t d = ((uint64_t)hw << 32) | lo;
        const uint64_t s = mad64(a.w[i], a.w[i], c);   // a_i^2 + c < 2^64
        const uint64_t u = s + d;
        c = u < s ? 1u : 0u;
        t[2 * i] = (uint32_t)u;
        t[2 * i + 1] = (uint32_t)(u >> 32);
    }
    fe8_reduce512(r, t);   // (2X + squares < 2^512: no carry out of word 15)
}

// a + b mod p: the carry out of 2^256 comes back as 2^32 + 977, twice at most
HD void fe8_add(fe8& r, const fe8& a, const fe8& b) {
    uint64_t acc = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        acc = (acc >> 32) + a.w[i] + b.w[i];
        r.w[i] = (uint32_t)acc;
    }
    HD_UNROLL for (int pass = 0; pass < 2; pass++) {
        const uint32_t c = (uint32_t)(acc >> 32);
        acc = (uint64_t)r.w[0] + c * HD_FE8_C0;
        r.w[0] = (uint32_t)acc;
        acc = (acc >> 32) + r.w[1] + c;
        r.w[1] = (uint32_t)acc;
        HD_UNROLL for (int i = 2; i < 8; i++) {
            acc = (acc >> 32) + r.w[i];
            r.w[i] = (uint32_t)acc;
        }
    }
}

// a - b mod p: a borrow out of 2^256 is taken back by subtracting 2^32 + 977
// (-2^256 == -(2^32 + 977)); a second borrow is possible only when the first
// result was below 2^32 + 977, and a third never
HD void fe8_sub(fe8& r, const fe8& a, const fe8& b) {
    uint64_t t = 0;
    uint32_t br = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        t = (uint64_t)a.w[i] - b.w[i] - br;
        r.w[i] = (uint32_t)t;
        br = (uint32_t)(t >> 63);
    }
    HD_UNROLL for (int pass = 0; pass < 2; pass++) {
        t = (uint64_t)r.w[0] - br * HD_FE8_C0;
        r.w[0] = (uint32_t)t;
        uint32_t b2 = (uint32_t)(t >> 63);
        t = (uint64_t)r.w[1] - br - b2;
        r.w[1] = (uint32_t)t;
        b2 = (uint32_t)(t >> 63);
        HD_UNROLL for (int i = 2; i < 8; i++) {
            t = (uint64_t)r.w[i] - b2;
            r.w[i] = (uint32_t)t;
            b2 = (uint32_t)(t >> 63);
        }
        br = b2;
    }
}

// the canonical value (< p): subtract p when the value is at least p, i.e.
// when adding 2^32 + 977 carries out of 2^256
HD void fe8_canon(fe8& r) {
    uint32_t s[8];
    uint64_t acc = (uint64_t)r.w[0] + HD_FE8_C0;
    s[0] = (uint32_t)acc;
    acc = (acc >> 32) + r.w[1] + 1u;
    s[1] = (uint32_t)acc;
    HD_UNROLL for (int i = 2; i < 8; i++) {
        acc = (acc >> 32) + r.w[i];
        s[i] = (uint32_t)acc;
    }
    const bool ge = (acc >> 32) != 0;
    HD_UNROLL for (int i = 0; i < 8; i++) r.w[i] = ge ? s[i] : r.w[i];
}

// p - a for a canonical a (a table point's y): a value in (0, p], i.e. p
// itself for a = 0 (== 0 mod p)
HD void fe8_neg_canon(fe8& r, const fe8& a) {
    const uint32_t P[8] = {0xFFFFFC2Fu, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                           0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    uint32_t br = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        const uint64_t t = (uint64_t)P[i] - a.w[i] - br;
        r.w[i] = (uint32_t)t;
        br = (uint32_t)(t >> 63);
    }
}

HD void fe8_set_u32(fe8& r, uint32_t v) {
    r.w[0] = v;
    HD_UNROLL for (int i = 1; i < 8; i++) r.w[i] = 0;
}
HD void fe8_cmov(fe8& r, const fe8& a, bool flag) {
    HD_UNROLL for (int i = 0; i < 8; i++) r.w[i] = flag ? a.w[i] : r.w[i];
}
// to radix 2^29 (hd_field.h), canonical
HD void fe_from_fe8(fe& r, const fe8& a) {
    fe8 c = a;
    fe8_canon(c);
    fe_from_le(r, c.w);
}

}  // namespace hd
