// hd_scmont.h -- scalar field (mod n) Montgomery products in radix 2^29 for
// the known-key check's scalar kernel (k_fast_scalars).
//
// sc_mul (hd_field.h) works on 8 x 32-bit limbs: every partial product needs
// a 96-bit column (mad + carry into a third word) and the accumulator's
// register pair moves at every column, ~530 instructions per product with
// its three folds by 2^256 - n.  Here a scalar is 9 limbs of 29 bits (value
// < 2n) and the product is interleaved Montgomery reduction (R = 2^261):
// column k accumulates a_i b_{k-i} and q_i n_{k-i} in ONE 64-bit chain of
// v_mad_u64_u32 (18 terms of < 2^58 at most: no carry flags), and for
// k < 9 picks q_k = acc n' mod 2^29 so that the column's low 29 bits vanish.
// 162 mads + 9 multiplies and ~30 other instructions.
//
// sm_mul(a, b) = a b R^-1 mod n, < 2n for a, b < 2n (R > 4n).
#pragma once
#include "hd_field.h"

namespace hd {

struct sm {
    uint32_t n[9];   // value = sum n[i] 2^(29 i); n[0..7] <= M29
};

// n in radix 2^29, n' = -n^-1 mod 2^29, R^2 mod n (R = 2^261)
#define HD_SMN0 0x10364141u
#define HD_SMN1 0x1E92F466u
#define HD_SMN2 0x12280EEFu
#define HD_SMN3 0x1DB9CD5Eu
#define HD_SMN4 0x1FFFEBAAu
#define HD_SMN8 0x00FFFFFFu
#define HD_SMNP 0x1588B13Fu

HD uint32_t sm_n_limb(int i) {
    return i == 0 ? HD_SMN0 : i == 1 ? HD_SMN1 : i == 2 ? HD_SMN2 : i == 3 ? HD_SMN3 : i == 4 ? HD_SMN4
                                                                                    : i == 8 ? HD_SMN8 : HD_M29;
}

HD void sm_r2(sm& r) {
    const uint32_t R2[9] = {0x09F6AB4Bu, 0x1F300D1Eu, 0x1C0BD5D8u, 0x0C8ADA8Cu, 0x11CEFA2Bu,
                            0x08B79A0Fu, 0x1E697F5Eu, 0x00E34DE2u, 0x009C7356u};
    HD_UNROLL for (int i = 0; i < 9; i++) r.n[i] = R2[i];
}

// 8 little-endian words (value < 2^256) -> radix 2^29
HD void sm_from_sc(sm& r, const sc& a) {
    HD_UNROLL for (int i = 0; i < 9; i++) {
        const int bit = 29 * i, word = bit >> 5, off = bit & 31;
        uint32_t v = a.v[word] >> off;
        if (off > 3 && word + 1 < 8) v |= a.v[word + 1] << (32 - off);
        r.n[i] = v & (i == 8 ? HD_M24 : HD_M29);
    }
}

// value < 2n -> canonical (< n) little-endian words
HD void sm_to_sc(sc& r, const sm& a) {
    // d = a - n; keep it when there is no borrow (a >= n)
    uint32_t d[9];
    uint32_t borrow = 0;
    HD_UNROLL for (int i = 0; i < 9; i++) {
        const uint32_t t = a.n[i] - sm_n_limb(i) - borrow;
        borrow = t >> 31;                      // limbs < 2^30: the sign bit is the borrow
        d[i] = t & HD_M29;
    }
    const bool ge = borrow == 0;
    uint32_t x[9];
    HD_UNROLL for (int i = 0; i < 9; i++) x[i] = ge ? d[i] : a.n[i];
    HD_UNROLL for (int k = 0; k < 8; k++) r.v[k] = 0;
    HD_UNROLL for (int i = 0; i < 9; i++) {
        const int bit = 29 * i, word = bit >> 5, off = bit & 31;
        r.v[word] |= x[i] << off;
        if (off > 3 && word + 1 < 8) r.v[word + 1] |= x[i] >> (32 - off);
    }
}

// out = a b R^-1 mod n (< 2n); out may alias a or b
HD void sm_mul(sm& out, const sm& a, const sm& b) {
    uint32_t N[9], q[9];
    HD_UNROLL for (int i = 0; i < 9; i++) N[i] = opaque_s32(sm_n_limb(i));
    const uint32_t NP = opaque_s32(HD_SMNP);
    sm r;
    uint64_t c = 0;
    HD_UNROLL for (int k = 0; k < 17; k++) {
        // two independent mad chains per column (a b and q n), joined once:
        // a single chain would wait out every mad's latency
        uint64_t acc = c, acq = 0;
        HD_UNROLL for (int i = 0; i < 9; i++) {
            const int j = k - i;
            if (j >= 0 && j < 9) acc = mad64(a.n[i], b.n[j], acc);
        }
        HD_UNROLL for (int i = 0; i < 9; i++) {
            const int j = k - i;
            if (i < k && j >= 0 && j < 9) acq = mad64(q[i], N[j], acq);
        }
        if (k > 0) acc += acq;
        if (k < 9) {
            q[k] = ((uint32_t)acc * NP) & HD_M29;
            acc = mad64(q[k], N[0], acc);   // the column's low 29 bits are now 0
        } else {
            r.n[k - 9] = (uint32_t)acc & HD_M29;
        }
        c = acc >> 29;
    }
    r.n[8] = (uint32_t)c;
    out = r;
}

}  // namespace hd
