// kara_proto.h -- round-5 prototype (fieldbench only, not product code): a
// one-level Karatsuba fe_mul over the 9 radix-2^29 limbs, split 5 + 4
// (x = xL + xH 2^145).  Column-wise the middle product is exact:
//   m_k = sum_{i+j=k} (x_i + x_{i+5})(y_j + y_{j+5}) = z0_k + z2_k + z1_k
// so z1 = m - z0 - z2 needs no borrows across columns.  66 limb products
// (25 + 16 + 25) instead of 81, plus 8 limb sums, 16 64-bit column
// subtractions and the recombination; the fold at 2^261 is then done on
// 29-bit limbs (no register-boundary trick).  Inputs T (limbs <= 2^29 + 1):
// sums < 2^30.1, five products per column < 2^62.4.
#pragma once
#include "../hyperdrive_amd/csrc/hd_field.h"

namespace hd {

HD void fe_mul_kara(fe& out, const fe& a, const fe& b) {
    uint32_t x[9], y[9];
    HD_UNROLL for (int i = 0; i < 9; i++) {
        x[i] = opaque_u32(a.n[i]);
        y[i] = opaque_u32(b.n[i]);
    }
    uint32_t s[5], t[5];
    HD_UNROLL for (int i = 0; i < 4; i++) {
        s[i] = x[i] + x[i + 5];
        t[i] = y[i] + y[i + 5];
    }
    s[4] = x[4];
    t[4] = y[4];
    uint64_t z0[9], z2[7], m[9];
    HD_UNROLL for (int k = 0; k < 9; k++) z0[k] = m[k] = 0;
    HD_UNROLL for (int k = 0; k < 7; k++) z2[k] = 0;
    HD_UNROLL for (int i = 0; i < 5; i++)
        HD_UNROLL for (int j = 0; j < 5; j++) {
            z0[i + j] = mad64(x[i], y[j], z0[i + j]);
            m[i + j] = mad64(s[i], t[j], m[i + j]);
        }
    HD_UNROLL for (int i = 0; i < 4; i++)
        HD_UNROLL for (int j = 0; j < 4; j++) z2[i + j] = mad64(x[i + 5], y[j + 5], z2[i + j]);
    // product columns P_k (weight 2^(29 k)), k = 0 .. 16
    uint64_t P[17];
    HD_UNROLL for (int k = 0; k < 17; k++) P[k] = 0;
    HD_UNROLL for (int k = 0; k < 9; k++) P[k] += z0[k];
    HD_UNROLL for (int k = 0; k < 7; k++) P[k + 10] += z2[k];
    HD_UNROLL for (int k = 0; k < 9; k++) P[k + 5] += m[k] - z0[k] - (k < 7 ? z2[k] : 0ull);
    // high columns 9 .. 16 -> 29-bit limbs h_0 .. h_8 (weight 2^(261 + 29 j))
    uint32_t h[9];
    uint64_t c = 0;
    HD_UNROLL for (int k = 9; k < 17; k++) {
        c += P[k];
        h[k - 9] = (uint32_t)c & HD_M29;
        c >>= 29;
    }
    h[8] = (uint32_t)c;   // < 2^35 would not fit: bounded < 2^29 for T inputs (top limb 24 bits)
    // fold: 2^261 == 2^8 2^29 + 0x7A20 (mod p)
    uint64_t L[10];
    HD_UNROLL for (int k = 0; k < 9; k++) L[k] = P[k];
    L[9] = 0;
    HD_UNROLL for (int j = 0; j < 9; j++) {
        L[j] = mad64(h[j], 0x7A20u, L[j]);
        L[j + 1] = mad64(h[j], 256u, L[j + 1]);
    }
    // carry the low columns; limb 8 keeps 24 bits, the rest folds at 2^256
    fe r;
    c = 0;
    HD_UNROLL for (int k = 0; k < 8; k++) {
        c += L[k];
        r.n[k] = (uint32_t)c & HD_M29;
        c >>= 29;
    }
    c += L[8];
    r.n[8] = (uint32_t)c & HD_M24;
    const uint64_t u = (c >> 24) + (L[9] << 5);   // L[9] at weight 2^261 = 2^5 2^256
    const uint64_t f0 = mad64((uint32_t)u, 977u, r.n[0]);
    const uint64_t g = mad64((uint32_t)(u >> 32), 977u * 8u, (f0 >> 29) + r.n[1]);
    const uint64_t f1 = g + (u << 3);
    r.n[0] = (uint32_t)f0 & HD_M29;
    r.n[1] = (uint32_t)f1 & HD_M29;
    r.n[2] = opaque_u32(r.n[2] + (uint32_t)(f1 >> 29));
    out = r;
}

}  // namespace hd
