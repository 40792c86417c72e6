// hd_sha256.h -- FIPS 180-4 SHA-256 for the three fixed-size inputs of the
// hot path, with the message schedule held in registers (no byte buffers):
//   * vote digest      SHA-256(BE64 h || BE64 r || value)            48 B, 1 block
//     (process/message.go:172-186, 270-284 -- identical for Prevote/Precommit)
//   * propose digest   SHA-256(BE64 h || BE64 r || BE64 vr || value) 56 B, 2 blocks
//     (process/message.go:60-78)
//   * signatory        SHA-256(pubkey)  SEC1 compressed 33 B (1 block), SEC1
//     uncompressed 65 B (2 blocks), raw X || Y 64 B (2 blocks) or X.Bytes() ||
//     Y.Bytes() (Go minimal encodings, <= 64 B, 1 or 2 blocks)
//     [renproject/id v0.4.2 NewSignatory; the encoding is a context setting]
// plus a small streaming context used only by the synthetic-workload signer
// (HMAC-SHA256 for RFC6979 nonces).
#pragma once
#include "hd_common.h"

namespace hd {

#define HD_ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

// Round constants; indexed only with compile-time indices (unrolled rounds),
// so they fold into instruction immediates on device.
HD uint32_t sha256_k(int i) {
        const uint32_t K[64] = {
            0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
            0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
            0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
            0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
            0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
            0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
            0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
            0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
        return K[i];
}

HD void sha256_init(uint32_t st[8]) {
    st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
    st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}

// One compression over 16 big-endian message words w[0..15] (w is clobbered).
HD void sha256_compress(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    HD_UNROLL
    for (int i = 0; i < 64; i++) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            uint32_t s0 = HD_ROR(w15, 7) ^ HD_ROR(w15, 18) ^ (w15 >> 3);
            uint32_t s1 = HD_ROR(w2, 17) ^ HD_ROR(w2, 19) ^ (w2 >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
        }
        uint32_t t1 = h + (HD_ROR(e, 6) ^ HD_ROR(e, 11) ^ HD_ROR(e, 25)) + ((e & f) ^ (~e & g)) + sha256_k(i) + wi;
        uint32_t t2 = (HD_ROR(a, 2) ^ HD_ROR(a, 13) ^ HD_ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Vote digest: words = BE64(h) BE64(r) value[8 words], 48 bytes.
HD void sha256_vote(uint32_t out[8], int64_t h, int64_t r, const uint32_t value_be[8]) {
    uint32_t st[8], w[16];
    sha256_init(st);
    w[0] = (uint32_t)((uint64_t)h >> 32); w[1] = (uint32_t)h;
    w[2] = (uint32_t)((uint64_t)r >> 32); w[3] = (uint32_t)r;
    HD_UNROLL for (int i = 0; i < 8; i++) w[4 + i] = value_be[i];
    w[12] = 0x80000000u; w[13] = 0; w[14] = 0; w[15] = 48 * 8;
    sha256_compress(st, w);
    HD_UNROLL for (int i = 0; i < 8; i++) out[i] = st[i];
}

// Propose digest: BE64(h) BE64(r) BE64(vr) value, 56 bytes -> 2 blocks.
HD void sha256_propose(uint32_t out[8], int64_t h, int64_t r, int64_t vr, const uint32_t value_be[8]) {
    uint32_t st[8], w[16];
    sha256_init(st);
    w[0] = (uint32_t)((uint64_t)h >> 32); w[1] = (uint32_t)h;
    w[2] = (uint32_t)((uint64_t)r >> 32); w[3] = (uint32_t)r;
    w[4] = (uint32_t)((uint64_t)vr >> 32); w[5] = (uint32_t)vr;
    HD_UNROLL for (int i = 0; i < 8; i++) w[6 + i] = value_be[i];
    w[14] = 0x80000000u; w[15] = 0;
    sha256_compress(st, w);
    HD_UNROLL for (int i = 0; i < 15; i++) w[i] = 0;
    w[15] = 56 * 8;
    sha256_compress(st, w);
    HD_UNROLL for (int i = 0; i < 8; i++) out[i] = st[i];
}

// Signatory of a compressed pubkey: SHA-256(prefix || X_be), 33 bytes.
// x_be[0] is the most significant word of X.
HD void sha256_pub33(uint32_t out[8], uint32_t prefix, const uint32_t x_be[8]) {
    uint32_t st[8], w[16];
    sha256_init(st);
    w[0] = (prefix << 24) | (x_be[0] >> 8);
    HD_UNROLL for (int i = 1; i < 8; i++) w[i] = (x_be[i - 1] << 24) | (x_be[i] >> 8);
    w[8] = (x_be[7] << 24) | 0x00800000u;
    HD_UNROLL for (int i = 9; i < 15; i++) w[i] = 0;
    w[15] = 33 * 8;
    sha256_compress(st, w);
    HD_UNROLL for (int i = 0; i < 8; i++) out[i] = st[i];
}

// Uncompressed pubkey 0x04 || X || Y, 65 bytes -> 2 blocks.
HD void sha256_pub65(uint32_t out[8], const uint32_t x_be[8], const uint32_t y_be[8]) {
    uint32_t st[8], w[16];
    sha256_init(st);
    w[0] = (0x04u << 24) | (x_be[0] >> 8);
    HD_UNROLL for (int i = 1; i < 8; i++) w[i] = (x_be[i - 1] << 24) | (x_be[i] >> 8);
    w[8] = (x_be[7] << 24) | (y_be[0] >> 8);
    HD_UNROLL for (int i = 9; i < 16; i++) w[i] = (y_be[i - 9] << 24) | (y_be[i - 8] >> 8);
    sha256_compress(st, w);
    w[0] = (y_be[7] << 24) | 0x00800000u;
    HD_UNROLL for (int i = 1; i < 15; i++) w[i] = 0;
    w[15] = 65 * 8;
    sha256_compress(st, w);
    HD_UNROLL for (int i = 0; i < 8; i++) out[i] = st[i];
}

// Raw pubkey X || Y, 64 bytes -> 2 blocks (the second is padding only).
HD void sha256_pub64(uint32_t out[8], const uint32_t x_be[8], const uint32_t y_be[8]) {
    uint32_t st[8], w[16];
    sha256_init(st);
    HD_UNROLL for (int i = 0; i < 8; i++) { w[i] = x_be[i]; w[8 + i] = y_be[i]; }
    sha256_compress(st, w);
    w[0] = 0x80000000u;
    HD_UNROLL for (int i = 1; i < 15; i++) w[i] = 0;
    w[15] = 64 * 8;
    sha256_compress(st, w);
    HD_UNROLL for (int i = 0; i < 8; i++) out[i] = st[i];
}

// Number of leading zero bytes of a big-endian 256-bit value (32 for zero).
HD uint32_t be_lead_zero_bytes(const uint32_t w[8]) {
    uint32_t lz = 0;
    bool found = false;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        if (!found) {
            if (w[i]) {
                lz += (uint32_t)__builtin_clz(w[i]);
                found = true;
            } else {
                lz += 32;
            }
        }
    }
    return lz >> 3;
}

// w <- w shifted towards word 0 by nb bytes (a big-endian byte string loses its
// first nb bytes), zero fill; nb < 4 N.  A barrel of word selects then one
// funnel shift per word: every index is a compile-time constant, so the array
// stays in registers.
template <int N>
HD void be_shl_bytes(uint32_t w[N], uint32_t nb) {
    const uint32_t q = nb >> 2, sh = 8u * (nb & 3u);
    HD_UNROLL for (int s = 16; s >= 1; s >>= 1) {
        if (s >= N) continue;
        const bool take = (q & (uint32_t)s) != 0;
        HD_UNROLL for (int i = 0; i < N; i++) w[i] = take ? (i + s < N ? w[i + s] : 0u) : w[i];
    }
    HD_UNROLL for (int i = 0; i < N; i++) {
        const uint32_t next = i + 1 < N ? w[i + 1] : 0u;
        w[i] = (uint32_t)(((((uint64_t)w[i]) << 32) | next) >> (32u - sh));
    }
}

// X.Bytes() || Y.Bytes(): Go big.Int minimal big-endian encodings (leading zero
// bytes of each coordinate dropped), L = 64 - zx - zy bytes; one block when
// L <= 55 (only when the coordinates have 9+ leading zero bytes between them),
// else two.
HD void sha256_pub_xy_stripped(uint32_t out[8], const uint32_t x_be[8], const uint32_t y_be[8]) {
    const uint32_t zx = be_lead_zero_bytes(x_be), zy = be_lead_zero_bytes(y_be);
    uint32_t ys[8];
    HD_UNROLL for (int i = 0; i < 8; i++) ys[i] = y_be[i];
    be_shl_bytes<8>(ys, zy % 32u);
    if (zy == 32) HD_UNROLL for (int i = 0; i < 8; i++) ys[i] = 0;
    uint32_t m[17];
    HD_UNROLL for (int i = 0; i < 8; i++) { m[i] = x_be[i]; m[8 + i] = ys[i]; }
    m[16] = 0;
    be_shl_bytes<17>(m, zx);  // X's zero bytes leave; stripped Y follows X's last byte
    const uint32_t L = 64u - zx - zy;
    HD_UNROLL for (int i = 0; i < 17; i++)
        if ((uint32_t)i == (L >> 2)) m[i] |= 0x80000000u >> (8u * (L & 3u));
    uint32_t st[8], w[16];
    sha256_init(st);
    const bool one = L <= 55;
    HD_UNROLL for (int i = 0; i < 16; i++) w[i] = m[i];
    if (one) w[15] = L * 8;
    sha256_compress(st, w);
    if (!one) {
        w[0] = m[16];
        HD_UNROLL for (int i = 1; i < 15; i++) w[i] = 0;
        w[15] = L * 8;
        sha256_compress(st, w);
    }
    HD_UNROLL for (int i = 0; i < 8; i++) out[i] = st[i];
}

// The signatory of an affine key in pubkey format `fmt` (include/hd_verify.h
// HD_PUBKEY_*: 0 uncompressed, 1 compressed, 2 raw X || Y, 3 X.Bytes() ||
// Y.Bytes()); y_odd = Y mod 2.
HD void sha256_pubkey(uint32_t out[8], int fmt, const uint32_t x_be[8], const uint32_t y_be[8], uint32_t y_odd) {
    if (fmt == 1) sha256_pub33(out, 2u | (y_odd & 1u), x_be);
    else if (fmt == 2) sha256_pub64(out, x_be, y_be);
    else if (fmt == 3) sha256_pub_xy_stripped(out, x_be, y_be);
    else sha256_pub65(out, x_be, y_be);
}

// ---------------------------------------------------------------------------
// Streaming context (signer only; byte buffer lives in scratch on device).
struct Sha256Ctx {
    uint32_t st[8];
    uint8_t buf[64];
    uint32_t fill;
    uint64_t total;
};

HD void sha256_begin(Sha256Ctx& c) {
    sha256_init(c.st);
    c.fill = 0;
    c.total = 0;
}

HD void sha256_flush_block(Sha256Ctx& c) {
    uint32_t w[16];
    for (int i = 0; i < 16; i++) w[i] = load_be32(c.buf + 4 * i);
    sha256_compress(c.st, w);
    c.fill = 0;
}

HD void sha256_update(Sha256Ctx& c, const uint8_t* p, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        c.buf[c.fill++] = p[i];
        if (c.fill == 64) sha256_flush_block(c);
    }
    c.total += n;
}

HD void sha256_final(Sha256Ctx& c, uint8_t out[32]) {
    uint64_t bits = c.total * 8;
    uint8_t pad = 0x80;
    sha256_update(c, &pad, 1);
    uint8_t z = 0;
    while (c.fill != 56) sha256_update(c, &z, 1);
    uint8_t len[8];
    for (int i = 0; i < 8; i++) len[i] = (uint8_t)(bits >> (56 - 8 * i));
    sha256_update(c, len, 8);
    for (int i = 0; i < 8; i++) store_be32(out + 4 * i, c.st[i]);
}

HD void hmac_sha256(uint8_t out[32], const uint8_t key[32], const uint8_t* m1, uint32_t n1,
                    const uint8_t* m2, uint32_t n2, const uint8_t* m3, uint32_t n3) {
    uint8_t pad[64];
    Sha256Ctx c;
    for (int i = 0; i < 64; i++) pad[i] = (uint8_t)((i < 32 ? key[i] : 0) ^ 0x36);
    sha256_begin(c);
    sha256_update(c, pad, 64);
    sha256_update(c, m1, n1);
    sha256_update(c, m2, n2);
    sha256_update(c, m3, n3);
    uint8_t inner[32];
    sha256_final(c, inner);
    for (int i = 0; i < 64; i++) pad[i] = (uint8_t)((i < 32 ? key[i] : 0) ^ 0x5c);
    sha256_begin(c);
    sha256_update(c, pad, 64);
    sha256_update(c, inner, 32);
    sha256_final(c, out);
}

}  // namespace hd
