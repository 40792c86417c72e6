// hd_keccak.h -- Keccak-f[1600] sponge, one message per lane.
//
// The optional digest lane of the north star.  The reference hashes with
// SHA-256 only (id.NewHash, process/message.go:77, 185, 283); this lane digests
// the same surge preimages with
//   * Keccak-256   rate 136 B, domain/pad byte 0x01 (the pre-FIPS padding
//                  Ethereum uses), or
//   * SHA3-256     rate 136 B, pad byte 0x06 (FIPS 202),
// both with the last byte of the rate block or'ed with 0x80.  The state is 25
// 64-bit lanes in registers (50 VGPRs); bytes map to lanes little-endian
// (FIPS 202 §B.1).  Round constants and rotation offsets are FIPS 202's; the
// Python oracle (oracle/keccak_oracle.py) derives them from their definitions
// (LFSR rc(t), (t+1)(t+2)/2 offsets) instead of copying them.
#pragma once
#include "hd_common.h"

namespace hd {

HD uint64_t keccak_rc(int i) {
    const uint64_t RC[24] = {
        0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
        0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
        0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
        0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
        0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
        0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
    return RC[i];
}

// rho offset of lane x + 5y
HD int keccak_rho(int i) {
    const int R[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
    return R[i];
}

HD uint64_t rotl64(uint64_t x, int n) { return n == 0 ? x : (x << n) | (x >> (64 - n)); }

// Keccak-f[1600]: 24 rounds of theta, rho, pi, chi, iota.  Fully unrolled so
// every lane index, offset and constant is a compile-time immediate.
HD void keccak_f1600(uint64_t a[25]) {
    HD_UNROLL for (int round = 0; round < 24; round++) {
        uint64_t c[5], b[25];
        HD_UNROLL for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
        HD_UNROLL for (int x = 0; x < 5; x++) {
            const uint64_t d = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
            HD_UNROLL for (int y = 0; y < 5; y++) a[x + 5 * y] ^= d;
        }
        // rho + pi: B[y, 2x + 3y] = rot(A[x, y], r[x, y])
        HD_UNROLL for (int x = 0; x < 5; x++)
            HD_UNROLL for (int y = 0; y < 5; y++)
                b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(a[x + 5 * y], keccak_rho(x + 5 * y));
        HD_UNROLL for (int y = 0; y < 5; y++)
            HD_UNROLL for (int x = 0; x < 5; x++)
                a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
        a[0] ^= keccak_rc(round);
    }
}

HD uint64_t bswap64(uint64_t x) {
    x = ((x & 0x00FF00FF00FF00FFull) << 8) | ((x >> 8) & 0x00FF00FF00FF00FFull);
    x = ((x & 0x0000FFFF0000FFFFull) << 16) | ((x >> 16) & 0x0000FFFF0000FFFFull);
    return (x << 32) | (x >> 32);
}

// lane holding BE64(v) (its 8 bytes little-endian)
HD uint64_t lane_be64(int64_t v) { return bswap64((uint64_t)v); }

// lane holding 8 bytes given as two big-endian words (bytes hi..lo order)
HD uint64_t lane_be_words(uint32_t w0, uint32_t w1) {
    return bswap64(((uint64_t)w0 << 32) | w1);
}

// Digest of a one-block preimage of `nl` 8-byte lanes (nl <= 16) already in
// a[0..nl-1] (rest zero): pad, permute, squeeze 32 bytes as big-endian words.
HD void keccak256_oneblock(uint32_t out_be[8], uint64_t a[25], int nl, uint8_t pad) {
    a[nl] ^= (uint64_t)pad;
    a[16] ^= 0x8000000000000000ull;   // last byte of the 136-byte rate block
    keccak_f1600(a);
    HD_UNROLL for (int k = 0; k < 4; k++) {
        const uint64_t be = bswap64(a[k]);
        out_be[2 * k] = (uint32_t)(be >> 32);
        out_be[2 * k + 1] = (uint32_t)be;
    }
}

// Vote preimage BE64(h) || BE64(r) || value (48 B, process/message.go:172-186,
// 270-284); value as 8 big-endian words.
HD void keccak256_vote(uint32_t out_be[8], int64_t h, int64_t r, const uint32_t value_be[8], uint8_t pad) {
    uint64_t a[25];
    HD_UNROLL for (int k = 0; k < 25; k++) a[k] = 0;
    a[0] = lane_be64(h);
    a[1] = lane_be64(r);
    HD_UNROLL for (int k = 0; k < 4; k++) a[2 + k] = lane_be_words(value_be[2 * k], value_be[2 * k + 1]);
    keccak256_oneblock(out_be, a, 6, pad);
}

// Propose preimage BE64(h) || BE64(r) || BE64(vr) || value (56 B, message.go:60-78)
HD void keccak256_propose(uint32_t out_be[8], int64_t h, int64_t r, int64_t vr, const uint32_t value_be[8],
                          uint8_t pad) {
    uint64_t a[25];
    HD_UNROLL for (int k = 0; k < 25; k++) a[k] = 0;
    a[0] = lane_be64(h);
    a[1] = lane_be64(r);
    a[2] = lane_be64(vr);
    HD_UNROLL for (int k = 0; k < 4; k++) a[3 + k] = lane_be_words(value_be[2 * k], value_be[2 * k + 1]);
    keccak256_oneblock(out_be, a, 7, pad);
}

// Arbitrary byte string through the sponge, bytes fetched by `get(i)` for
// i < len (a callable, so the device version can fetch from HBM).
template <typename Get>
HD void keccak256_bytes(uint32_t out_be[8], uint64_t len, uint8_t pad, Get get) {
    uint64_t a[25];
    HD_UNROLL for (int k = 0; k < 25; k++) a[k] = 0;
    uint64_t pos = 0;
    // full blocks
    HD_NOUNROLL while (len - pos >= 136) {
        HD_UNROLL for (int k = 0; k < 17; k++) a[k] ^= get(pos + 8 * k);
        keccak_f1600(a);
        pos += 136;
    }
    // final block: the remaining rem < 136 bytes, then pad
    const uint32_t rem = (uint32_t)(len - pos);
    HD_UNROLL for (int k = 0; k < 17; k++) {
        if (8u * k < rem) {
            uint64_t lane = get(pos + 8 * k);
            const uint32_t have = rem - 8u * k;   // bytes of this lane inside the message
            if (have < 8) lane &= (1ull << (8 * have)) - 1;
            a[k] ^= lane;
        }
    }
    a[rem / 8] ^= (uint64_t)pad << (8 * (rem % 8));
    a[16] ^= 0x8000000000000000ull;
    keccak_f1600(a);
    HD_UNROLL for (int k = 0; k < 4; k++) {
        const uint64_t be = bswap64(a[k]);
        out_be[2 * k] = (uint32_t)(be >> 32);
        out_be[2 * k + 1] = (uint32_t)be;
    }
}

}  // namespace hd
