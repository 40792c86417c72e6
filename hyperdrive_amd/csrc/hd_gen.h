// hd_gen.h -- seeded synthetic signed-vote workload.
//
// This is input construction, the role processutil.RandomPrevote & co play in
// the reference tests (process/processutil/processutil.go:276-353) plus the
// signing step the reference tests do with id.PrivKey.Sign
// (process/message_test.go:150).  It mirrors oracle/hd_pyoracle.py's
// gen_message() bit-for-bit (tests/test_gen.py compares them).
//
// Signing = libsecp256k1 secp256k1_ecdsa_sign_recoverable: RFC6979
// HMAC-SHA256 nonce (key32 || msg32, no extra data), r = (kG).x mod n,
// s = k^-1 (m + r d), low-S normalisation with recid flip.
#pragma once
#include "hd_verify_msg.h"

namespace hd {

#define HD_GEN_SEED 0x48595045ull
#define HD_NONADMITTED_BASE 1000000u
#define HD_N_ADV_CLASSES 13
#define HD_NONADMITTED_KEYS 16

enum GenKind : uint32_t { GEN_VOTES = 0, GEN_ROUNDS = 1 };

HD uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
HD uint64_t gen_rnd(uint64_t i, uint32_t stream) {
    return splitmix64(splitmix64(HD_GEN_SEED) ^ ((i << 4) | stream));
}

// sk_idx = (SHA-256("hd-sk" || BE32(idx)) mod (n-1)) + 1
HD void signer_sk(sc& sk, uint32_t idx) {
    uint32_t st[8], w[16];
    sha256_init(st);
    // "hd-sk" = 68 64 2d 73 6b, then BE32(idx): 9 bytes
    w[0] = 0x68642d73u;
    w[1] = (0x6bu << 24) | (idx >> 8);
    w[2] = (idx << 24) | 0x00800000u;
    HD_UNROLL for (int i = 3; i < 15; i++) w[i] = 0;
    w[15] = 9 * 8;
    sha256_compress(st, w);
    uint32_t m[8];
    HD_UNROLL for (int i = 0; i < 8; i++) m[i] = st[7 - i];
    // n - 1
    const uint32_t NM1[8] = {HD_N0 - 1, HD_N1, HD_N2, HD_N3, HD_N4, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    bool lt = false, gt = false;
    HD_UNROLL for (int i = 7; i >= 0; i--) {
        bool g = !lt && !gt && m[i] > NM1[i];
        bool l = !lt && !gt && m[i] < NM1[i];
        gt = gt || g;
        lt = lt || l;
    }
    if (!lt) {  // m >= n-1 : m -= n-1
        uint64_t br = 0;
        HD_UNROLL for (int i = 0; i < 8; i++) {
            uint64_t t = (uint64_t)m[i] - NM1[i] - br;
            m[i] = (uint32_t)t;
            br = t >> 63;
        }
    }
    uint64_t c = 1;
    HD_UNROLL for (int i = 0; i < 8; i++) { c += m[i]; sk.v[i] = (uint32_t)c; c >>= 32; }
}

// k*G with 8-bit Booth windows (256 doublings + 33 mixed additions)
template <typename GTab>
HD void ecmult_gen(gej& out, const sc& k, GTab gtab) {
    gej acc;
    gej_set_inf(acc);
    HD_NOUNROLL for (int j = HD_NWIN_G - 1; j >= 0; j--) {
        if (j != HD_NWIN_G - 1) {
            HD_NOUNROLL for (int t = 0; t < HD_WG; t++) gej_dbl(acc, acc);
        }
        int d = booth_digit<HD_WG>(k, j);
        int ad = d < 0 ? -d : d;
        ge t = gtab[ad == 0 ? 0 : ad - 1];
        if (d < 0) fe_neg(t.y, t.y);
        gej s;
        gej_add_ge(s, acc, t);
        gej_cmov(acc, s, d != 0);
    }
    out = acc;
}

template <typename GTab>
HD void pubkey_signatory(uint32_t out_be[8], const sc& sk, int pkfmt, GTab gtab) {
    gej P;
    ecmult_gen(P, sk, gtab);
    fe x, y;
    gej_to_ge(x, y, P);
    uint32_t xb[8], yb[8];
    fe_to_be(xb, x);
    fe_to_be(yb, y);
    sha256_pubkey(out_be, pkfmt, xb, yb, y.n[0] & 1u);
}

HD void sc_to_bytes(uint8_t b[32], const sc& a) {
    for (int i = 0; i < 8; i++) store_be32(b + 4 * i, a.v[7 - i]);
}

// libsecp256k1 sign_recoverable with nonce_function_rfc6979.
// sig = r(32 BE) || s(32 BE) || recid
template <typename GTab>
HD void ecdsa_sign(uint32_t r_be[8], uint32_t s_be[8], uint32_t& recid, const sc& sk,
                   const uint32_t digest_be[8], GTab gtab) {
    uint8_t key32[32], msg32[32], V[32], K[32];
    sc_to_bytes(key32, sk);
    for (int i = 0; i < 8; i++) store_be32(msg32 + 4 * i, digest_be[i]);
    for (int i = 0; i < 32; i++) { V[i] = 1; K[i] = 0; }
    uint8_t b0 = 0, b1 = 1;
    uint8_t seed[64];
    for (int i = 0; i < 32; i++) { seed[i] = key32[i]; seed[32 + i] = msg32[i]; }
    // K = HMAC(K, V || 0x00 || seed); V = HMAC(K, V)
    hmac_sha256(K, K, V, 32, &b0, 1, seed, 64);
    hmac_sha256(V, K, V, 32, 0, 0, 0, 0);
    hmac_sha256(K, K, V, 32, &b1, 1, seed, 64);
    hmac_sha256(V, K, V, 32, 0, 0, 0, 0);
    sc m;
    sc_from_be_reduce(m, digest_be);
    bool first = true;
    for (;;) {
        if (!first) {
            hmac_sha256(K, K, V, 32, &b0, 1, 0, 0);
            hmac_sha256(V, K, V, 32, 0, 0, 0, 0);
        }
        first = false;
        hmac_sha256(V, K, V, 32, 0, 0, 0, 0);
        sc k;
        for (int i = 0; i < 8; i++) k.v[i] = load_be32(V + 4 * (7 - i));
        if (sc_is_zero(k) || sc_ge_n(k.v)) continue;
        gej Rj;
        ecmult_gen(Rj, k, gtab);
        fe rx, ry;
        gej_to_ge(rx, ry, Rj);
        uint32_t rid = ry.n[0] & 1u;
        uint32_t xm[8];
        fe_to_le(xm, rx);
        if (sc_ge_n(xm)) { sc_sub_n(xm); rid |= 2u; }
        sc r;
        for (int i = 0; i < 8; i++) r.v[i] = xm[i];
        sc t, kinv, s;
        sc_mul(t, r, sk);
        // t = t + m mod n
        {
            uint32_t o[8];
            uint64_t c = 0;
            for (int i = 0; i < 8; i++) { c += (uint64_t)t.v[i] + m.v[i]; o[i] = (uint32_t)c; c >>= 32; }
            if (c || sc_ge_n(o)) sc_sub_n(o);
            for (int i = 0; i < 8; i++) t.v[i] = o[i];
        }
        sc_inv_divsteps(kinv, k);
        sc_mul(s, kinv, t);
        if (sc_is_zero(r) || sc_is_zero(s)) continue;
        // high-S: s > n/2
        const uint32_t NH[8] = {0x681B20A0u, 0xDFE92F46u, 0x57A4501Du, 0x5D576E73u,
                                0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};
        bool lt = false, gt = false;
        for (int i = 7; i >= 0; i--) {
            bool g = !lt && !gt && s.v[i] > NH[i];
            bool l = !lt && !gt && s.v[i] < NH[i];
            gt = gt || g;
            lt = lt || l;
        }
        if (gt) { sc_neg(s, s); rid ^= 1u; }
        for (int i = 0; i < 8; i++) { r_be[i] = r.v[7 - i]; s_be[i] = s.v[7 - i]; }
        recid = rid;
        return;
    }
}

// canonical V(h, r) = SHA-256("hd-v" || BE64 h || BE64 r)  (20 bytes)
HD void canonical_value(uint32_t out_be[8], int64_t h, int64_t r) {
    uint32_t st[8], w[16];
    sha256_init(st);
    w[0] = 0x68642d76u;  // "hd-v"
    w[1] = (uint32_t)((uint64_t)h >> 32);
    w[2] = (uint32_t)h;
    w[3] = (uint32_t)((uint64_t)r >> 32);
    w[4] = (uint32_t)r;
    w[5] = 0x80000000u;
    HD_UNROLL for (int i = 6; i < 15; i++) w[i] = 0;
    w[15] = 20 * 8;
    sha256_compress(st, w);
    HD_UNROLL for (int i = 0; i < 8; i++) out_be[i] = st[i];
}
HD void random_value(uint32_t out_be[8], uint64_t i) {
    HD_UNROLL for (int j = 0; j < 4; j++) {
        uint64_t x = gen_rnd(i, 1 + j);
        out_be[2 * j] = (uint32_t)(x >> 32);
        out_be[2 * j + 1] = (uint32_t)x;
    }
}
HD void vote_value(uint32_t out_be[8], uint64_t i, int64_t h, int64_t r) {
    uint64_t u = gen_rnd(i, 0) % 100;
    if (u < 90) canonical_value(out_be, h, r);
    else if (u < 95) { HD_UNROLL for (int j = 0; j < 8; j++) out_be[j] = 0; }
    else random_value(out_be, i);
}

struct GenMsg {
    uint32_t type;
    int64_t h, r, vr;
    uint32_t value_be[8];
    uint32_t signer;  // index of the signing key (NONADMITTED_BASE + k for foreign keys)
};

HD void base_message(GenMsg& g, uint32_t kind, uint64_t i, uint32_t S) {
    g.vr = -1;
    if (kind == GEN_VOTES) {
        g.signer = (uint32_t)(i % S);
        g.type = T_PREVOTE + (uint32_t)((i / S) % 2);
        g.h = 1 + (int64_t)(i / (2ull * S));
        g.r = 0;
        vote_value(g.value_be, i, g.h, g.r);
        return;
    }
    uint64_t per = 1 + 2ull * S;
    g.r = (int64_t)(i / per);
    uint64_t k = i % per;
    g.h = 1;
    if (k == 0) {
        g.type = T_PROPOSE;
        g.signer = (uint32_t)((uint64_t)(g.h + g.r) % S);
        canonical_value(g.value_be, g.h, g.r);
    } else if (k <= S) {
        g.type = T_PREVOTE;
        g.signer = (uint32_t)(k - 1);
        vote_value(g.value_be, i, g.h, g.r);
    } else {
        g.type = T_PRECOMMIT;
        g.signer = (uint32_t)(k - S - 1);
        vote_value(g.value_be, i, g.h, g.r);
    }
}

HD void put_be64(uint8_t* p, int64_t x) {
    uint64_t u = (uint64_t)x;
    for (int i = 0; i < 8; i++) p[i] = (uint8_t)(u >> (56 - 8 * i));
}

// Generate message i.  signatories: S entries of 8 BE words (admitted keys),
// foreign: 16 entries (non-admitted keys NONADMITTED_BASE + k).
// Writes the SoA fields of one message; returns the adversarial class (-1 = none).
template <typename GTab, typename SigTab>
HD int gen_message(uint32_t kind, uint64_t i, uint32_t S, uint32_t adv_pct, GTab gtab, SigTab signatories,
                   SigTab foreign, uint8_t& type_out, int64_t& h_out, int64_t& r_out, int64_t& vr_out,
                   uint8_t* value32, uint8_t* from32, uint8_t* sig65) {
    GenMsg g;
    base_message(g, kind, i, S);
    int cls = -1;
    if (adv_pct && gen_rnd(i, 5) % 100 < adv_pct) cls = (int)(gen_rnd(i, 6) % HD_N_ADV_CLASSES);
    uint64_t w = gen_rnd(i, 8);
    uint32_t sk_idx = g.signer;
    if ((cls == 11 || cls == 12) && i > 0) {
        GenMsg p;
        base_message(p, kind, i - 1, S);
        g.type = p.type; g.h = p.h; g.r = p.r; g.vr = p.vr; g.signer = p.signer;
        sk_idx = p.signer;
        if (cls == 12) { for (int j = 0; j < 8; j++) g.value_be[j] = p.value_be[j]; }
        else random_value(g.value_be, i);
    }
    uint32_t from_be[8];
    if (cls == 6) {
        sk_idx = HD_NONADMITTED_BASE + (uint32_t)(i % HD_NONADMITTED_KEYS);
        for (int j = 0; j < 8; j++) from_be[j] = foreign[(i % HD_NONADMITTED_KEYS) * 8 + j];
    } else {
        for (int j = 0; j < 8; j++) from_be[j] = signatories[sk_idx * 8 + j];
    }
    MsgIn m;
    m.type = g.type;
    m.h = (cls == 7) ? g.h + 1 : g.h;
    m.r = g.r;
    m.vr = g.vr;
    for (int j = 0; j < 8; j++) m.value_be[j] = g.value_be[j];
    uint32_t d[8];
    message_digest(d, m);
    sc sk;
    signer_sk(sk, sk_idx);
    uint8_t sig[65];
    {
        uint32_t rb[8], sb[8], rid;
        ecdsa_sign(rb, sb, rid, sk, d, gtab);
        for (int j = 0; j < 8; j++) { store_be32(sig + 4 * j, rb[j]); store_be32(sig + 32 + 4 * j, sb[j]); }
        sig[64] = (uint8_t)rid;
    }
    if (cls == 0) {
        uint8_t raw[72];
        for (int j = 0; j < 9; j++) {
            uint64_t x = gen_rnd(i, 7 + j);
            for (int b = 0; b < 8; b++) raw[8 * j + b] = (uint8_t)(x >> (56 - 8 * b));
        }
        for (int j = 0; j < 65; j++) sig[j] = raw[j];
    } else if (cls == 1) {
        sig[64] = (uint8_t)(4 + (w % 252));
    } else if (cls == 2) {
        uint8_t* p = (w & 1) ? sig : sig + 32;
        for (int j = 0; j < 32; j++) p[j] = 0;
    } else if (cls == 3) {
        // n + ((w >> 1) & 0xFFFF)
        uint32_t o[8] = {HD_N0, HD_N1, HD_N2, HD_N3, HD_N4, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        uint64_t c = (uint64_t)o[0] + ((w >> 1) & 0xFFFFu);
        o[0] = (uint32_t)c; c >>= 32;
        for (int j = 1; j < 8; j++) { c += o[j]; o[j] = (uint32_t)c; c >>= 32; }
        uint8_t* p = (w & 1) ? sig : sig + 32;
        for (int j = 0; j < 8; j++) store_be32(p + 4 * j, o[7 - j]);
    } else if (cls == 4) {
        sig[64] |= 2;
        // (p - n) + w
        uint32_t o[8] = {0x2FC9BAEEu, 0x402DA172u, 0x50B75FC4u, 0x45512319u, 1u, 0u, 0u, 0u};
        uint64_t c = (uint64_t)o[0] + (uint32_t)w;
        o[0] = (uint32_t)c; c >>= 32;
        c += (uint64_t)o[1] + (uint32_t)(w >> 32);
        o[1] = (uint32_t)c; c >>= 32;
        for (int j = 2; j < 8; j++) { c += o[j]; o[j] = (uint32_t)c; c >>= 32; }
        for (int j = 0; j < 8; j++) store_be32(sig + 4 * j, o[7 - j]);
    } else if (cls == 5) {
        // smallest x >= w (as a 65-bit integer) with x^3 + 7 a non-residue
        uint32_t xw[8] = {(uint32_t)w, (uint32_t)(w >> 32), 0u, 0u, 0u, 0u, 0u, 0u};
        for (;;) {
            fe x, y2, y, seven;
            fe_from_le(x, xw);
            fe_sqr(y2, x);
            fe_mul(y2, y2, x);
            fe_set_u32(seven, 7);
            fe_add(y2, y2, seven);
            if (!fe_sqrt(y, y2)) break;
            uint64_t c = (uint64_t)xw[0] + 1;
            xw[0] = (uint32_t)c;
            c = (uint64_t)xw[1] + (c >> 32);
            xw[1] = (uint32_t)c;
            xw[2] += (uint32_t)(c >> 32);
        }
        for (int j = 0; j < 8; j++) store_be32(sig + 4 * j, xw[7 - j]);
        sig[64] &= 1;
    } else if (cls == 8) {
        if (m.type == T_PREVOTE || m.type == T_PRECOMMIT) m.type = (m.type == T_PREVOTE) ? T_PRECOMMIT : T_PREVOTE;
        else cls = 9;
    }
    if (cls == 9) {
        sc s;
        for (int j = 0; j < 8; j++) s.v[j] = load_be32(sig + 32 + 4 * (7 - j));
        sc_neg(s, s);
        for (int j = 0; j < 8; j++) store_be32(sig + 32 + 4 * j, s.v[7 - j]);
        sig[64] ^= 1;
    } else if (cls == 10) {
        sc k;
        for (int j = 0; j < 8; j++) k.v[j] = 0;
        uint64_t kk = w + 1;  // w % (n-1) + 1 for a 64-bit w
        k.v[0] = (uint32_t)kk;
        k.v[1] = (uint32_t)(kk >> 32);
        if (kk == 0) k.v[2] = 1;  // w = 2^64-1 -> 2^64
        gej Rj;
        ecmult_gen(Rj, k, gtab);
        fe rx, ry;
        gej_to_ge(rx, ry, Rj);
        sc mm, kinv, s;
        sc_from_be_reduce(mm, d);
        sc_inv_divsteps(kinv, k);
        sc_mul(s, mm, kinv);
        uint32_t rxw[8];
        fe_to_le(rxw, rx);
        if (!sc_ge_n(rxw) && !sc_is_zero(s)) {
            for (int j = 0; j < 8; j++) { store_be32(sig + 4 * j, rxw[7 - j]); store_be32(sig + 32 + 4 * j, s.v[7 - j]); }
            sig[64] = (uint8_t)(ry.n[0] & 1u);
        }
    }
    type_out = (uint8_t)m.type;
    h_out = g.h;
    r_out = g.r;
    vr_out = g.vr;
    for (int j = 0; j < 8; j++) { store_be32(value32 + 4 * j, g.value_be[j]); store_be32(from32 + 4 * j, from_be[j]); }
    for (int j = 0; j < 65; j++) sig65[j] = sig[j];
    return cls;
}

}  // namespace hd
