/*
 * hd_oracle.c -- plain-C CPU restatement of hyperdrive's message
 * authentication path.  TEST INFRASTRUCTURE ONLY: built into
 * oracle/_build/liboracle.so and loaded by tests/ (as the checker) and by
 * bench.py's cpu_baseline leg (as the timed CPU port).  Never linked into the
 * product library.
 *
 * Independent of the device implementation on purpose: 4 x 64-bit limbs with
 * unsigned __int128 (the device code uses 8 x 32-bit limbs), generic Jacobian
 * formulas with explicit special cases, fixed-window exponentiation.
 *
 * Restates (see oracle/hd_pyoracle.py for the full citation list):
 *   - digest preimage + SHA-256: process/message.go:53-78, 165-186, 263-284
 *   - recovery: go-ethereum v1.9.5 crypto/secp256k1 (checkSignature V < 4) ->
 *     libsecp256k1 parse_compact / ecdsa_sig_recover; high-S accepted
 *   - signatory: SHA-256 of the pubkey encoding `compressed` selects:
 *     1 SEC1 compressed (33 B), 0 SEC1 uncompressed (65 B), 2 raw X || Y (64 B),
 *     3 X.Bytes() || Y.Bytes() (Go big.Int minimal encodings, <= 64 B)
 *     [renproject/id v0.4.2]
 *   - membership: procsAllowed at mq/mq.go:49-51
 * Parity anchoring: tests/test_oracle.py (KATs + OpenSSL + pyoracle).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------ sha256 */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(uint32_t st[8], const uint8_t* p) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; i++) {
        uint32_t t1 = h + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

void oracle_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    size_t off = 0;
    for (; off + 64 <= len; off += 64) sha256_block(st, msg + off);
    uint8_t tail[128];
    size_t rem = len - off;
    memset(tail, 0, sizeof tail);
    memcpy(tail, msg + off, rem);
    tail[rem] = 0x80;
    size_t tl = (rem + 9 <= 64) ? 64 : 128;
    uint64_t bits = (uint64_t)len * 8;
    for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha256_block(st, tail);
    if (tl == 128) sha256_block(st, tail + 64);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = st[i] >> 24; out[4 * i + 1] = st[i] >> 16; out[4 * i + 2] = st[i] >> 8; out[4 * i + 3] = st[i];
    }
}

/* ------------------------------------------------------- 256-bit helpers */
typedef struct { uint64_t v[4]; } u256;

static const u256 PP = {{0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL}};
static const u256 NN = {{0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL}};
/* 2^256 - n */
static const uint64_t NC[3] = {0x402DA1732FC9BEBFULL, 0x4551231950B75FC4ULL, 1ULL};
static const u256 GXX = {{0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL, 0x79BE667EF9DCBBACULL}};
static const u256 GYY = {{0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL, 0x483ADA7726A3C465ULL}};

static void u256_from_be(u256* r, const uint8_t* b) {
    for (int i = 0; i < 4; i++) {
        uint64_t x = 0;
        for (int j = 0; j < 8; j++) x = (x << 8) | b[(3 - i) * 8 + j];
        r->v[i] = x;
    }
}
static void u256_to_be(uint8_t* b, const u256* a) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) b[(3 - i) * 8 + j] = (uint8_t)(a->v[i] >> (56 - 8 * j));
}
static int u256_cmp(const u256* a, const u256* b) {
    for (int i = 3; i >= 0; i--) {
        if (a->v[i] != b->v[i]) return a->v[i] < b->v[i] ? -1 : 1;
    }
    return 0;
}
static int u256_is_zero(const u256* a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }
static uint64_t u256_add(u256* r, const u256* a, const u256* b) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) { c += (u128)a->v[i] + b->v[i]; r->v[i] = (uint64_t)c; c >>= 64; }
    return (uint64_t)c;
}
static uint64_t u256_sub(u256* r, const u256* a, const u256* b) {
    uint64_t br = 0;
    for (int i = 0; i < 4; i++) {
        uint64_t x = a->v[i], y = b->v[i];
        uint64_t d = x - y - br;
        br = (x < y) || (x - y < br);
        r->v[i] = d;
    }
    return br;
}
static void mul_256x256(uint64_t t[8], const u256* a, const u256* b) {
    memset(t, 0, 8 * sizeof(uint64_t));
    for (int i = 0; i < 4; i++) {
        u128 c = 0;
        for (int j = 0; j < 4; j++) {
            c += (u128)a->v[i] * b->v[j] + t[i + j];
            t[i + j] = (uint64_t)c;
            c >>= 64;
        }
        t[i + 4] = (uint64_t)c;
    }
}

/* ---------------------------------------------------------- field mod p */
static void fe_norm(u256* r) { if (u256_cmp(r, &PP) >= 0) u256_sub(r, r, &PP); }
static void fe_add(u256* r, const u256* a, const u256* b) {
    if (u256_add(r, a, b)) { u256 c = {{0x1000003D1ULL, 0, 0, 0}}; u256_add(r, r, &c); }
    fe_norm(r);
}
static void fe_sub(u256* r, const u256* a, const u256* b) {
    if (u256_sub(r, a, b)) u256_add(r, r, &PP);
}
static void fe_mul(u256* r, const u256* a, const u256* b) {
    uint64_t t[8];
    mul_256x256(t, a, b);
    uint64_t a5[5];
    u128 c = 0;
    for (int i = 0; i < 4; i++) { c += (u128)t[4 + i] * 0x1000003D1ULL + t[i]; a5[i] = (uint64_t)c; c >>= 64; }
    a5[4] = (uint64_t)c;
    c = (u128)a5[4] * 0x1000003D1ULL + a5[0];
    r->v[0] = (uint64_t)c; c >>= 64;
    for (int i = 1; i < 4; i++) { c += a5[i]; r->v[i] = (uint64_t)c; c >>= 64; }
    if (c) { u256 k = {{0x1000003D1ULL, 0, 0, 0}}; u256_add(r, r, &k); }
    fe_norm(r);
}
static void fe_sqr(u256* r, const u256* a) { fe_mul(r, a, a); }
/* fixed 4-bit window exponentiation, e given big-endian as u256 */
static void fe_pow(u256* r, const u256* a, const u256* e) {
    u256 tab[16];
    tab[0] = (u256){{1, 0, 0, 0}};
    tab[1] = *a;
    for (int i = 2; i < 16; i++) fe_mul(&tab[i], &tab[i - 1], a);
    u256 acc = tab[0];
    for (int i = 63; i >= 0; i--) {
        for (int k = 0; k < 4; k++) fe_sqr(&acc, &acc);
        int d = (int)((e->v[i / 16] >> ((i % 16) * 4)) & 15);
        if (d) fe_mul(&acc, &acc, &tab[d]);
    }
    *r = acc;
}
static void fe_inv(u256* r, const u256* a) {
    u256 e = PP; e.v[0] -= 2;
    fe_pow(r, a, &e);
}

/* --------------------------------------------------------- scalar mod n */
static void sc_reduce512(u256* r, const uint64_t tin[8]) {
    uint64_t t[8];
    memcpy(t, tin, sizeof t);
    while (t[4] | t[5] | t[6] | t[7]) {
        uint64_t u[8] = {0};
        /* u = hi * NC */
        for (int i = 0; i < 4; i++) {
            u128 c = 0;
            for (int j = 0; j < 3; j++) {
                c += (u128)t[4 + i] * NC[j] + u[i + j];
                u[i + j] = (uint64_t)c;
                c >>= 64;
            }
            for (int k = i + 3; c && k < 8; k++) { c += u[k]; u[k] = (uint64_t)c; c >>= 64; }
        }
        /* t = lo + u */
        u128 c = 0;
        for (int i = 0; i < 8; i++) {
            c += (u128)u[i] + (i < 4 ? t[i] : 0);
            t[i] = (uint64_t)c;
            c >>= 64;
        }
    }
    u256 x = {{t[0], t[1], t[2], t[3]}};
    while (u256_cmp(&x, &NN) >= 0) u256_sub(&x, &x, &NN);
    *r = x;
}
static void sc_mul(u256* r, const u256* a, const u256* b) {
    uint64_t t[8];
    mul_256x256(t, a, b);
    sc_reduce512(r, t);
}
static void sc_inv(u256* r, const u256* a) {
    u256 e = NN; e.v[0] -= 2;
    u256 tab[16];
    tab[0] = (u256){{1, 0, 0, 0}};
    tab[1] = *a;
    for (int i = 2; i < 16; i++) sc_mul(&tab[i], &tab[i - 1], a);
    u256 acc = tab[0];
    for (int i = 63; i >= 0; i--) {
        for (int k = 0; k < 4; k++) sc_mul(&acc, &acc, &acc);
        int d = (int)((e.v[i / 16] >> ((i % 16) * 4)) & 15);
        if (d) sc_mul(&acc, &acc, &tab[d]);
    }
    *r = acc;
}
static void sc_neg(u256* r, const u256* a) {
    if (u256_is_zero(a)) { *r = *a; return; }
    u256_sub(r, &NN, a);
}

/* ------------------------------------------------------ Jacobian points */
typedef struct { u256 x, y, z; int inf; } gej;

static void gej_dbl(gej* r, const gej* a) {
    if (a->inf || u256_is_zero(&a->y)) { r->inf = 1; return; }
    u256 A, B, C, D, E, F, t, x3, y3, z3;
    fe_sqr(&A, &a->x);           /* A = X^2 */
    fe_sqr(&B, &a->y);           /* B = Y^2 */
    fe_sqr(&C, &B);              /* C = B^2 */
    fe_add(&t, &a->x, &B);
    fe_sqr(&t, &t);
    fe_sub(&t, &t, &A);
    fe_sub(&t, &t, &C);
    fe_add(&D, &t, &t);          /* D = 2((X+B)^2 - A - C) */
    fe_add(&E, &A, &A);
    fe_add(&E, &E, &A);          /* E = 3A */
    fe_sqr(&F, &E);              /* F = E^2 */
    fe_add(&t, &D, &D);
    fe_sub(&x3, &F, &t);         /* X3 = F - 2D */
    fe_sub(&t, &D, &x3);
    fe_mul(&t, &E, &t);
    u256 c8;
    fe_add(&c8, &C, &C); fe_add(&c8, &c8, &c8); fe_add(&c8, &c8, &c8);
    fe_sub(&y3, &t, &c8);        /* Y3 = E(D - X3) - 8C */
    fe_mul(&z3, &a->y, &a->z);
    fe_add(&z3, &z3, &z3);       /* Z3 = 2YZ */
    r->x = x3; r->y = y3; r->z = z3; r->inf = 0;
}

static void gej_add(gej* r, const gej* a, const gej* b) {
    if (a->inf) { *r = *b; return; }
    if (b->inf) { *r = *a; return; }
    u256 z1z1, z2z2, u1, u2, s1, s2, h, rr, t;
    fe_sqr(&z1z1, &a->z);
    fe_sqr(&z2z2, &b->z);
    fe_mul(&u1, &a->x, &z2z2);
    fe_mul(&u2, &b->x, &z1z1);
    fe_mul(&t, &b->z, &z2z2); fe_mul(&s1, &a->y, &t);
    fe_mul(&t, &a->z, &z1z1); fe_mul(&s2, &b->y, &t);
    fe_sub(&h, &u2, &u1);
    fe_sub(&rr, &s2, &s1);
    if (u256_is_zero(&h)) {
        if (u256_is_zero(&rr)) { gej_dbl(r, a); return; }
        r->inf = 1;
        return;
    }
    u256 hh, hhh, v, x3, y3, z3;
    fe_sqr(&hh, &h);
    fe_mul(&hhh, &hh, &h);
    fe_mul(&v, &u1, &hh);
    fe_sqr(&x3, &rr);
    fe_sub(&x3, &x3, &hhh);
    fe_sub(&x3, &x3, &v);
    fe_sub(&x3, &x3, &v);        /* X3 = r^2 - H^3 - 2 U1 H^2 */
    fe_sub(&t, &v, &x3);
    fe_mul(&t, &rr, &t);
    u256 t2;
    fe_mul(&t2, &s1, &hhh);
    fe_sub(&y3, &t, &t2);        /* Y3 = r (V - X3) - S1 H^3 */
    fe_mul(&z3, &a->z, &b->z);
    fe_mul(&z3, &z3, &h);        /* Z3 = Z1 Z2 H */
    r->x = x3; r->y = y3; r->z = z3; r->inf = 0;
}

/* wNAF recoding, window w; returns length */
static int wnaf(int8_t* out, const u256* k, int w) {
    u256 x = *k;
    int len = 0;
    memset(out, 0, 260);
    while (!u256_is_zero(&x)) {
        int d = 0;
        if (x.v[0] & 1) {
            d = (int)(x.v[0] & ((1u << w) - 1));
            if (d >= (1 << (w - 1))) d -= (1 << w);
            u256 dd = {{(uint64_t)(d < 0 ? -d : d), 0, 0, 0}};
            if (d > 0) u256_sub(&x, &x, &dd); else u256_add(&x, &x, &dd);
        }
        out[len++] = (int8_t)d;
        /* x >>= 1 */
        for (int i = 0; i < 3; i++) x.v[i] = (x.v[i] >> 1) | (x.v[i + 1] << 63);
        x.v[3] >>= 1;
    }
    return len;
}

#define WG 6
#define WR 5
static gej G_TAB[1 << (WG - 2)];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void build_gtab(void) {
    gej g = {GXX, GYY, {{1, 0, 0, 0}}, 0}, g2;
    gej_dbl(&g2, &g);
    G_TAB[0] = g;
    for (int i = 1; i < (1 << (WG - 2)); i++) gej_add(&G_TAB[i], &G_TAB[i - 1], &g2);
}

static void gej_neg(gej* r, const gej* a) {
    *r = *a;
    if (!a->inf) fe_sub(&r->y, &(u256){{0, 0, 0, 0}}, &a->y);
}

/* r = u1*G + u2*R (Strauss-Shamir with wNAF) */
static void ecmult(gej* out, const gej* R, const u256* u1, const u256* u2) {
    pthread_once(&g_once, build_gtab);
    gej rt[1 << (WR - 2)], r2;
    rt[0] = *R;
    gej_dbl(&r2, R);
    for (int i = 1; i < (1 << (WR - 2)); i++) gej_add(&rt[i], &rt[i - 1], &r2);
    int8_t n1[260], n2[260];
    int l1 = wnaf(n1, u1, WG), l2 = wnaf(n2, u2, WR);
    int l = l1 > l2 ? l1 : l2;
    gej acc;
    acc.inf = 1;
    for (int i = l - 1; i >= 0; i--) {
        gej_dbl(&acc, &acc);
        if (n1[i]) {
            gej t;
            if (n1[i] > 0) t = G_TAB[(n1[i] - 1) / 2]; else gej_neg(&t, &G_TAB[(-n1[i] - 1) / 2]);
            gej_add(&acc, &acc, &t);
        }
        if (n2[i]) {
            gej t;
            if (n2[i] > 0) t = rt[(n2[i] - 1) / 2]; else gej_neg(&t, &rt[(-n2[i] - 1) / 2]);
            gej_add(&acc, &acc, &t);
        }
    }
    *out = acc;
}

/* ---------------------------------------------------------- recovery */
enum { V_VALID = 0, V_BAD_RECID, V_BAD_RS, V_NO_POINT, V_INFINITY, V_MISMATCH, V_NOT_ADMITTED, V_BAD_TYPE };

/* returns verdict; on VALID writes x,y of Q (affine) */
static int recover(const uint8_t digest[32], const uint8_t sig[65], u256* qx, u256* qy) {
    uint8_t v = sig[64];
    if (v >= 4) return V_BAD_RECID;
    u256 r, s, m;
    u256_from_be(&r, sig);
    u256_from_be(&s, sig + 32);
    if (u256_cmp(&r, &NN) >= 0 || u256_cmp(&s, &NN) >= 0) return V_BAD_RS;
    if (u256_is_zero(&r) || u256_is_zero(&s)) return V_BAD_RS;
    u256 x = r;
    if (v & 2) {
        u256 pmn;
        u256_sub(&pmn, &PP, &NN);
        if (u256_cmp(&x, &pmn) >= 0) return V_NO_POINT;
        u256_add(&x, &x, &NN);
    }
    u256 y2, y, t, seven = {{7, 0, 0, 0}};
    fe_sqr(&t, &x);
    fe_mul(&t, &t, &x);
    fe_add(&y2, &t, &seven);
    u256 e = PP; /* (p+1)/4 */
    {
        u256 one = {{1, 0, 0, 0}};
        u256_add(&e, &e, &one);
        for (int i = 0; i < 3; i++) e.v[i] = (e.v[i] >> 2) | (e.v[i + 1] << 62);
        e.v[3] >>= 2;
    }
    fe_pow(&y, &y2, &e);
    fe_sqr(&t, &y);
    if (u256_cmp(&t, &y2) != 0) return V_NO_POINT;
    if ((int)(y.v[0] & 1) != (v & 1)) fe_sub(&y, &(u256){{0, 0, 0, 0}}, &y);
    u256_from_be(&m, digest);
    while (u256_cmp(&m, &NN) >= 0) u256_sub(&m, &m, &NN);
    u256 rinv, u1, u2;
    sc_inv(&rinv, &r);
    sc_mul(&u1, &m, &rinv);
    sc_neg(&u1, &u1);
    sc_mul(&u2, &s, &rinv);
    gej R = {x, y, {{1, 0, 0, 0}}, 0}, Q;
    ecmult(&Q, &R, &u1, &u2);
    if (Q.inf) return V_INFINITY;
    u256 zi, zi2, zi3;
    fe_inv(&zi, &Q.z);
    fe_sqr(&zi2, &zi);
    fe_mul(&zi3, &zi2, &zi);
    fe_mul(qx, &Q.x, &zi2);
    fe_mul(qy, &Q.y, &zi3);
    return V_VALID;
}

int oracle_recover(const uint8_t digest[32], const uint8_t sig[65], uint8_t pub65[65]) {
    u256 qx, qy;
    int v = recover(digest, sig, &qx, &qy);
    if (v == V_VALID) {
        pub65[0] = 4;
        u256_to_be(pub65 + 1, &qx);
        u256_to_be(pub65 + 33, &qy);
    }
    return v;
}

static void put_be64(uint8_t* b, int64_t x) {
    uint64_t u = (uint64_t)x;
    for (int i = 0; i < 8; i++) b[i] = (uint8_t)(u >> (56 - 8 * i));
}

/* digest of message (surge preimage + SHA-256) */
void oracle_digest(uint8_t type, int64_t h, int64_t r, int64_t vr, const uint8_t value[32], uint8_t out[32]) {
    uint8_t buf[56];
    put_be64(buf, h);
    put_be64(buf + 8, r);
    if (type == 1) {
        put_be64(buf + 16, vr);
        memcpy(buf + 24, value, 32);
        oracle_sha256(buf, 56, out);
    } else {
        memcpy(buf + 16, value, 32);
        oracle_sha256(buf, 48, out);
    }
}

typedef struct {
    uint32_t n;
    const uint8_t* type;
    const int64_t* height;
    const int64_t* round;
    const int64_t* valid_round;
    const uint8_t* value32;
    const uint8_t* from32;
    const uint8_t* sig65;
    const uint8_t* admitted32; /* sorted ascending */
    uint32_t n_admitted;
    int compressed;
    uint8_t* verdict;
    uint8_t* recovered32;
    uint32_t lo, hi;
} job_t;

static int admitted_has(const job_t* j, const uint8_t* s) {
    uint32_t lo = 0, hi = j->n_admitted;
    while (lo < hi) {
        uint32_t mid = (lo + hi) / 2;
        int c = memcmp(j->admitted32 + 32 * (size_t)mid, s, 32);
        if (c == 0) return 1;
        if (c < 0) lo = mid + 1; else hi = mid;
    }
    return 0;
}

static void* run_job(void* arg) {
    job_t* j = (job_t*)arg;
    for (uint32_t i = j->lo; i < j->hi; i++) {
        uint8_t t = j->type[i];
        uint8_t* rec = j->recovered32 ? j->recovered32 + 32 * (size_t)i : NULL;
        if (rec) memset(rec, 0, 32);
        if (t < 1 || t > 3) { j->verdict[i] = V_BAD_TYPE; continue; }
        uint8_t d[32];
        oracle_digest(t, j->height[i], j->round[i], j->valid_round ? j->valid_round[i] : -1,
                      j->value32 + 32 * (size_t)i, d);
        u256 qx, qy;
        int v = recover(d, j->sig65 + 65 * (size_t)i, &qx, &qy);
        if (v != V_VALID) { j->verdict[i] = (uint8_t)v; continue; }
        uint8_t pk[65], sg[32];
        size_t pl;
        if (j->compressed == 1) {
            pk[0] = 2 | (uint8_t)(qy.v[0] & 1);
            u256_to_be(pk + 1, &qx);
            pl = 33;
        } else if (j->compressed == 2) {
            u256_to_be(pk, &qx);
            u256_to_be(pk + 32, &qy);
            pl = 64;
        } else if (j->compressed == 3) {
            /* Go big.Int.Bytes(): minimal big-endian, leading zero bytes dropped */
            uint8_t xb[32], yb[32];
            size_t zx = 0, zy = 0;
            u256_to_be(xb, &qx);
            u256_to_be(yb, &qy);
            while (zx < 32 && xb[zx] == 0) zx++;
            while (zy < 32 && yb[zy] == 0) zy++;
            memcpy(pk, xb + zx, 32 - zx);
            memcpy(pk + 32 - zx, yb + zy, 32 - zy);
            pl = 64 - zx - zy;
        } else {
            pk[0] = 4;
            u256_to_be(pk + 1, &qx);
            u256_to_be(pk + 33, &qy);
            pl = 65;
        }
        oracle_sha256(pk, pl, sg);
        if (rec) memcpy(rec, sg, 32);
        if (memcmp(sg, j->from32 + 32 * (size_t)i, 32) != 0) { j->verdict[i] = V_MISMATCH; continue; }
        if (!admitted_has(j, sg)) { j->verdict[i] = V_NOT_ADMITTED; continue; }
        j->verdict[i] = V_VALID;
    }
    return NULL;
}

static int cmp32(const void* a, const void* b) { return memcmp(a, b, 32); }

/* Verify [0, n) on nthreads host threads.  admitted32 need not be sorted. */
int oracle_verify_batch(uint32_t n, const uint8_t* type, const int64_t* height, const int64_t* round,
                        const int64_t* valid_round, const uint8_t* value32, const uint8_t* from32,
                        const uint8_t* sig65, const uint8_t* admitted32, uint32_t n_admitted, int compressed,
                        uint8_t* verdict, uint8_t* recovered32, int nthreads) {
    pthread_once(&g_once, build_gtab);
    uint8_t* adm = (uint8_t*)malloc(32 * (size_t)(n_admitted ? n_admitted : 1));
    if (!adm) return -1;
    if (n_admitted) memcpy(adm, admitted32, 32 * (size_t)n_admitted);
    qsort(adm, n_admitted, 32, cmp32);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    job_t jobs[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; t++) {
        job_t* j = &jobs[t];
        j->n = n; j->type = type; j->height = height; j->round = round; j->valid_round = valid_round;
        j->value32 = value32; j->from32 = from32; j->sig65 = sig65; j->admitted32 = adm;
        j->n_admitted = n_admitted; j->compressed = compressed; j->verdict = verdict; j->recovered32 = recovered32;
        j->lo = (uint32_t)((uint64_t)n * t / nthreads);
        j->hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
    }
    for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, run_job, &jobs[t]);
    run_job(&jobs[0]);
    for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
    free(adm);
    return 0;
}

/* ---- tally + quorum decisions (process/process.go) ---------------------
 * TEST INFRASTRUCTURE / CPU baseline: the first-wins vote logs of
 * insertPrevote / insertPrecommit (process.go:823-892) over the VALID
 * Prevotes / Precommits in batch order, and the counts the 2f+1 / f+1 rules
 * read (process.go:486-494, 534, 574-582, 626-632, 658, 696-702, 751):
 *   counts  (h, r, type, value) -> number of first-wins votes, rows in order of
 *           the group's first logged vote (rep)
 *   hr      (h, r) -> len(PrevoteLogs[r]), len(PrecommitLogs[r]), distinct vote
 *           signers, rep = the first candidate of the round
 *   decide  per hr row, with f and the propose value `pv` (32 B per hr row,
 *           NULL: none): bit 0 L34 timeout_prevote, 1 L44 precommit_nil, 2
 *           L47 reached (>=), 3 L47 exact (==), 4 L55 skip (no propose signer),
 *           5 L36 precommit_value, 6 L49 commit -- hyperdrive_amd.quorum.decide
 * Open-addressing tables keyed by batch index (keys compared in the batch). */
typedef struct {
    uint32_t* slot;
    uint32_t mask;
} otab_t;

static uint64_t omix(uint64_t x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull; x ^= x >> 31;
    return x;
}
static uint64_t ohash_bytes(const uint8_t* p, size_t n, uint64_t h) {
    for (size_t k = 0; k + 8 <= n; k += 8) {
        uint64_t w;
        memcpy(&w, p + k, 8);
        h = omix(h ^ w);
    }
    return h;
}

typedef struct {
    const uint8_t* type; const int64_t* h; const int64_t* r; const uint8_t* value; const uint8_t* from;
} obatch_t;

/* mode 0: (h, r); 1: (h, r, type, from); 2: (h, r, from); 3: (h, r, type, value) */
static uint64_t okey_hash(const obatch_t* b, uint32_t i, int mode) {
    uint64_t x = omix((uint64_t)b->h[i] * 0x9E3779B97F4A7C15ull ^ omix((uint64_t)b->r[i]) ^ (uint64_t)mode << 60);
    if (mode == 1 || mode == 3) x = omix(x ^ b->type[i]);
    if (mode == 1 || mode == 2) x = ohash_bytes(b->from + 32 * (size_t)i, 32, x);
    if (mode == 3) x = ohash_bytes(b->value + 32 * (size_t)i, 32, x);
    return x;
}
static int okey_eq(const obatch_t* b, uint32_t i, uint32_t j, int mode) {
    if (b->h[i] != b->h[j] || b->r[i] != b->r[j]) return 0;
    if ((mode == 1 || mode == 3) && b->type[i] != b->type[j]) return 0;
    if ((mode == 1 || mode == 2) && memcmp(b->from + 32 * (size_t)i, b->from + 32 * (size_t)j, 32)) return 0;
    if (mode == 3 && memcmp(b->value + 32 * (size_t)i, b->value + 32 * (size_t)j, 32)) return 0;
    return 1;
}
/* the slot of i's key: its first index there, *fresh = 1 when i created it */
static uint32_t ofind(otab_t* t, const obatch_t* b, uint32_t i, int mode, int* fresh) {
    uint32_t s = (uint32_t)okey_hash(b, i, mode) & t->mask;
    for (;;) {
        uint32_t c = t->slot[s];
        if (c == 0xFFFFFFFFu) { t->slot[s] = i; *fresh = 1; return s; }
        if (okey_eq(b, i, c, mode)) { *fresh = 0; return s; }
        s = (s + 1) & t->mask;
    }
}

int oracle_tally(uint32_t n, const uint8_t* type, const int64_t* height, const int64_t* round, const uint8_t* value32,
                 const uint8_t* from32, const uint8_t* verdict, uint32_t f, const uint8_t* pv_by_hr,
                 int64_t* counts /* 5 x n: h r type rep n (row-major) */, uint32_t* n_counts,
                 int64_t* hr /* 6 x n: h r prevotes precommits any rep */, uint32_t* n_hr, uint8_t* decide) {
    obatch_t b = {type, height, round, value32, from32};
    uint32_t cap = 1024;
    while (cap < 2 * (uint64_t)n + 2) cap <<= 1;
    otab_t T[4];
    uint32_t* row_of[4];
    for (int k = 0; k < 4; k++) {
        T[k].slot = (uint32_t*)malloc(4 * (size_t)cap);
        row_of[k] = (uint32_t*)malloc(4 * (size_t)cap);
        if (!T[k].slot || !row_of[k]) return -1;
        memset(T[k].slot, 0xFF, 4 * (size_t)cap);
        T[k].mask = cap - 1;
    }
    uint32_t nh = 0, nc = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (verdict[i] != 0 || (type[i] != 2 && type[i] != 3)) continue;
        int fresh;
        uint32_t s = ofind(&T[0], &b, i, 0, &fresh);
        if (fresh) {
            int64_t* o = hr + 6 * (size_t)nh;
            o[0] = height[i]; o[1] = round[i]; o[2] = o[3] = o[4] = 0; o[5] = i;
            row_of[0][s] = nh++;
        }
        int64_t* g = hr + 6 * (size_t)row_of[0][s];
        ofind(&T[1], &b, i, 1, &fresh);          /* first wins per (h, r, type, From) */
        if (!fresh) continue;
        g[type[i] == 2 ? 2 : 3]++;
        ofind(&T[2], &b, i, 2, &fresh);          /* distinct signers of the round */
        if (fresh) g[4]++;
        s = ofind(&T[3], &b, i, 3, &fresh);
        if (fresh) {
            int64_t* o = counts + 5 * (size_t)nc;
            o[0] = height[i]; o[1] = round[i]; o[2] = type[i]; o[3] = i; o[4] = 0;
            row_of[3][s] = nc++;
        }
        counts[5 * (size_t)row_of[3][s] + 4]++;
    }
    *n_counts = nc;
    *n_hr = nh;
    if (decide) {
        /* count of (h, r, type, value v) by probing T[3] with a scratch key */
        const int64_t q = 2 * (int64_t)f + 1;
        static const uint8_t nil[32] = {0};
        for (uint32_t k = 0; k < nh; k++) {
            const int64_t* g = hr + 6 * (size_t)k;
            int64_t cnt[3] = {0, 0, 0};   /* prevotes nil, prevotes pv, precommits pv */
            const uint8_t* pv = pv_by_hr ? pv_by_hr + 32 * (size_t)k : NULL;
            for (int c = 0; c < 3; c++) {
                const uint8_t* val = c == 0 ? nil : pv;
                const uint8_t ty = c == 2 ? 3 : 2;
                if (!val) continue;
                /* a one-message batch view holding the probe key */
                int64_t hh = g[0], rr = g[1];
                uint8_t tt = ty;
                obatch_t kb = {&tt, &hh, &rr, val, from32};
                uint32_t s = (uint32_t)okey_hash(&kb, 0, 3) & T[3].mask;
                for (;;) {
                    uint32_t e = T[3].slot[s];
                    if (e == 0xFFFFFFFFu) break;
                    if (height[e] == hh && round[e] == rr && type[e] == ty && !memcmp(value32 + 32 * (size_t)e, val, 32)) {
                        cnt[c] = counts[5 * (size_t)row_of[3][s] + 4];
                        break;
                    }
                    s = (s + 1) & T[3].mask;
                }
            }
            uint8_t d = 0;
            d |= (g[2] >= q) << 0;
            d |= (cnt[0] >= q) << 1;
            d |= (g[3] >= q) << 2;
            d |= (g[3] == q) << 3;
            d |= (g[4] >= (int64_t)f + 1) << 4;
            if (pv) {
                d |= (cnt[1] >= q) << 5;
                d |= (cnt[2] >= q) << 6;
            }
            decide[k] = d;
        }
    }
    for (int k = 0; k < 4; k++) { free(T[k].slot); free(row_of[k]); }
    return 0;
}
