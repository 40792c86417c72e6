// hd_fixedbase.h -- verification against a known public key with fixed-base
// tables (the fast path of k_verify; DESIGN.md §4 "Known-key fast path").
//
// The reference authenticates a message by recovering the public key Q from
// (digest, r, s, v) and comparing SHA-256(Q) with the claimed From
// (libsecp256k1 recover; process/message_test.go:147-154).
// Once a signatory's public key P is known -- learned from a message of that
// signatory that verified VALID through the full recovery, so SHA-256(P) is
// its signatory -- a message claiming that From is VALID iff its recovered key
// is P, i.e. iff
//
//     R == s^-1 (m G + r P)        R = lift(r [+ n], v & 1), m = digest mod n
//
// (then Q = r^-1 (s R - m G) = P).  Both scalar multiplications have fixed
// bases, so they run without doublings over per-base tables of W-bit Booth
// windows: entry (j, d) = d 2^(W j) B for 1 <= d <= 2^(W-1), and each signed
// digit costs one mixed addition (W = 16: 16 windows, 32 additions per
// message for the two scalars, 36 MB of affine points per base).  No square
// root is needed: the affine result is compared with x and the parity of y.
//
// verify_fast returns V_VALID only when that identity holds, an exact early
// verdict (BAD_RECID, BAD_RS, NO_POINT for r + n >= p) where the reference's
// first checks decide, and HD_NEEDS_SLOW otherwise; the caller then runs the
// full recovery, which yields the reference verdict and recovered signatory.
#pragma once
#include "hd_group.h"

namespace hd {

#ifndef HD_FB_W
#define HD_FB_W 16    // per-key tables: 16 windows, 15 x 32768 + 65536 points (36 MB)
#endif
#ifndef HD_FB_WW
#define HD_FB_WW 20   // wide per-key tables: 13 windows, 12 x 2^19 + 2^16 points (407 MB), when the budget holds them
#endif
#ifndef HD_FB_WX
#define HD_FB_WX 22   // widest per-key tables: 12 windows, 11 x 2^21 + 2^14 points (1.48 GB), when every admitted
                      // key's fits the device's budget (round 6: one addition fewer than 20-bit, -4 % k_fast_sums)
#endif
#ifndef HD_FB_WN
#define HD_FB_WN 13   // narrow per-key tables: 20 windows, 19 x 4096 + 512 points (5.0 MB), when even the 16-bit
                      // tables of every admitted key exceed the budget (thousands of signatories)
#endif
#ifndef HD_FB_WG
#define HD_FB_WG 24   // the one shared G table: 11 windows, 10 x 2^23 + 2^16 points (6.0 GB)
#endif

// Windows 0 .. NWIN-2 take signed Booth digits |d| <= 2^(W-1); the top window
// takes the remaining TOPBITS bits plus the Booth carry unsigned,
// 0 <= d <= 2^TOPBITS, so no extra window is spent on the carry.  Entry
// (j, d) of a base B is d 2^(W j) B at index j N + d - 1.
template <int W>
struct FbL {
    static constexpr int NWIN = (256 + W - 1) / W;
    static constexpr uint32_t N = 1u << (W - 1);
    static constexpr int TOPBITS = 256 - W * (NWIN - 1);
    static constexpr uint32_t NTOP = 1u << TOPBITS;
    static constexpr uint32_t TAB = (uint32_t)(NWIN - 1) * N + NTOP;   // affine entries per base
};
#define HD_FB_NWIN (FbL<HD_FB_W>::NWIN)
#define HD_FB_N (FbL<HD_FB_W>::N)
#define HD_FB_TAB (FbL<HD_FB_W>::TAB)
#define HD_NEEDS_SLOW 0xFEu

// The foreign-key dictionary (HD_VAR_FOREIGN_KEYS): Froms outside the
// admitted set whose key a NOT_ADMITTED recovery has shown, each with a table
// slot.  HD_FD_BUCKETS buckets, linear probing over at most 8: words
// [0, B) claim (0 empty, 1 being written, 2 written), [B, 2B) slot (or
// 0xFFFFFFFF: no slot was left), then 8 big-endian From words per bucket.
#define HD_FD_BUCKETS 128u
#define HD_FD_WORDS (10u * HD_FD_BUCKETS)
HD uint32_t fdict_bucket(const uint32_t w[8]) {
    return (w[0] ^ (w[3] * 0x9E3779B1u) ^ (w[7] * 0x85EBCA77u)) & (HD_FD_BUCKETS - 1u);
}
// slot of a known foreign From, or -1
HD int32_t fdict_find(const uint32_t* fd, const uint32_t from_be[8]) {
    uint32_t b = fdict_bucket(from_be);
    for (int p = 0; p < 8; p++, b = (b + 1u) & (HD_FD_BUCKETS - 1u)) {
        const uint32_t c = fd[b];
        if (c == 0u) return -1;
        if (c != 2u) continue;
        uint32_t diff = 0;
        HD_UNROLL for (int w = 0; w < 8; w++) diff |= fd[2u * HD_FD_BUCKETS + 8u * b + w] ^ from_be[w];
        if (!diff) {
            const uint32_t s = fd[HD_FD_BUCKETS + b];
            return s == 0xFFFFFFFFu ? -1 : (int32_t)s;
        }
    }
    return -1;
}

// The dictionary rebuilt on the host (fb_evict) from n entries in priority
// order -- slot holders first, then the slotless Froms worth keeping:
// nd (HD_FD_WORDS words, zeroed here) gets each entry in the first free
// bucket of its probe run, where[k] its bucket (-1: dropped).  A slotless
// entry without a free bucket within the 8 probes is dropped; a slot holder
// without one makes the rebuild fail (returns false): dropping it would
// leave its slot READY / LEARNED with no From mapping to it, lost to every
// later pass, so the caller keeps the old dictionary instead.
inline bool fdict_rebuild(uint32_t* nd, int32_t* where, const uint32_t* ent_from_be, const uint32_t* ent_slot,
                          uint32_t n) {
    for (uint32_t w = 0; w < HD_FD_WORDS; w++) nd[w] = 0u;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t* from = ent_from_be + 8 * (size_t)k;
        uint32_t b = fdict_bucket(from);
        int p = 0;
        for (; p < 8 && nd[b] != 0u; p++) b = (b + 1u) & (HD_FD_BUCKETS - 1u);
        if (p == 8) {
            if (ent_slot[k] != 0xFFFFFFFFu) return false;
            where[k] = -1;
            continue;
        }
        nd[b] = 2u;
        nd[HD_FD_BUCKETS + b] = ent_slot[k];
        for (int w = 0; w < 8; w++) nd[2u * HD_FD_BUCKETS + 8u * b + w] = from[w];
        where[k] = (int32_t)b;
    }
    return true;
}

// slot states of the per-signatory tables (device memory, hd_fastverify.hip)
#define HD_FB_EMPTY 0u     // no key known
#define HD_FB_CLAIMED 1u   // a recovering lane is writing the key
#define HD_FB_LEARNED 2u   // key known, tables not built yet
#define HD_FB_READY 3u     // tables built

// A table point as the device stores it: canonical affine coordinates as 8
// little-endian words each, 64 B aligned -- one 64-B HBM access per random
// read instead of the two or three a 72-B radix-2^29 entry straddles.  The
// reader unpacks to radix 2^29 (a few shifts per limb).
struct alignas(64) gp {
    uint32_t x[8], y[8];
};
HD void gp_pack(gp& o, const ge& a) {   // a canonical (gej_to_ge output)
    fe_to_le(o.x, a.x);
    fe_to_le(o.y, a.y);
}
HD void gp_unpack(ge& o, const gp& a) {
    fe_from_le(o.x, a.x);
    fe_from_le(o.y, a.y);
}
// a packed table read as affine points (fb_accumulate / verify_fast2 take any
// indexable table)
struct GpTab {
    const gp* p;
    HD_MEMBER ge operator[](size_t i) const {
        const gp v = p[i];
        ge o;
        gp_unpack(o, v);
        return o;
    }
    HD_MEMBER GpTab operator+(size_t k) const { return GpTab{p + k}; }
};

// a + b for a finite Jacobian a and an affine b, with no exceptional cases:
// the madd of gej_add_ge (8M + 3S, Z3 = 2 Z1 H) without its a = inf and
// a = +-b branches.  If a = +-b then H = 0 and Z3 = 0, and since every later
// Z is a multiple of this one the sum ends with Z = 0: verify_fast then
// hands the message to the full recovery, so no answer depends on it.
HD void gej_add_ge_nx(gej& r, const gej& a, const ge& b) {
    HD_REQUIRE_T(a.x, "gej_add_ge_nx: x");
    HD_REQUIRE_T(a.y, "gej_add_ge_nx: y");
    HD_REQUIRE_T(a.z, "gej_add_ge_nx: z");
    HD_REQUIRE_T(b.x, "gej_add_ge_nx: b.x");
    fe z1z1, u2, s2, h, R, t;
    fe_sqr(z1z1, a.z);         // T
    fe_mul(u2, b.x, z1z1);     // T
    fe_mul(s2, b.y, a.z);      // T (2T x T)
    fe_mul(s2, s2, z1z1);      // T
    fe_sub_k<2>(h, u2, a.x);
    fe_norm_weak(h);           // H = U2 - X1       T
    fe_sub_k<2>(R, s2, a.y);   // r = S2 - Y1       3T
    gej o;
    fe_add(t, a.z, a.z);
    fe_mul(o.z, t, h);         // Z3 = 2 Z1 H       T
    fe hh, i4, j, v;
    fe_norm_weak(R);
    fe_add(R, R, R);           // 2r                2T
    fe_sqr(hh, h);             // T
    fe_mul_int(i4, hh, 4);     // I = 4 H^2         4T
    fe_mul(j, h, i4);          // J = H I           T
    fe_mul(v, a.x, i4);        // V = X1 I          T
    fe_sqr(o.x, R);            // T
    fe_add(t, v, v);
    fe_add(t, t, j);           // 2V + J            3T
    fe_sub_k<4>(o.x, o.x, t);
    fe_norm_weak(o.x);         // X3                T
    fe_sub_k<2>(t, v, o.x);    // V - X3            3T
    fe_mul(t, R, t);           // r (V - X3)        T (2T x 3T)
    fe_mul(j, a.y, j);
    fe_add(j, j, j);           // 2 Y1 J            2T
    fe_sub_k<3>(o.y, t, j);
    fe_norm_weak(o.y);         // Y3                T
    r = o;
}

// a + b for two affine points, no exceptional cases: gej_add_ge_nx with
// Z1 = 1 (Z1Z1 = 1, U2 = X2, S2 = Y2), 4M + 2S instead of 8M + 3S -- the
// first addition of a fixed-base sum, whose accumulator is still the first
// window's table point.  a = +-b gives Z3 = 0, like gej_add_ge_nx.
HD void gej_add_ge_z1(gej& r, const ge& a, const ge& b) {
    HD_REQUIRE_T(a.x, "gej_add_ge_z1: a.x");
    HD_REQUIRE_T(a.y, "gej_add_ge_z1: a.y");
    HD_REQUIRE_T(b.x, "gej_add_ge_z1: b.x");
    fe h, R, t;
    fe_sub_k<2>(h, b.x, a.x);
    fe_norm_weak(h);           // H = X2 - X1       T
    fe_sub_k<2>(R, b.y, a.y);  // r = Y2 - Y1       3T (b.y <= 2T)
    gej o;
    fe_add(o.z, h, h);
    fe_norm_weak(o.z);         // Z3 = 2 H          T
    fe hh, i4, j, v;
    fe_norm_weak(R);
    fe_add(R, R, R);           // 2r                2T
    fe_sqr(hh, h);             // T
    fe_mul_int(i4, hh, 4);     // I = 4 H^2         4T
    fe_mul(j, h, i4);          // J = H I           T
    fe_mul(v, a.x, i4);        // V = X1 I          T
    fe_sqr(o.x, R);            // T
    fe_add(t, v, v);
    fe_add(t, t, j);           // 2V + J            3T
    fe_sub_k<4>(o.x, o.x, t);
    fe_norm_weak(o.x);         // X3                T
    fe_sub_k<2>(t, v, o.x);    // V - X3            3T
    fe_mul(t, R, t);           // r (V - X3)        T (2T x 3T)
    fe_mul(j, a.y, j);
    fe_add(j, j, j);           // 2 Y1 J            2T
    fe_sub_k<3>(o.y, t, j);
    fe_norm_weak(o.y);         // Y3                T
    r = o;
}

// ---- XYZZ sums (k_fast_sums) ------------------------------------------------
// The known-key check's fixed-base sums accumulate in XYZZ coordinates
// ("extended Jacobian"): x = X / ZZ, y = Y / ZZZ with ZZ^3 = ZZZ^2, and
// ZZ = 0 for infinity.  A mixed addition is 8M + 2S
// (madd-2008-s) against 8M + 3S for Jacobian (gej_add_ge_nx), and the loop
// carries X and Y unnormalised (limb classes below), which saves two weak
// normalisations per addition as well.  The sum leaves the loop as
// (X ZZZ, Y ZZ, ZZ ZZZ): one inversion w of the last gives x = X ZZZ w and
// y = Y ZZ w (xz_finish / fast_final_xz).
//
// Limb classes (hd_field.h): X <= 5T, Y <= 3T, ZZ and ZZZ tight; the table
// point's x is T and its y T or 2T (negated).  tests/test_field_bounds.py
// certifies every step for all inputs of these classes.
struct gxz { fe x, y, zz, zzz; };

HD void gxz_set_ge(gxz& r, const ge& a) {
    r.x = a.x;
    r.y = a.y;
    fe_set_u32(r.zz, 1);
    fe_set_u32(r.zzz, 1);
}
HD void gxz_cmov(gxz& r, const gxz& a, bool flag) {
    fe_cmov(r.x, a.x, flag);
    fe_cmov(r.y, a.y, flag);
    fe_cmov(r.zz, a.zz, flag);
    fe_cmov(r.zzz, a.zzz, flag);
}
HD bool gxz_is_inf(const gxz& a) { return fe_is_zero(a.zz); }

// X3, Y3 of both XYZZ additions from P, R and X1, Y1 (the shared tail):
// X3 = R^2 - PPP - 2Q, Y3 = R (Q - X3) - Y1 PPP with Q = X1 PP.  zz / zzz:
// ZZ1 and ZZZ1 (in: nullptr for an affine a), multiplied by PP and PPP as
// soon as those exist, so that ZZ1 and ZZZ1 die early (k_fast_sums runs at
// 168 VGPRs for 3 waves per SIMD).
HD void gxz_add_tail(gxz& o, const fe& x1, const fe& y1, const fe& p, const fe& R, const fe* zz1, const fe* zzz1) {
    fe pp, ppp, q, t;
    fe_sqr(pp, p);             // PP               T
    fe_mul(q, x1, pp);         // Q = X1 PP        T (5T x T)
    fe_mul(ppp, p, pp);        // PPP              T
    if (zz1) {
        fe_mul(o.zz, *zz1, pp);       // ZZ3 = ZZ1 PP      T
        fe_mul(o.zzz, *zzz1, ppp);    // ZZZ3 = ZZZ1 PPP   T
    } else {
        o.zz = pp;
        o.zzz = ppp;
    }
    fe_sqr(o.x, R);            // R^2              T
    fe_add(t, q, q);
    fe_add(t, t, ppp);         // 2Q + PPP         3T
    fe_sub_k<4>(o.x, o.x, t);  // X3               5T
    fe_sub_k<6>(t, q, o.x);    // Q - X3           7T
    fe_mul(t, R, t);           // R (Q - X3)       T (T x 7T)
    fe_mul(q, y1, ppp);        // Y1 PPP           T (3T x T)
    fe_sub_k<2>(o.y, t, q);    // Y3               3T
}

// a + b for a finite XYZZ a and an affine b, no exceptional branches: if
// a = +-b then P = 0, so ZZ3 = ZZZ3 = 0 and every later ZZ is a multiple of
// it; the sum ends with ZZ = 0 and the message takes the full recovery, as
// with gej_add_ge_nx.
HD void gxz_add_ge_nx(gxz& r, const gxz& a, const ge& b) {
    fe u2, s2, p, R;
    fe_mul(u2, b.x, a.zz);     // U2 = X2 ZZ1      T
    fe_mul(s2, b.y, a.zzz);    // S2 = Y2 ZZZ1     T (2T x T)
    fe_sub_k<6>(p, u2, a.x);
    fe_norm_weak(p);           // P = U2 - X1      T
    fe_sub_k<4>(R, s2, a.y);
    fe_norm_weak(R);           // R = S2 - Y1      T
    gxz o;
    gxz_add_tail(o, a.x, a.y, p, R, &a.zz, &a.zzz);
    r = o;
}

// a + b for two affine points (a.y weakly normalised, b.y T or 2T): ZZ1 =
// ZZZ1 = 1, 4M + 2S; a = +-b gives ZZ3 = 0 like gxz_add_ge_nx.
HD void gxz_add_ge_z1(gxz& r, const ge& a, const ge& b) {
    fe p, R;
    fe_sub_k<2>(p, b.x, a.x);
    fe_norm_weak(p);           // P = X2 - X1      T
    fe_sub_k<2>(R, b.y, a.y);
    fe_norm_weak(R);           // R = Y2 - Y1      T
    gxz o;
    gxz_add_tail(o, a.x, a.y, p, R, nullptr, nullptr);
    r = o;
}

// Keeps a wavefront-uniform branch a branch (the compiler would otherwise
// turn a short guarded block into selects that every caller executes).
HD void hd_branch_barrier() {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" ::: "memory");
#endif
}

// One window step of k_fast_sums (and of its host check,
// tests/native/hd_host_check.cpp hdh_xyzz_sum): dst = src + the window's
// table point g (negated when neg); FIRST: src is still the first window's
// affine point p0, so the affine + affine formula applies.  The kernel
// alternates two accumulators (dst and src swap roles every step), so the
// addition never overwrites its own inputs: the compiler schedules it more
// freely than an in-place update (measured ~2 % faster), and the old sum is
// still at hand for the rare repair.  `rare` (the kernel: some lane of the
// wavefront has a zero digit, nz false, or a sum not yet started) runs the
// repair in a branch of its own:
//  * a zero digit's lane keeps the old sum (it added the window's entry 0,
//    read in its place);
//  * a lane whose sum had not started starts it at the window's point.
template <bool FIRST>
HD void gxz_sum_step(gxz& dst, const gxz& src, bool& started, const ge& p0, const ge& g, bool neg, bool nz,
                     bool rare) {
    ge cur = g;
    if (neg) fe_neg(cur.y, g.y);
    if (FIRST) gxz_add_ge_z1(dst, p0, cur);
    else gxz_add_ge_nx(dst, src, cur);
    if (rare) {
        hd_branch_barrier();
        gxz first;
        gxz_cmov(dst, src, !nz);
        gxz_set_ge(first, cur);
        fe_norm_weak(first.y);
        gxz_cmov(dst, first, !started);
        started = started || nz;
    }
}

// the sum as k_fast_sums stores it: X ZZZ, Y ZZ and the value to invert, ZZ ZZZ
HD void gxz_finish(fe& xn, fe& yn, fe& t, const gxz& a) {
    fe_mul(xn, a.x, a.zzz);
    fe_mul(yn, a.y, a.zz);
    fe_mul(t, a.zz, a.zzz);
}

// Booth digit j of u for the table width: bits [W j - 1, W j + W - 1] of u
// (bits outside [0, 256) read 0).  The words are picked with selects over
// the 8 limbs instead of a runtime array index, which would put u in scratch.
HD uint32_t sc_word_sel(const sc& k, int w) {
    uint32_t o = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) o = (w == i) ? k.v[i] : o;
    return o;
}
template <int W>
HD int fb_digit(const sc& k, int j) {
    const int lo = W * j - 1;                       // lowest bit of the window (may be -1)
    const int wlo = lo < 0 ? 0 : (lo >> 5);
    const uint32_t a = sc_word_sel(k, wlo), b = sc_word_sel(k, wlo + 1);   // b = 0 past the top
    const uint64_t pair = ((uint64_t)b << 32) | a;
    const uint32_t m = (1u << (W + 1)) - 1;
    const uint32_t x = lo < 0 ? (uint32_t)(pair << 1) & m : (uint32_t)(pair >> (lo & 31)) & m;
    if (j == FbL<W>::NWIN - 1) return (int)((x >> 1) + (x & 1));   // top window: unsigned, bits past 255 are 0
    return (int)((x >> 1) + (x & 1)) - (int)((x >> W) << W);
}
// table entry (window, multiple) of entry number e (builder side)
template <int W>
HD void fb_entry_pos(uint32_t e, int& j, uint32_t& d) {
    const uint32_t jj = e / FbL<W>::N;
    j = (int)(jj < (uint32_t)(FbL<W>::NWIN - 1) ? jj : (uint32_t)(FbL<W>::NWIN - 1));
    d = e - (uint32_t)j * FbL<W>::N + 1;
}

// acc += u B over the base's HD_FB_TAB entries.  `started` is false while acc
// is still the point at infinity (no non-zero digit yet); the first non-zero
// digit sets acc to its table point.  The next window's point is loaded
// before the current addition, so its HBM latency hides under the math.
template <int W, typename Tab>
HD void fb_accumulate(gej& acc, bool& started, const sc& u, Tab tab) {
    int d = fb_digit<W>(u, 0);
    ge t = tab[(d < 0 ? -d : d) == 0 ? 0 : (d < 0 ? -d : d) - 1];
    HD_NOUNROLL for (int j = 0; j < FbL<W>::NWIN; j++) {
        ge cur = t;
        const int dc = d;
        if (j + 1 < FbL<W>::NWIN) {
            d = fb_digit<W>(u, j + 1);
            const int ad = d < 0 ? -d : d;
            t = tab[(j + 1) * FbL<W>::N + (ad == 0 ? 0 : ad - 1)];
        }
        if (dc < 0) fe_neg(cur.y, cur.y);
        gej s;
        gej_add_ge_nx(s, acc, cur);
        gej first;
        gej_set_ge(first, cur);
        fe_norm_weak(first.y);
        gej_cmov(s, first, !started);
        gej_cmov(acc, s, dc != 0);
        started = started || dc != 0;
    }
}

// The reference's first checks (recover, SURVEY Appendix A items 2-4 up to
// the lift): V >= 4, r / s range, r + n >= p.  On success x = r (+ n) as a
// canonical field element and r, s as scalars; returns V_VALID to continue.
HD uint8_t sig_prefix(sc& r, sc& s, fe& x, const uint32_t r_be[8], const uint32_t s_be[8], uint32_t v) {
    if (v >= 4) return V_BAD_RECID;
    HD_UNROLL for (int i = 0; i < 8; i++) { r.v[i] = r_be[7 - i]; s.v[i] = s_be[7 - i]; }
    if (sc_ge_n(r.v) || sc_ge_n(s.v)) return V_BAD_RS;
    if (sc_is_zero(r) || sc_is_zero(s)) return V_BAD_RS;
    uint32_t xw[8];
    HD_UNROLL for (int i = 0; i < 8; i++) xw[i] = r.v[i];
    if (v & 2) {
        // r + n < p  <=>  r < p - n = 0x14551231950B75FC4402DA1722FC9BAEE
        const uint32_t PMN[8] = {0x2FC9BAEEu, 0x402DA172u, 0x50B75FC4u, 0x45512319u, 1u, 0u, 0u, 0u};
        bool lt = false, gt = false;
        HD_UNROLL for (int i = 7; i >= 0; i--) {
            const bool g = !lt && !gt && r.v[i] > PMN[i];
            const bool l = !lt && !gt && r.v[i] < PMN[i];
            gt = gt || g;
            lt = lt || l;
        }
        if (!lt) return V_NO_POINT;
        const uint32_t N[8] = {HD_N0, HD_N1, HD_N2, HD_N3, HD_N4, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        uint64_t c = 0;
        HD_UNROLL for (int i = 0; i < 8; i++) { c += (uint64_t)xw[i] + N[i]; xw[i] = (uint32_t)c; c >>= 32; }
    }
    fe_from_le(x, xw);
    return V_VALID;
}

// VALID iff lift(r [+n], v & 1) == s^-1 (m G + r P); see the header comment.
template <typename GT, typename PT>
HD uint8_t verify_fast(const uint32_t digest_be[8], const uint32_t r_be[8], const uint32_t s_be[8], uint32_t v,
                       GT gtab, PT ptab) {
    sc r, s;
    fe x;
    const uint8_t pre = sig_prefix(r, s, x, r_be, s_be, v);
    if (pre != V_VALID) return pre;
    sc m, sinv, u1, u2;
    sc_from_be_reduce(m, digest_be);
    sc_inv_divsteps(sinv, s);
    sc_mul(u1, m, sinv);
    sc_mul(u2, r, sinv);
    gej acc;
    gej_set_inf(acc);
    bool started = false;
    fb_accumulate<HD_FB_WG>(acc, started, u1, gtab);
    fb_accumulate<HD_FB_W>(acc, started, u2, ptab);
    // infinity, or a degenerate addition on the way (Z = 0): full recovery
    if (!started || gej_is_inf(acc)) return HD_NEEDS_SLOW;
    fe zi, zi2, ax, ay;
    fe_inv_divsteps(zi, acc.z);
    fe_sqr(zi2, zi);
    fe_mul(ax, acc.x, zi2);
    fe_mul(zi2, zi2, zi);
    fe_mul(ay, acc.y, zi2);
    fe_normalize(ax);
    fe_normalize(ay);
    uint32_t diff = (ay.n[0] & 1u) ^ (v & 1u);
    HD_UNROLL for (int i = 0; i < 9; i++) diff |= ax.n[i] ^ x.n[i];
    return diff ? HD_NEEDS_SLOW : V_VALID;
}

// ---- two messages per lane ------------------------------------------------
// The two inversions (s^-1 mod n, Z^-1 mod p) are a third of the check.  A
// lane that checks two messages inverts the products s_a s_b and Z_a Z_b once
// and recovers each inverse with one multiply (Montgomery's trick): half an
// inversion per message.  A message that cannot take part (early verdict,
// unknown key, degenerate sum) contributes a factor 1 and keeps its outcome.
struct FastIn {
    uint32_t digest_be[8];
    uint32_t r_be[8];
    uint32_t s_be[8];
    uint32_t v;
    bool ready;                 // key tables available for this message
};

// Parking space for the first message's sum and x while the second one is
// computed (the kernel passes a per-lane slot in LDS: keeping both sums in
// registers spills to scratch).
struct FastPark {
    gej acc;
    fe x;
};

// stage 1 of one message: the early checks and the scalars
HD bool fast_prefix(uint8_t& out, sc& r, sc& s, sc& m, fe& x, const FastIn& in) {
    HD_UNROLL for (int i = 0; i < 8; i++) r.v[i] = s.v[i] = m.v[i] = 0u;
    fe_clear(x);
    out = HD_NEEDS_SLOW;
    if (!in.ready) return false;
    const uint8_t pre = sig_prefix(r, s, x, in.r_be, in.s_be, in.v);
    if (pre != V_VALID) {
        out = pre;
        return false;
    }
    sc_from_be_reduce(m, in.digest_be);
    return true;
}

// stage 2 of one message: u1 G + u2 P with u1 = m / s, u2 = r / s
template <typename GT, typename PT>
HD bool fast_sum(gej& acc, bool live, const sc& m, const sc& r, const sc& sinv, GT gtab, PT ptab) {
    sc u1, u2;
    sc_mul(u1, m, sinv);
    sc_mul(u2, r, sinv);
    gej_set_inf(acc);
    bool started = false;
    fb_accumulate<HD_FB_WG>(acc, started, u1, gtab);
    fb_accumulate<HD_FB_W>(acc, started, u2, ptab);
    return live && started && !gej_is_inf(acc);
}

// stage 3 of one message: affine x and y parity against (x, v & 1)
HD uint8_t fast_final(const gej& acc, const fe& zinv, const fe& x, uint32_t v) {
    fe z2, ax, ay;
    fe_sqr(z2, zinv);
    fe_mul(ax, acc.x, z2);
    fe_mul(z2, z2, zinv);
    fe_mul(ay, acc.y, z2);
    fe_normalize(ax);
    fe_normalize(ay);
    uint32_t diff = (ay.n[0] & 1u) ^ (v & 1u);
    HD_UNROLL for (int i = 0; i < 9; i++) diff |= ax.n[i] ^ x.n[i];
    return diff ? HD_NEEDS_SLOW : V_VALID;
}

// fast_final for a sum stored by gxz_finish: w = (ZZ ZZZ)^-1, so x = (X ZZZ) w
// and y = (Y ZZ) w
HD uint8_t fast_final_xz(const fe& xn, const fe& yn, const fe& w, const fe& x, uint32_t v) {
    fe ax, ay;
    fe_mul(ax, xn, w);
    fe_mul(ay, yn, w);
    fe_normalize(ax);
    fe_normalize(ay);
    uint32_t diff = (ay.n[0] & 1u) ^ (v & 1u);
    HD_UNROLL for (int i = 0; i < 9; i++) diff |= ax.n[i] ^ x.n[i];
    return diff ? HD_NEEDS_SLOW : V_VALID;
}

// The stages are written out per message (no arrays indexed by the message:
// the compiler keeps such a loop rolled and the arrays in scratch).
template <typename GT, typename PT>
HD void verify_fast2(uint8_t out[2], const FastIn in[2], GT gtab, PT ptab0, PT ptab1, FastPark* park) {
    sc r0, s0, m0, r1, s1, m1;
    fe x0, x1;
    uint8_t o0, o1;
    const bool live0 = fast_prefix(o0, r0, s0, m0, x0, in[0]);
    const bool live1 = fast_prefix(o1, r1, s1, m1, x1, in[1]);
    // s^-1 for both from one inversion
    sc one;
    HD_UNROLL for (int i = 0; i < 8; i++) one.v[i] = i == 0 ? 1u : 0u;
    sc sa = live0 ? s0 : one, sb = live1 ? s1 : one, prod, inv, ia, ib;
    sc_mul(prod, sa, sb);
    sc_inv_divsteps(inv, prod);
    sc_mul(ia, inv, sb);
    sc_mul(ib, inv, sa);
    gej acc;
    const bool ok0 = fast_sum(acc, live0, m0, r0, ia, gtab, ptab0);
    park->acc = acc;
    park->x = x0;
    gej acc1;
    const bool ok1 = fast_sum(acc1, live1, m1, r1, ib, gtab, ptab1);
    acc = park->acc;
    x0 = park->x;
    // Z^-1 for both from one inversion
    fe fone;
    fe_set_u32(fone, 1);
    fe za = acc.z, zb = acc1.z, zp, zi, zia, zib;
    fe_cmov(za, fone, !ok0);
    fe_cmov(zb, fone, !ok1);
    fe_mul(zp, za, zb);
    fe_inv_divsteps(zi, zp);
    fe_mul(zia, zi, zb);
    fe_mul(zib, zi, za);
    out[0] = ok0 ? fast_final(acc, zia, x0, in[0].v) : o0;
    out[1] = ok1 ? fast_final(acc1, zib, x1, in[1].v) : o1;
}

// ---- the INFINITY verdict from the fixed-base G table ------------------------
// The recovery returns the point at infinity (V_INFINITY, nothing recovered)
// iff u2 R = -u1' G for its u1' = -m / r, u2 = s / r, i.e. iff s R = m G, i.e.
// iff R == u1 G with u1 = m / s (n is prime, s != 0).  For a leftover of the
// known-key check (m and s at hand) that is one scalar inversion and the
// fixed-base G sum -- no doublings -- instead of the full recovery.  R is the
// lifted point (y of the parity v & 1).  Returns true only when the sum is
// exactly R; a degenerate partial sum (ZZ = 0) answers false, and the full
// recovery then decides as before.
template <int W, typename Tab>
HD bool fb_is_infinity(const sc& m, const sc& s, const ge& R, Tab gtab) {
    sc sinv, u1;
    sc_inv_divsteps(sinv, s);
    sc_mul(u1, m, sinv);
    gxz acc;
    bool started = false;
    HD_NOUNROLL for (int j = 0; j < FbL<W>::NWIN; j++) {
        const int d = fb_digit<W>(u1, j);
        if (d == 0) continue;
        ge t = gtab[(size_t)j * FbL<W>::N + (uint32_t)((d < 0 ? -d : d) - 1)];
        if (d < 0) fe_neg(t.y, t.y);
        if (!started) {
            fe_norm_weak(t.y);
            gxz_set_ge(acc, t);
            started = true;
        } else {
            gxz_add_ge_nx(acc, acc, t);
        }
    }
    if (!started || gxz_is_inf(acc)) return false;   // u1 G = infinity, or a degenerate sum
    fe t;
    fe_mul(t, R.x, acc.zz);                          // x: X == x_R ZZ
    if (!fe_eq(acc.x, t)) return false;
    fe_mul(t, R.y, acc.zzz);                         // y: Y == y_R ZZZ
    return fe_eq(acc.y, t);
}

// ---- the full recovery's multiplication over the fixed-base G table --------
// Q = u1 G + u2 R as ecmult_glv computes it, with u1 G taken out of the
// ladder: the ladder keeps u2 R (GLV halves, 4-bit windows, 128 doublings on
// the isomorphic curve of the R table) and u1 G runs as fixed-base additions
// from the W-bit G table of the known-key check (FbL<W>: one table point per
// window, no doublings) in an accumulator of its own.  Its additions are
// interleaved with the ladder (one per third ladder window, the rest after it)
// but never on the ladder's dependency chain, and there are NWIN of them
// instead of the 2 x 11 G additions of the GLV ladder.  Every addition is the
// exact gej_add_ge / gej_add (infinity and P = +-Q handled), so the result is
// the same point; the caller's checks on it are unchanged.
template <int W, typename FbTab>
HD void ecmult_glv_fbg(gej& out, const ge& R, const sc& u1, const sc& u2, FbTab fbg) {
    ge rt[HD_RTAB_N], lt[HD_RTAB_N];
    fe zg;
    build_rtab_iso(rt, lt, zg, R);
    int16_t dra[HD_GLV_NWIN_R], drb[HD_GLV_NWIN_R];
    {
        sc k1, k2;
        uint32_t a[5];
        sc_split_lambda(k1, k2, u2);
        bool neg = sc_signed_abs(a, k1);
        HD_UNROLL for (int j = 0; j < HD_GLV_NWIN_R; j++) dra[j] = (int16_t)booth_digit160<HD_WR>(a, j, neg);
        neg = sc_signed_abs(a, k2);
        HD_UNROLL for (int j = 0; j < HD_GLV_NWIN_R; j++) drb[j] = (int16_t)booth_digit160<HD_WR>(a, j, neg);
    }
    gej acc, accg;
    gej_set_inf(acc);
    gej_set_inf(accg);
    int gw = 0;   // next G window
    auto g_step = [&]() {
        const int d = fb_digit<W>(u1, gw);
        if (d != 0) {
            const int ad = d < 0 ? -d : d;
            ge t = fbg[(size_t)gw * FbL<W>::N + (uint32_t)(ad - 1)];
            if (d < 0) fe_neg(t.y, t.y);
            gej_add_ge(accg, accg, t);
        }
        gw++;
    };
    HD_NOUNROLL for (int j = HD_GLV_NWIN_R - 1; j >= 0; j--) {
        if (j != HD_GLV_NWIN_R - 1) {
            HD_NOUNROLL for (int k = 0; k < HD_WR; k++) gej_dbl(acc, acc);
        }
        if (j % 3 == 0 && gw < FbL<W>::NWIN) g_step();
        HD_NOUNROLL for (int half = 0; half < 2; half++) {
            const int d = half ? drb[j] : dra[j];
            const int ad = d < 0 ? -d : d;
            ge t = half ? lt[ad == 0 ? 0 : ad - 1] : rt[ad == 0 ? 0 : ad - 1];
            if (d < 0) fe_neg(t.y, t.y);
            gej s;
            gej_add_ge(s, acc, t);
            gej_cmov(acc, s, d != 0);
        }
    }
    HD_NOUNROLL while (gw < FbL<W>::NWIN) g_step();
    fe_mul(acc.z, acc.z, zg);  // back from E' to E
    if (gej_is_inf(accg)) {
        out = acc;
    } else {
        gej q;
        gej_add(q, acc, accg);
        out = q;
    }
}
template <int W, typename FbTab>
struct GlvFbgMult {
    FbTab fbg;
    HD_MEMBER void operator()(gej& out, const ge& R, const sc& u1, const sc& u2) const {
        ecmult_glv_fbg<W>(out, R, u1, u2, fbg);
    }
};

// ---- table construction (one entry per lane) --------------------------
// 2^(W j) B, affine canonical
HD void fb_window_base(ge& out, const ge& B, int W, int j) {
    gej a;
    gej_set_ge(a, B);
    HD_NOUNROLL for (int k = 0; k < W * j; k++) gej_dbl(a, a);
    gej_to_ge(out.x, out.y, a);
}

// d B (Jacobian) for 1 <= d < 2^32: double-and-add from the top bit
HD void fb_mul_small(gej& a, const ge& B, uint32_t d) {
    int top = 31;
    while (top > 0 && !((d >> top) & 1u)) top--;
    gej_set_ge(a, B);
    HD_NOUNROLL for (int b = top - 1; b >= 0; b--) {
        gej_dbl(a, a);
        if ((d >> b) & 1u) gej_add_ge(a, a, B);
    }
}

// d Bj for 1 <= d <= 2^(W-1) (2^TOPBITS in the top window), affine canonical:
// the entry definition (the device builds tables by runs, k_fb_runs; the
// host tests check entries against this)
HD void fb_entry(ge& out, const ge& Bj, uint32_t d) {
    gej a;
    fb_mul_small(a, Bj, d);
    gej_to_ge(out.x, out.y, a);
}

}  // namespace hd
