// hd_verify_msg.h -- the per-message hot path, one message per lane:
//   digest (surge preimage + SHA-256)  -> recover (libsecp256k1 semantics)
//   -> signatory = SHA-256(pubkey)     -> Equal(From)  -> From in admitted set
//
// Reference: process/message.go:53-78, 165-186, 263-284 (preimages);
// process/message_test.go:147-154 (sign -> Signatory(&hash) -> Equal);
// mq/mq.go:49-51 + replica/replica.go:69-72 (procsAllowed membership).
#pragma once
#include "hd_fixedbase.h"
#include "hd_group.h"
#include "hd_sha256.h"

namespace hd {

struct MsgIn {
    uint32_t type;
    int64_t h, r, vr;
    uint32_t value_be[8];
    uint32_t from_be[8];
    uint32_t r_be[8], s_be[8];
    uint32_t v;
};

HD void message_digest(uint32_t d[8], const MsgIn& m) {
    if (m.type == T_PROPOSE) sha256_propose(d, m.h, m.r, m.vr, m.value_be);
    else sha256_vote(d, m.h, m.r, m.value_be);
}

// lexicographic compare of two 32-byte strings held as 8 big-endian words
HD int cmp_be256(const uint32_t a[8], const uint32_t b[8]) {
    int res = 0;
    HD_UNROLL for (int i = 7; i >= 0; i--) {
        int c = a[i] < b[i] ? -1 : (a[i] > b[i] ? 1 : 0);
        res = c != 0 ? c : res;
    }
    return res;
}

// Admitted table: n entries of 8 big-endian words, sorted ascending.  Returns
// the index or -1.  Uniform iteration count (ceil log2) for all lanes.
template <typename AdmTab>
HD int32_t admitted_find(AdmTab adm, uint32_t n, int steps, const uint32_t key[8]) {
    uint32_t lo = 0, len = n;
    HD_NOUNROLL for (int s = 0; s < steps; s++) {
        uint32_t half = len >> 1;
        uint32_t mid = lo + half;
        uint32_t e[8];
        bool ok = mid < n && len > 1;
        uint32_t idx = ok ? mid : 0u;
        HD_UNROLL for (int w = 0; w < 8; w++) e[w] = adm[idx * 8 + w];
        if (ok && cmp_be256(e, key) <= 0) lo = mid;
        len = len - half;
    }
    if (n == 0) return -1;
    uint32_t e[8];
    HD_UNROLL for (int w = 0; w < 8; w++) e[w] = adm[lo * 8 + w];
    return cmp_be256(e, key) == 0 ? (int32_t)lo : -1;
}

// Hashed index of the admitted table (hd_set_signatories builds it), searched
// by every message of the batch-wide kernels (k_fast_prep, the tally and
// route passes): an open-addressing array of sorted indices at load factor
// <= 1/4, keyed by the first four words of the From.  A lookup is one or two
// dependent loads of the slot array (L2-resident, 4 B per slot) and one
// 32-byte compare, where the binary search takes log2(n) dependent 32-byte
// steps and wanted the table staged in LDS by every block.  Same answer as
// admitted_find: the sorted index of the entry equal to key, or -1.
struct AdmIndex {
    const uint32_t* adm;    // the sorted table (8 BE words per entry)
    const uint32_t* slot;   // sorted index per slot, 0xFFFFFFFF empty
    uint32_t mask;          // slots - 1
};
HD uint32_t adm_hash(const uint32_t key[8]) {
    uint64_t x = ((uint64_t)key[0] << 32 | key[1]) ^ (((uint64_t)key[2] << 32 | key[3]) * 0x9E3779B97F4A7C15ull);
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    return (uint32_t)x;
}
template <typename AdmTab>
HD int32_t adm_index_find(const AdmTab adm, const uint32_t* slot, uint32_t mask, const uint32_t key[8]) {
    uint32_t s = adm_hash(key) & mask;
    while (true) {
        const uint32_t idx = slot[s];
        if (idx == 0xFFFFFFFFu) return -1;
        bool eq = true;
        HD_UNROLL for (int w = 0; w < 8; w++) eq &= adm[idx * 8 + w] == key[w];
        if (eq) return (int32_t)idx;
        s = (s + 1) & mask;
    }
}
HD int32_t adm_index_find(const AdmIndex& ix, const uint32_t key[8]) {
    return adm_index_find(ix.adm, ix.slot, ix.mask, key);
}
// host: the slot array for n sorted entries (words: 8 BE words each); slots =
// the smallest power of two >= max(16, 4n)
HD_HOSTONLY uint32_t adm_index_slots(uint32_t n) {
    uint32_t c = 16;
    while (c < 4 * n) c <<= 1;
    return c;
}
HD_HOSTONLY void adm_index_build(const uint32_t* words, uint32_t n, uint32_t* slot, uint32_t slots) {
    for (uint32_t s = 0; s < slots; s++) slot[s] = 0xFFFFFFFFu;
    for (uint32_t k = 0; k < n; k++) {
        uint32_t s = adm_hash(words + 8 * (size_t)k) & (slots - 1);
        while (slot[s] != 0xFFFFFFFFu) s = (s + 1) & (slots - 1);
        slot[s] = k;
    }
}

// Full verdict for one message.  Src supplies the message fields on demand
// (type(), h(), r(), vr(), value(w), from(w), sig_r(w), sig_s(w), sig_v(),
// and has_digest() / digest(w) when the digest is given rather than computed),
// so the kernel loads each field from HBM in the phase that uses it and
// nothing but the accumulator stays live across the ladder.  rec_be receives
// the recovered signatory (zeros when recovery failed); signer the
// admitted-table index; qout (optional) the recovered key of a VALID message.
// fbg (optional, device): the known-key check's fixed-base G table; the
// recovery then takes u1 G from it (ecmult_glv_fbg) instead of the GLV ladder.
template <typename Src, typename GTab, typename AdmTab>
HD uint8_t verify_msg_src(const Src& src, GTab gtab, AdmTab adm, uint32_t n_adm, int adm_steps, int pkfmt,
                          uint32_t rec_be[8], int32_t& signer, ge* qout = nullptr, const gp* fbg = nullptr) {
    signer = -1;
    HD_UNROLL for (int i = 0; i < 8; i++) rec_be[i] = 0;
    const uint32_t type = src.type();
    if (type < 1 || type > 3) return V_BAD_TYPE;
    uint32_t d[8];
    if (src.has_digest()) {
        // caller-supplied digest (include/hd_digest.h), e.g. a Keccak-256 lane
        HD_UNROLL for (int w = 0; w < 8; w++) d[w] = src.digest(w);
    } else {
        uint32_t value_be[8];
        HD_UNROLL for (int w = 0; w < 8; w++) value_be[w] = src.value(w);
        if (type == T_PROPOSE) sha256_propose(d, src.h(), src.r(), src.vr(), value_be);
        else sha256_vote(d, src.h(), src.r(), value_be);
    }
    fe qx, qy;
    uint8_t verdict;
    {
        uint32_t r_be[8], s_be[8];
        HD_UNROLL for (int w = 0; w < 8; w++) { r_be[w] = src.sig_r(w); s_be[w] = src.sig_s(w); }
        if (fbg) verdict = recover_m(qx, qy, d, r_be, s_be, src.sig_v(), GlvFbgMult<HD_FB_WG, GpTab>{GpTab{fbg}});
        else verdict = recover(qx, qy, d, r_be, s_be, src.sig_v(), gtab);
    }
    if (verdict != V_VALID) return verdict;
    {
        uint32_t xb[8], yb[8];
        fe_to_be(xb, qx);
        fe_to_be(yb, qy);
        sha256_pubkey(rec_be, pkfmt, xb, yb, qy.n[0] & 1u);
    }
    uint32_t from_be[8];
    uint32_t diff = 0;
    HD_UNROLL for (int i = 0; i < 8; i++) {
        from_be[i] = src.from(i);
        diff |= rec_be[i] ^ from_be[i];
    }
    if (diff) return V_SIGNATORY_MISMATCH;
    if (qout) {  // the recovered key (== From's), for the known-key tables (hd_fixedbase.h)
        qout->x = qx;
        qout->y = qy;
    }
    int32_t idx = admitted_find(adm, n_adm, adm_steps, from_be);
    if (idx < 0) return V_NOT_ADMITTED;
    signer = idx;
    return V_VALID;
}

// MsgIn-backed source (host harness, generator)
struct MsgSrc {
    const MsgIn& m;
    HD_MEMBER uint32_t type() const { return m.type; }
    HD_MEMBER int64_t h() const { return m.h; }
    HD_MEMBER int64_t r() const { return m.r; }
    HD_MEMBER int64_t vr() const { return m.vr; }
    HD_MEMBER uint32_t value(int w) const { return m.value_be[w]; }
    HD_MEMBER uint32_t from(int w) const { return m.from_be[w]; }
    HD_MEMBER uint32_t sig_r(int w) const { return m.r_be[w]; }
    HD_MEMBER uint32_t sig_s(int w) const { return m.s_be[w]; }
    HD_MEMBER uint32_t sig_v() const { return m.v; }
    HD_MEMBER bool has_digest() const { return false; }
    HD_MEMBER uint32_t digest(int) const { return 0; }
};

template <typename GTab, typename AdmTab>
HD uint8_t verify_msg(const MsgIn& m, GTab gtab, AdmTab adm, uint32_t n_adm, int adm_steps, int pkfmt,
                      uint32_t rec_be[8], int32_t& signer) {
    MsgSrc src{m};
    return verify_msg_src(src, gtab, adm, n_adm, adm_steps, pkfmt, rec_be, signer);
}

}  // namespace hd
