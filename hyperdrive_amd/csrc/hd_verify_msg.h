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

// The admitted table is searched by every message of a batch.  Kernels stage
// it in LDS (dynamic shared memory, one copy per block) when it holds at most
// HD_ADM_LDS_MAX entries, so the binary search's dependent loads are LDS reads
// instead of L2 round trips.
#define HD_ADM_LDS_MAX 1024u
#if defined(__HIPCC__)
__device__ __forceinline__ void adm_stage(uint32_t* sh, const uint32_t* __restrict__ adm, uint32_t n) {
    for (uint32_t k = threadIdx.x; k < 8 * n; k += blockDim.x) sh[k] = adm[k];
    __syncthreads();
}
#endif
HD_HOSTONLY size_t adm_lds_bytes(uint32_t n) { return n <= HD_ADM_LDS_MAX ? 32 * (size_t)n : 0; }

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
