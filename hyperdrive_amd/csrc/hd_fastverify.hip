// hd_fastverify.hip -- the known-key fast path of hd_verify_batch_device and
// the tables it runs on (hd_fixedbase.h).
//
// Per batch, stream-ordered, no host synchronisation:
//   k_fast_prep / k_fast_sinv / k_fast_sums / k_fast_zinv / k_fast_cmp
//                   the split known-key check (the default, see "the split
//                   check" below): a message whose claimed From is an
//                   admitted signatory with a known key is checked with two
//                   fixed-base multiplications (23 mixed additions, no
//                   doublings, no square root); VALID / early exact verdicts
//                   are final, everything else is appended to a list
//   k_verify        (hd_verify.hip) the full libsecp256k1-semantics recovery
//                   over that list only; VALID messages of signatories without
//                   a known key publish the recovered key to their slot
//   k_fb_list / k_fb_bases / k_fb_runs / k_fb_ready
//                   build the tables of newly learned keys (window bases,
//                   then the affine multiples by segments of consecutive
//                   entries, one addition per entry); with nothing learned
//                   each exits at once
// Table memory is capped by HD_FB_MAX_BYTES (default 64 GiB of the 288 GB):
// signatories beyond the cap always take the full recovery.
// G has one table with wider windows (HD_FB_WG bits), built once per device
// and process (fb_g_table).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/hd_verify.h"
#include "hd_fixedbase.h"
#include "hd_scmont.h"
#include "hd_internal.h"
#include "hd_verify_msg.h"

using namespace hd;

struct FbWork {
    const gp* gtab = nullptr;   // the shared G table of the device (fb_g_table)
    uint32_t nslots = 0;        // slots with a table (whole chunks); slot 0 is unused
    uint32_t max_slots = 0;     // from HD_FB_MAX_BYTES (slot 0 included)
    // Per-key tables live in chunks of HD_FB_CHUNK slots that are allocated
    // when the admitted set first needs them and never moved: a set change
    // that adds keys allocates only new chunks (no regrow, no copy of the
    // tables already built).  tabs[slot] points at the slot's table.
    gp** tabs = nullptr;        // device: max_slots table pointers
    std::vector<gp*> chunks;    // host: the chunk allocations
    ge* base = nullptr;         // max_slots x HD_FB_NWIN window bases
    ge* pub = nullptr;          // max_slots keys
    uint32_t* state = nullptr;  // max_slots HD_FB_* states
    int32_t* adm_slot = nullptr;  // admitted sorted index -> slot
    bool map_ok = true;           // the last hd_fb_map_signatories succeeded (else: full recovery only)
    size_t cap_adm_slot = 0;
    uint32_t* list = nullptr;     // slot work list (max_slots)
    uint32_t* counts = nullptr;   // [0] slots to build (the table builder's)
    uint32_t* zr = nullptr;       // the table builder's z ratios (k_fb_runs: HD_FB_RUN x 9 words per thread)
    // Per-call scratch, HD_FB_NSCRATCH sets used round robin, so that verify
    // calls issued on different streams can run concurrently on the device:
    // the next call's one-message-per-lane kernels fill the SIMDs that this
    // call's inversion kernels (n / K lanes), the last partial round of its
    // k_fast_sums and its fallback recovery leave idle.
    struct Scratch {
        uint32_t* rows = nullptr;     // the split check's per-message rows (SplitRows, 62 words per message)
        size_t cap_rows = 0;
        uint32_t* slow = nullptr;     // message index list: the known-key check's leftovers
        size_t cap_slow = 0;
        uint32_t* count = nullptr;    // its length (device words: [0] leftovers, [1] after k_slow_lift)
        uint32_t* slow2 = nullptr;    // the leftovers that pass the lift: the full recovery's list
        size_t cap_slow2 = 0;
        hipEvent_t done = nullptr;    // recorded after the last call that used this set
        hipStream_t stream = nullptr; // that call's stream
        bool used = false;
    };
    static constexpr int NSCRATCH = 3;
    Scratch sc[NSCRATCH];
    int next = 0;                 // the set the next call takes
    int last_set = -1;            // the set of the last call (hd_ctx_fastpath_stats)
    // Mapped slots whose key is not READY, in pinned host memory the device
    // also writes (k_fb_ready subtracts what it finished): 0 means nothing
    // can be learned any more, so a verify call launches no table-build
    // kernels.  Set exactly (after a device sync) whenever the admitted set
    // or the key format changes; UINT32_MAX = unknown.
    uint32_t* nr_host = nullptr;
    uint32_t* nr_dev = nullptr;
    // The fallback list lengths of the latest calls ([0] leftovers of the
    // check, [1] those past the lift), stored by k_slow_lift / k_verify into
    // pinned host memory: they size the next calls' fallback grids (both
    // kernels walk their list grid-stride, so any size is correct; a grid
    // sized by the last list instead of the batch keeps ~2,000 blocks that
    // would only start and exit from queueing for SIMD slots behind a
    // concurrent call's k_fast_sums).  UINT32_MAX = none seen yet.
    uint32_t* est_host = nullptr;
    uint32_t* est_dev = nullptr;
    // Ordering between calls (hd_fb_verify): a call waits (on the device) for
    // the last call that used its scratch set.  While keys can still be
    // learned (nr_host != 0), or on the first call after the last key became
    // READY, a call also waits for the previous call, whatever its stream:
    // learning writes the shared tables, states and builder scratch.  In the
    // steady state (every mapped key READY, nothing written but per-call
    // scratch and the caller's outputs) calls on different streams overlap.
    hipEvent_t done = nullptr;    // recorded after every call
    hipStream_t last = nullptr;
    bool any = false;
    bool steady = false;          // the previous call ran with nothing to learn
    // hd_ctx_profile: event pairs around whole calls and around k_fast_sums
    bool prof = false;
    std::vector<hipEvent_t> ev_call, ev_sums;
    size_t n_call = 0, n_sums = 0;   // pairs in use
    std::unordered_map<std::string, uint32_t> slot_of;  // signatory -> slot
    std::vector<uint32_t> free_slots;
    uint32_t used = 1;            // slots handed out so far (slot 0 = G)
    int wp = HD_FB_W;             // window width of the per-key tables (HD_FB_W or HD_FB_WW)
    int last_k = 8;               // messages per inversion of the last split check (split_k_for)
    double budget = 0;            // table bytes allowed (HD_FB_MAX_BYTES), shared per device
    size_t bytes = 0;             // table bytes this context holds
    // Foreign keys (HD_VAR_FOREIGN_KEYS): fres slots fbase .. reserved once
    // (a contiguous block, kept across set changes) for authenticated Froms
    // outside the admitted set, of which the first fcap are in use (fcap is
    // re-read from the variant at every set change: 0 turns learning off,
    // the block stays reserved); fdict maps such a From to its slot (emptied
    // on every set change).  k_verify stores the claim count into fpend_host;
    // a change since fseen makes the next call build the new tables.
    uint32_t* fdict = nullptr;
    uint32_t* fnext = nullptr;
    uint32_t fbase = 0, fcap = 0, fres = 0;
    uint32_t* fpend_host = nullptr;   // [0] claim count, [1] the fmiss flag (SlowCtl)
    uint32_t* fpend_dev = nullptr;
    uint32_t fseen = 0;
    // Slot eviction (fb_evict): fhit[0, 64) counts each foreign slot's
    // known-key checks, fhit[64, 64 + HD_FD_BUCKETS) the recoveries of each
    // slotless dictionary entry (fbhit), fkey the slotless entries' keys.
    // fwait / fcalls: calls between checks while misses are flagged
    // (doubling, up to HD_FD_EVICT_WAIT_MAX, while checks swap nothing).
    uint32_t* fhit = nullptr;
    ge* fkey = nullptr;
    uint32_t fwait = 1, fcalls = 0;
    bool fforce = false;   // build the LEARNED slots at this call's end (an eviction re-keyed one)
    uint32_t evictions = 0;
    uint32_t evict_checks = 0;   // fb_evict passes that waited for the context's calls
    uint32_t evict_aborts = 0;   // passes whose new dictionary had no bucket for a slot holder
};

namespace {

#define FBCHK(expr, what)                                \
    do {                                                 \
        hipError_t e_ = (expr);                          \
        if (e_ != hipSuccess) return hd_ctx_fail(ctx, e_, what); \
    } while (0)

// message i of a device batch, fields on demand (as DevSrc in hd_verify.hip)
struct FastSrc {
    const DevBatch& b;
    uint32_t i;
    const uint8_t* dg;
    __device__ __forceinline__ uint32_t type() const { return b.type[i]; }
    __device__ __forceinline__ uint32_t value(int w) const { return load_be32(b.value32 + 32 * (size_t)i + 4 * w); }
    __device__ __forceinline__ uint32_t from(int w) const { return load_be32(b.from32 + 32 * (size_t)i + 4 * w); }
    __device__ __forceinline__ uint32_t sig_r(int w) const { return load_be32(b.sig65 + 65 * (size_t)i + 4 * w); }
    __device__ __forceinline__ uint32_t sig_s(int w) const { return load_be32(b.sig65 + 65 * (size_t)i + 32 + 4 * w); }
    __device__ __forceinline__ uint32_t sig_v() const { return b.sig65[65 * (size_t)i + 64]; }
    // whole fields with wide loads (hd_common.h)
    __device__ __forceinline__ void sig(uint32_t r_be[8], uint32_t s_be[8], uint32_t& v) const {
        load_sig65(r_be, s_be, v, b.sig65, i, b.n);
    }
    __device__ __forceinline__ void from_words(uint32_t w[8]) const { load_row32_be(w, b.from32, i); }
    __device__ __forceinline__ void value_words(uint32_t w[8]) const { load_row32_be(w, b.value32, i); }
};

// ---- the split check: K messages per lane share each inversion ----------
// The known-key check in five kernels: the two inversions (of s mod n, of Z
// mod p) serve K messages of a lane each (Montgomery's trick over K), and
// everything else runs one message per lane, so that only the inversion
// kernels have the low occupancy of n / K lanes.  Per-message state sits in word-major HBM rows
// between them (lane t reads word w of message i at w * n + i, coalesced):
//   k_fast_prep     one per lane: lookup, digest, early checks; m, r, s
//   k_fast_sinv     K per lane: prefix products of s, one inversion mod n,
//                   s^-1 of each message
//   k_fast_sums     one per lane: u1 = m / s, u2 = r / s as window digits
//                   (into LDS), then u1 G + u2 P (the first window's point
//                   loaded, one XYZZ mixed addition per further window)
//   k_fast_zinv     K per lane: prefix products of Z, one inversion mod p,
//                   Z^-1 of each message
//   k_fast_cmp      one per lane: the comparison, the outputs, the valid
//                   bitmap and the fallback list
// Message i of lane t of an inversion kernel is i = j T + t (j < K,
// T = ceil(n / K)), so every step j of a wave touches consecutive messages.
// The verdicts are the ones verify_fast2 (hd_fixedbase.h, host-tested) gives:
// same early checks, same sums, same comparison.
#define HD_FAST_LIVE 0xFDu   // aux code: keep going (the rest are final verdicts or HD_NEEDS_SLOW)

template <int NW>
HD void soa_load(uint32_t (&w)[NW], const uint32_t* __restrict__ p, uint32_t n, uint32_t i) {
    HD_UNROLL for (int k = 0; k < NW; k++) w[k] = p[(size_t)k * n + i];
}
template <int NW>
HD void soa_store(uint32_t* __restrict__ p, uint32_t n, uint32_t i, const uint32_t (&w)[NW]) {
    HD_UNROLL for (int k = 0; k < NW; k++) p[(size_t)k * n + i] = w[k];
}

struct SplitRows {
    uint32_t* aux;   // n: slot << 8 | code
    int32_t* idx;    // n: admitted (sorted) index
    uint32_t* u1;    // 8n: m
    uint32_t* u2;    // 8n: r
    uint32_t* s;     // 8n: s
    uint32_t* pre;   // 9n: prefix products of s, then s^-1 R (radix 2^29); later of Z, then Z^-1
    uint32_t* xyz;   // 27n: the XYZZ sum as (X ZZZ, Y ZZ, Z = ZZ ZZZ) (gxz_finish)
    int prio;        // wave priority of the short kernels (HD_VAR_WAVE_PRIO)
};

// s_setprio takes an immediate: a uniform branch per level
HD void wave_prio(int p) {
    if (p == 1) __builtin_amdgcn_s_setprio(1);
    else if (p == 2) __builtin_amdgcn_s_setprio(2);
    else if (p >= 3) __builtin_amdgcn_s_setprio(3);
}

// a Booth digit of window w as a reference into the base's table: entry
// index | HD_REF_NEG for a negative digit, HD_REF_ZERO for 0 (entry 0 of the
// window is then read and discarded)
#define HD_REF_NEG 0x80000000u
#define HD_REF_ZERO 0x40000000u
#define HD_REF_IDX 0x3FFFFFFFu
template <int W>
HD uint32_t fb_ref(int d, int w) {
    const uint32_t ad = (uint32_t)(d < 0 ? -d : d);
    const uint32_t base = (uint32_t)w * FbL<W>::N;
    return d == 0 ? (base | HD_REF_ZERO) : ((base + ad - 1) | (d < 0 ? HD_REF_NEG : 0u));
}

// one message per lane (occupancy hides the lookup's dependent loads): type,
// admitted lookup, key state, digest, the early checks; m and r to the rows
__global__ __launch_bounds__(256) void k_fast_prep(DevBatch b, const uint8_t* __restrict__ digest_in,
                                                   const uint32_t* __restrict__ state,
                                                   const int32_t* __restrict__ adm_slot, AdmIndex ix,
                                                   uint32_t n_adm, SplitRows rows, const uint32_t* __restrict__ fdict,
                                                   uint32_t* __restrict__ fhit, uint32_t fbase) {
    wave_prio(rows.prio);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = b.n;
    if (i >= n) return;
    FastSrc src{b, i, digest_in};
    const uint32_t type = src.type();
    uint32_t code = HD_NEEDS_SLOW, slot = 0;
    int32_t idx = -1;
    if (type < 1 || type > 3) {
        code = V_BAD_TYPE;
    } else {
        uint32_t from_be[8];
        src.from_words(from_be);
        idx = n_adm ? adm_index_find(ix, from_be) : -1;
        int32_t sl = idx >= 0 ? adm_slot[idx] : -1;
        if (idx < 0 && fdict) {
            // an authenticated From outside the admitted set with a known key:
            // the check's success means NOT_ADMITTED (idx -2 marks it)
            sl = fdict_find(fdict, from_be);
            if (sl >= 0) idx = -2;
        }
        if (sl >= 0 && state[sl] == HD_FB_READY) {
            slot = (uint32_t)sl;
            if (idx == -2) atomicAdd(&fhit[sl - (int32_t)fbase], 1u);   // a foreign slot's use (fb_evict)
            FastIn in;
            if (digest_in) {
                load_row32_be(in.digest_be, digest_in, i);
            } else {
                uint32_t value_be[8];
                src.value_words(value_be);
                if (type == T_PROPOSE)
                    sha256_propose(in.digest_be, b.height[i], b.round[i], b.valid_round ? b.valid_round[i] : -1,
                                   value_be);
                else
                    sha256_vote(in.digest_be, b.height[i], b.round[i], value_be);
            }
            src.sig(in.r_be, in.s_be, in.v);
            in.ready = true;
            sc r, s, m;
            fe x;
            uint8_t o;
            if (fast_prefix(o, r, s, m, x, in)) {
                code = HD_FAST_LIVE;
                soa_store(rows.u1, n, i, m.v);
                soa_store(rows.u2, n, i, r.v);
                soa_store(rows.s, n, i, s.v);
            } else {
                code = o;
            }
        }
    }
    rows.aux[i] = slot << 8 | code;
    rows.idx[i] = idx;
}

// K per lane: prefix products of s over the lane's live messages, one
// inversion mod n, then s^-1 of each.  The products are Montgomery products in
// radix 2^29 (hd_scmont.h, R = 2^261): with P_l = prod_{i<=l} s_i R^-l the l-th
// live prefix, inv = P_last^-1 R gives, walking back, s_l^-1 R =
// M(inv_l, P_{l-1}) and inv_{l-1} = M(inv_l, s_l).  s^-1 R leaves in the pre
// row.  The lane's K scalars and prefixes stay in registers (both walks are
// unrolled), and the loads of all K messages issue together up front: with
// n / K lanes there are too few waves to hide a load per step.
template <int K>
__global__ __launch_bounds__(256) void k_fast_sinv(uint32_t n, uint32_t T, SplitRows rows) {
    wave_prio(rows.prio);
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    sc sv[K];
    uint32_t live = 0;   // bit j: message j of this lane goes on
    static_for<K>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const uint32_t i = (uint32_t)j * T + t;
        const uint32_t ic = i < n ? i : n - 1;   // rows exist up to n - 1
        const uint32_t a = rows.aux[ic];
        soa_load(sv[j].v, rows.s, n, ic);
        live |= (i < n && (a & 0xFFu) == HD_FAST_LIVE) ? 1u << j : 0u;
    });
    if (!live) return;
    sm pre[K], acc;
    HD_UNROLL for (int k = 0; k < 9; k++) acc.n[k] = 0;
    static_for<K>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if ((live >> j) & 1u) {
            sm ss;
            sm_from_sc(ss, sv[j]);
            if (live & ((1u << j) - 1u)) sm_mul(acc, acc, ss);
            else acc = ss;
        }
        pre[j] = acc;   // the product of the live messages up to j
    });
    sm inv;
    {
        sc p, pinv;
        sm_to_sc(p, acc);
        sc_inv_divsteps(pinv, p);   // a product of scalars in [1, n) times R^-k: never 0
        sm_from_sc(inv, pinv);
        sm r2;
        sm_r2(r2);
        sm_mul(inv, inv, r2);
    }
    static_for<K>([&](auto jc) {
        constexpr int j = K - 1 - decltype(jc)::value;
        if (!((live >> j) & 1u)) return;
        const uint32_t i = (uint32_t)j * T + t;
        if (j > 0 && (live & ((1u << j) - 1u))) {   // a live message before this one
            sm sinv, ss;
            sm_mul(sinv, inv, pre[j > 0 ? j - 1 : 0]);
            sm_from_sc(ss, sv[j]);
            sm_mul(inv, inv, ss);
            soa_store(rows.pre, n, i, sinv.n);
        } else {
            soa_store(rows.pre, n, i, inv.n);
        }
    });
}

// u1 G + u2 P from the digit rows: the first G window's point starts the
// sum (no addition), then one mixed addition per further window, the next
// point loaded one addition ahead.  A zero digit contributes nothing; while
// no digit has been non-zero the sum is the point at infinity.  Zero digits
// are rare (~2^-W per window), so the selects they need run only in a
// wavefront that has one (a uniform branch); every other step is the bare
// addition.  (Sending such messages to the full recovery instead costs a
// whole recovery's latency per verify call: measured 1.95 -> 3.0 ms per 1M.)
// The sums are XYZZ (gxz, hd_fixedbase.h: 8M + 2S per addition).
// One window step (gxz_sum_step, hd_fixedbase.h): dst = src + the window's
// point; the repair branch runs in a wavefront with a zero digit or a
// not-yet-started sum.
template <bool FIRST>
HD void sum_add(gxz& dst, const gxz& src, bool& started, const ge& p0, const ge& g, uint32_t ec) {
    const bool nz = !(ec & HD_REF_ZERO);
    const bool rare = __ballot(!(started && nz)) != 0ull;
    gxz_sum_step<FIRST>(dst, src, started, p0, g, (ec & HD_REF_NEG) != 0, nz, rare);
}

// the window digits of u1 = m / s and u2 = r / s (Montgomery products with
// s^-1 R come out plain) as table references: G windows, then P windows;
// dst[w * stride] for window w
template <int WP>
HD void fast_digit_refs(uint32_t* dst, size_t stride, const SplitRows& rows, uint32_t n, uint32_t i) {
    sm sinv, x;
    soa_load(sinv.n, rows.pre, n, i);
    sc u;
    soa_load(u.v, rows.u1, n, i);
    sm_from_sc(x, u);
    sm_mul(x, x, sinv);
    sm_to_sc(u, x);
    HD_UNROLL for (int w = 0; w < FbL<HD_FB_WG>::NWIN; w++)
        dst[(size_t)w * stride] = fb_ref<HD_FB_WG>(fb_digit<HD_FB_WG>(u, w), w);
    soa_load(u.v, rows.u2, n, i);
    sm_from_sc(x, u);
    sm_mul(x, x, sinv);
    sm_to_sc(u, x);
    HD_UNROLL for (int w = 0; w < FbL<WP>::NWIN; w++)
        dst[(size_t)(FbL<HD_FB_WG>::NWIN + w) * stride] = fb_ref<WP>(fb_digit<WP>(u, w), w);
}

// a table point read through a global (address space 1) pointer (k_fast_sums)
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(1))) const gp gp_global;
#else
typedef const gp gp_global;
#endif

// The digits are computed here, into this lane's column of an LDS array (no
// digit pass, no digit rows in HBM).
template <int WAVES, int WP, int PF>
__global__ __launch_bounds__(256, WAVES) void k_fast_sums(uint32_t n, const gp* __restrict__ gtab,
                                                          const gp* const* __restrict__ tabs, SplitRows rows) {
    constexpr int NG = FbL<HD_FB_WG>::NWIN, NT = NG + FbL<WP>::NWIN;
    static_assert(PF >= 0 && PF <= 2, "prefetch depth");
    __shared__ uint32_t sdig[NT * 256];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t a = rows.aux[i];
    if ((a & 0xFFu) != HD_FAST_LIVE) return;
    // The table pointers as global (address space 1) pointers: the loads
    // are then global_load (counted in vmcnt only).  A flat load -- what a
    // pointer read from memory (tabs[]) compiles to -- also counts in
    // lgkmcnt, so the wait for the next digit's LDS read would wait for the
    // point prefetched one addition ahead as well, exposing its latency.
    const gp_global* gt = (const gp_global*)gtab;
    const gp_global* pt = (const gp_global*)tabs[a >> 8];
    // a lane reads back only its own column: no barrier
    const size_t dstride = 256;
    const uint32_t* dp = sdig + threadIdx.x;
    fast_digit_refs<WP>(sdig + threadIdx.x, 256, rows, n, i);
    uint32_t e = dp[0];
    gxz acc;
    ge p0;
    gp_unpack(p0, gt[e & HD_REF_IDX]);
    if (e & HD_REF_NEG) fe_neg(p0.y, p0.y);
    fe_norm_weak(p0.y);
    gxz_set_ge(acc, p0);
    bool started = !(e & HD_REF_ZERO);   // (while not started, acc is never read)
    // The next PF windows' points, packed (16 words each) until used; the
    // digit of the window after those is read one addition earlier still, so
    // no load waits on another load inside an addition.  Window indices past
    // the last are clamped to it (a wasted but valid load), so every load is
    // unconditional and lands straight in the registers that carry it.
    auto tab = [&](int w) { return w < NG ? gt : pt; };
    auto dig = [&](int w) { return dp[(size_t)(w < NT - 1 ? w : NT - 1) * dstride]; };
    uint32_t c1 = dig(1), c2 = 0, dn = 0;
    gp q1, q2;
    if (PF > 0) q1 = gt[c1 & HD_REF_IDX];
    if (PF == 2) {
        c2 = dig(2);
        q2 = tab(2)[c2 & HD_REF_IDX];
    }
    if (PF > 0) dn = dig(PF + 1);
    // window j's point and digit reference, advancing the prefetch queue
    // (PF = 0: loaded when used; the other waves of the SIMD cover the wait)
    auto advance = [&](int j, gp& cur, uint32_t& ec) {
        if (PF == 0) {
            ec = j == 1 ? c1 : dig(j);
            cur = tab(j)[ec & HD_REF_IDX];
            return;
        }
        cur = q1;
        ec = c1;
        if (PF == 2) {
            q1 = q2;
            c1 = c2;
            c2 = dn;
            q2 = tab(j + 2 < NT ? j + 2 : NT - 1)[c2 & HD_REF_IDX];
        } else {
            c1 = dn;
            q1 = tab(j + 1 < NT ? j + 1 : NT - 1)[c1 & HD_REF_IDX];
        }
        dn = dig(j + PF + 1);
    };
    // two accumulators in turn (gxz_sum_step): window 1 into b, then a, b, ...
    gxz b;
    auto step = [&](int j, gxz& dst, const gxz& src) {
        gp cur;
        uint32_t ec;
        advance(j, cur, ec);
        ge g;
        gp_unpack(g, cur);
        if (j == 1) sum_add<true>(dst, src, started, p0, g, ec);
        else sum_add<false>(dst, src, started, p0, g, ec);
    };
    step(1, b, acc);
    HD_NOUNROLL for (int j = 2; j + 1 < NT; j += 2) {
        step(j, acc, b);
        step(j + 1, b, acc);
    }
    if constexpr ((NT - 2) % 2 == 1) step(NT - 1, acc, b);   // an odd number of windows after the first two
    else acc = b;
    // infinity, or a degenerate addition on the way (ZZ = 0): full recovery
    if (!started || gxz_is_inf(acc)) {
        rows.aux[i] = (a & ~0xFFu) | HD_NEEDS_SLOW;
        return;
    }
    // (X ZZZ, Y ZZ, ZZ ZZZ): k_fast_zinv inverts the third like a Jacobian Z
    fe xn, yn, t;
    gxz_finish(xn, yn, t, acc);
    soa_store(rows.xyz, n, i, xn.n);
    soa_store(rows.xyz + 9 * (size_t)n, n, i, yn.n);
    soa_store(rows.xyz + 18 * (size_t)n, n, i, t.n);
}

// Batch inversion over the K messages of a lane as a product tree (K a power
// of two), node[i] = node[2i] node[2i+1] with the leaves at K .. 2K-1: K - 1
// products up, one inversion of the root, 2 (K - 1) products down
// (node[2i] <- node[i] node[2i+1], node[2i+1] <- node[i] node[2i]) -- the
// product count of Montgomery's trick, but at most log2 K products on any
// dependency chain instead of 3 (K - 1): the inversion kernels run one wave
// per SIMD, where a single chain leaves the SIMD waiting on each product.
// Every index is a compile-time constant (static_for), so node[] lives in
// registers.  A message that is not live takes the leaf 1.
//
// k_fast_zinv: K per lane, Z^-1 of the lane's live sums by that product
// tree (plain field products), into the pre row.  (k_fast_sinv keeps the
// linear walk: its Montgomery-form tree needs more registers than a wave has
// and spills -- measured 90 -> 100-129 us, while the tree takes zinv 76 -> 73.)
template <int K>
__global__ __launch_bounds__(256) void k_fast_zinv(uint32_t n, uint32_t T, SplitRows rows) {
    static_assert(K >= 2 && (K & (K - 1)) == 0, "K: a power of two");
    wave_prio(rows.prio);
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const uint32_t* zrow = rows.xyz + 18 * (size_t)n;
    fe node[2 * K];
    uint32_t live = 0;
    static_for<K>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const uint32_t i = (uint32_t)j * T + t;
        const uint32_t ic = i < n ? i : n - 1;
        const uint32_t a = rows.aux[ic];
        fe z;
        soa_load(z.n, zrow, n, ic);
        const bool on = i < n && (a & 0xFFu) == HD_FAST_LIVE;
        live |= on ? 1u << j : 0u;
        HD_UNROLL for (int k = 1; k < 9; k++) z.n[k] = on ? z.n[k] : 0u;
        z.n[0] = on ? z.n[0] : 1u;
        node[K + j] = z;
    });
    if (!live) return;
    static_for<K - 1>([&](auto ic) {
        constexpr int i = K - 1 - decltype(ic)::value;
        fe_mul(node[i], node[2 * i], node[2 * i + 1]);
    });
    fe_inv_divsteps(node[1], node[1]);   // a product of non-zero Z (and ones): never 0
    static_for<K - 1>([&](auto ic) {
        constexpr int i = 1 + decltype(ic)::value;
        fe a, b;
        fe_mul(a, node[i], node[2 * i + 1]);
        fe_mul(b, node[i], node[2 * i]);
        node[2 * i] = a;
        node[2 * i + 1] = b;
    });
    static_for<K>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if ((live >> j) & 1u) soa_store(rows.pre, n, (uint32_t)j * T + t, node[K + j].n);
    });
}

// x = r (+ n when v & 2) as a field element: the x coordinate of R (the range
// checks of sig_prefix passed in k_fast_prep)
HD void fast_rx(fe& x, const sc& r, uint32_t v) {
    uint32_t xw[8];
    HD_UNROLL for (int k = 0; k < 8; k++) xw[k] = r.v[k];
    if (v & 2) {
        const uint32_t N[8] = {HD_N0, HD_N1, HD_N2, HD_N3, HD_N4, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        uint64_t c = 0;
        HD_UNROLL for (int k = 0; k < 8; k++) { c += (uint64_t)xw[k] + N[k]; xw[k] = (uint32_t)c; c >>= 32; }
    }
    fe_from_le(x, xw);
}

// The comparison of message i (zi: the inverse of its stored ZZ ZZZ, read
// from the rows when null), its outputs when its verdict is final, its
// place on the fallback list, and its bit of the valid bitmap.  Every lane
// of the wavefront calls it together (ballots) for 64 consecutive, 64-aligned
// message indices; `present` is false past the batch.
__device__ __forceinline__ void cmp_one(const DevBatch& b, const SplitRows& rows, const int32_t* __restrict__ adm_perm,
                       uint8_t* __restrict__ verdict, uint8_t* __restrict__ rec32, int32_t* __restrict__ signer,
                       uint32_t* __restrict__ slow, uint32_t* __restrict__ n_slow, uint32_t* __restrict__ bitmap,
                       bool auth, uint32_t i, bool present, const fe* zi) {
    const uint32_t n = b.n;
    uint8_t v = HD_NEEDS_SLOW;
    if (present) {
        v = (uint8_t)(rows.aux[i] & 0xFFu);
        if (v == HD_FAST_LIVE) {
            fe xn, yn, w, x;
            soa_load(xn.n, rows.xyz, n, i);
            soa_load(yn.n, rows.xyz + 9 * (size_t)n, n, i);
            if (zi) w = *zi;
            else soa_load(w.n, rows.pre, n, i);
            sc r;
            soa_load(r.v, rows.u2, n, i);
            const uint32_t sv = b.sig65[65 * (size_t)i + 64];
            fast_rx(x, r, sv);
            v = fast_final_xz(xn, yn, w, x, sv);
            // authentication only: From's key does not give R, so the
            // recovered key is not From's -- final, without the recovery
            if (auth && v == HD_NEEDS_SLOW) v = V_NOT_AUTHENTIC;
            if (v == V_VALID && rows.idx[i] == -2) v = V_NOT_ADMITTED;   // a foreign key's check
        }
        if (v != HD_NEEDS_SLOW) {
            const bool ok = v == V_VALID;
            verdict[i] = v;
            if (rec32) {
                uint32_t f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                if (ok || (v == V_NOT_ADMITTED && rows.idx[i] == -2)) load_row32_be(f, b.from32, i);
                store_row32_be(rec32, i, f);
            }
            if (signer) signer[i] = ok ? adm_perm[rows.idx[i]] : -1;
        }
    }
    const bool to_slow = present && v == HD_NEEDS_SLOW;
    const unsigned long long bal = __ballot(to_slow);
    const uint32_t lane = threadIdx.x & 63u;
    if (bal) {
        const uint32_t leader = (uint32_t)__ffsll((long long)bal) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(n_slow, (uint32_t)__popcll(bal));
        base = __shfl(base, (int)leader);
        if (to_slow) slow[base + (uint32_t)__popcll(bal & ((1ull << lane) - 1))] = i;
    }
    if (bitmap) {
        const unsigned long long ok = __ballot(present && v == V_VALID);
        const uint32_t i0 = i - lane;   // multiple of 64
        if (lane == 0 && i0 < n) {
            bitmap[i0 >> 5] = (uint32_t)ok;
            if (i0 + 32 < n) bitmap[(i0 >> 5) + 1] = (uint32_t)(ok >> 32);
        }
    }
}

// One message per lane over a grid of whole wavefronts: the comparison of a
// live message, the outputs of every message that has its final verdict, the
// fallback list, and the valid bitmap -- a wavefront covers 64 consecutive
// messages, two bitmap words written from one ballot.  Messages handed to the
// full recovery get bit 0 here; k_verify sets theirs.
__global__ __launch_bounds__(256) void k_fast_cmp(DevBatch b, SplitRows rows, const int32_t* __restrict__ adm_perm,
                                                  uint8_t* __restrict__ verdict, uint8_t* __restrict__ rec32,
                                                  int32_t* __restrict__ signer, uint32_t* __restrict__ slow,
                                                  uint32_t* __restrict__ n_slow, uint32_t* __restrict__ bitmap,
                                                  bool auth) {
    wave_prio(rows.prio);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    cmp_one(b, rows, adm_perm, verdict, rec32, signer, slow, n_slow, bitmap, auth, i, i < b.n, nullptr);
}

// Before the full recovery of the leftovers: the reference's first checks
// and the lift of R (V >= 4, r / s range,
// r + n >= p, x^3 + 7 a square), in recover_m's order.  A message that fails
// one has its final verdict (nothing recovered) for one square-root chain,
// ~7 % of a recovery -- the "x not on the curve" adversarial class, and the
// malformed signatures of signatories without a known key; the rest go to
// the compacted list `out` (*n_out) that k_verify walks.  Leftovers are ~10 %
// of a 30 %-adversarial batch, so the saving is in the recovery's throughput
// cost, which overlapping calls expose.
//
// Round 4: a leftover that went through the known-key check (aux code still
// HD_FAST_LIVE, so m and s are in the rows) and lifts is tested for the
// INFINITY verdict with the fixed-base G table (fb_is_infinity: R == (m / s) G).
// That class -- cheap for anyone to craft (R = k G, s = m / k) -- then costs a
// scalar inversion and 11 additions instead of a full recovery each.
__global__ __launch_bounds__(256) void k_slow_lift(DevBatch b, const uint32_t* __restrict__ list,
                                                   const uint32_t* __restrict__ count, uint8_t* __restrict__ verdict,
                                                   uint8_t* __restrict__ rec32, int32_t* __restrict__ signer,
                                                   uint32_t* __restrict__ out, uint32_t* __restrict__ n_out,
                                                   int prio, uint32_t* __restrict__ est, SplitRows rows,
                                                   const gp* __restrict__ gtab) {
    wave_prio(prio);
    const uint32_t total = *count, stride = gridDim.x * blockDim.x;
    if (est && blockIdx.x == 0 && threadIdx.x == 0) est[0] = total;
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t base = blockIdx.x * blockDim.x; base < total; base += stride) {
        const uint32_t p = base + threadIdx.x;
        bool keep = false;
        uint32_t i = 0;
        if (p < total) {
            i = list[p];
            uint32_t r_be[8], s_be[8], v;
            load_sig65(r_be, s_be, v, b.sig65, i, b.n);
            sc r, s;
            fe x;
            uint8_t pre = sig_prefix(r, s, x, r_be, s_be, v);
            if (pre == V_VALID) {
                fe y2, y, seven;
                fe_sqr(y2, x);
                fe_mul(y2, y2, x);
                fe_set_u32(seven, 7);
                fe_add(y2, y2, seven);
                if (!fe_sqrt(y, y2)) {
                    pre = V_NO_POINT;
                } else if (gtab && rows.aux && (rows.aux[i] & 0xFFu) == HD_FAST_LIVE) {
                    ge R;
                    R.x = x;
                    R.y = y;
                    if (fe_is_odd(y) != ((v & 1u) != 0)) fe_neg(R.y, y);
                    sc m;   // (s is sig_prefix's; m as k_fast_prep left it)
                    soa_load(m.v, rows.u1, b.n, i);
                    if (fb_is_infinity<HD_FB_WG>(m, s, R, GpTab{gtab})) pre = V_INFINITY;
                }
            }
            keep = pre == V_VALID;
            if (!keep) {
                verdict[i] = pre;
                if (rec32) {
                    const uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                    store_row32_be(rec32, i, z);
                }
                if (signer) signer[i] = -1;
            }
        }
        const unsigned long long bal = __ballot(keep);
        if (bal) {
            const uint32_t leader = (uint32_t)__ffsll((long long)bal) - 1;
            uint32_t o = 0;
            if (lane == leader) o = atomicAdd(n_out, (uint32_t)__popcll(bal));
            o = __shfl(o, (int)leader);
            if (keep) out[o + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = i;
        }
    }
}

__global__ void k_fb_list(uint32_t nslots, const uint32_t* __restrict__ state, uint32_t* __restrict__ list,
                          uint32_t* __restrict__ count) {
    __shared__ uint32_t c;
    if (threadIdx.x == 0) c = 0;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nslots; k += blockDim.x)
        if (state[k] == HD_FB_LEARNED) list[atomicAdd(&c, 1u)] = k;
    __syncthreads();
    if (threadIdx.x == 0) *count = c;
}

template <int W>
__global__ __launch_bounds__(256) void k_fb_bases(const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                                                  const ge* __restrict__ pub, ge* __restrict__ base) {
    constexpr int NW = FbL<W>::NWIN;
    const uint32_t total = *count * NW;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        const uint32_t slot = list[t / NW], j = t % NW;
        ge o;
        fb_window_base(o, pub[slot], W, (int)j);
        base[(size_t)slot * NW + j] = o;
    }
}

// Table entries by segments of HD_FB_SEG consecutive multiples of one window
// base B: a lane computes the segment's first point d0 B once (double-and-add)
// and walks the rest with one mixed addition each, in blocks of HD_FB_RUN:
// the forward walk keeps each step's z ratio (Z_{k+1} = Z_k zr_k) and parks
// the Jacobian X, Y canonically in the entry's own 64-B table slot; one
// inversion of the block's last Z, then the backward walk makes each entry
// affine (1/Z_k = 1/Z_{k+1} zr_k).  Per entry one addition and ~5 products
// plus a share of one inversion, instead of a double-and-add and an
// inversion per entry (fb_entry, the definition the host tests check).
// The walk never adds B to +-B: its first point is d0 B with d0 >= 2 (d = 1
// is B itself, written directly), so (d0 + k) B = +-B cannot occur.
#define HD_FB_RUN 32
#define HD_FB_SEG 512
#define HD_FB_CHUNK 8   // slots per table allocation (fb_grow_slots)
template <int W>
__global__ __launch_bounds__(256) void k_fb_runs(const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                                                 const ge* __restrict__ base, gp* const* __restrict__ tabs,
                                                 uint32_t* __restrict__ zr_scratch) {
    constexpr uint32_t N = FbL<W>::N, NW = FbL<W>::NWIN;
    constexpr uint32_t SW = N / HD_FB_SEG;                                  // segments per full window
    constexpr uint32_t SB = (NW - 1) * SW + FbL<W>::NTOP / HD_FB_SEG;      // segments per base
    static_assert(N % HD_FB_SEG == 0 && FbL<W>::NTOP % HD_FB_SEG == 0 && HD_FB_SEG % HD_FB_RUN == 0, "segments");
    const uint32_t T = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t total = (uint64_t)*count * SB;
    for (uint64_t g = tid; g < total; g += T) {
        const uint32_t slot = list[g / SB];
        const uint32_t rem = (uint32_t)(g % SB);
        const uint32_t j = min(rem / SW, NW - 1);
        const uint32_t d0 = 1 + (rem - j * SW) * HD_FB_SEG;
        const ge B = base[(size_t)slot * NW + j];
        gp* out = tabs[slot] + (size_t)j * N + (d0 - 1);
        gej a;
        uint32_t k0 = 0;   // first entry of the segment the walk produces
        if (d0 == 1) {
            gp q;
            gp_pack(q, B);   // bases are canonical affine
            out[0] = q;
            gej b;
            gej_set_ge(b, B);
            gej_dbl(a, b);
            k0 = 1;
        } else {
            fb_mul_small(a, B, d0);
        }
        for (uint32_t blk = 0; blk < HD_FB_SEG; blk += HD_FB_RUN) {
            const uint32_t lo = blk + (blk == 0 ? k0 : 0), hi = blk + HD_FB_RUN;
            HD_NOUNROLL for (uint32_t k = lo; k < hi; k++) {
                if (k > lo) {
                    fe zr;
                    gej_add_ge_zr(a, a, B, zr);
                    HD_UNROLL for (int w = 0; w < 9; w++)
                        zr_scratch[((size_t)(k - 1 - blk) * 9 + w) * T + tid] = zr.n[w];
                }
                fe x = a.x, y = a.y;
                fe_normalize(x);
                fe_normalize(y);
                gp q;
                fe_to_le(q.x, x);
                fe_to_le(q.y, y);
                out[k] = q;
            }
            fe zinv;
            fe_inv_divsteps(zinv, a.z);
            HD_NOUNROLL for (uint32_t k = hi; k-- > lo;) {
                ge p;
                gp_unpack(p, out[k]);
                fe z2, ax, ay;
                fe_sqr(z2, zinv);
                fe_mul(ax, p.x, z2);
                fe_mul(z2, z2, zinv);
                fe_mul(ay, p.y, z2);
                fe_normalize(ax);
                fe_normalize(ay);
                gp q;
                fe_to_le(q.x, ax);
                fe_to_le(q.y, ay);
                out[k] = q;
                if (k > lo) {
                    fe zr;
                    HD_UNROLL for (int w = 0; w < 9; w++) zr.n[w] = zr_scratch[((size_t)(k - 1 - blk) * 9 + w) * T + tid];
                    fe_mul(zinv, zinv, zr);
                }
            }
            // the next block continues the walk from this block's last point
            if (hi < HD_FB_SEG) {
                fe zr;
                gej_add_ge_zr(a, a, B, zr);
            }
        }
    }
}

// One block.  not_ready counts admitted slots only: the foreign block
// [f0, f1) is left out, counted inside the parallel walk (one LDS atomic per
// thread), so a set change that builds 10^5-10^6 admitted tables pays no
// serial walk over the list.
__global__ void k_fb_ready(const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                           uint32_t* __restrict__ state, uint32_t* not_ready, uint32_t f0, uint32_t f1) {
    __shared__ uint32_t sh_admitted;
    const uint32_t c = *count;
    if (threadIdx.x == 0) sh_admitted = 0;
    __syncthreads();
    uint32_t mine = 0;
    for (uint32_t k = threadIdx.x; k < c; k += blockDim.x) {
        const uint32_t sl = list[k];
        state[sl] = HD_FB_READY;
        mine += (sl >= f0 && sl < f1) ? 0u : 1u;
    }
    if (mine) atomicAdd(&sh_admitted, mine);
    __syncthreads();
    if (threadIdx.x == 0 && c && not_ready) {
        const uint32_t ca = sh_admitted;
        const uint32_t v = *(volatile uint32_t*)not_ready;
        *(volatile uint32_t*)not_ready = v >= ca ? v - ca : 0u;
    }
}

// per-key table geometry of width wp
size_t fb_tab_entries(int wp) {
    return wp == HD_FB_WX   ? FbL<HD_FB_WX>::TAB
           : wp == HD_FB_WW ? FbL<HD_FB_WW>::TAB
           : wp == HD_FB_WN ? FbL<HD_FB_WN>::TAB
                            : FbL<HD_FB_W>::TAB;
}
int fb_nwin(int wp) {
    return wp == HD_FB_WX   ? FbL<HD_FB_WX>::NWIN
           : wp == HD_FB_WW ? FbL<HD_FB_WW>::NWIN
           : wp == HD_FB_WN ? FbL<HD_FB_WN>::NWIN
                            : FbL<HD_FB_W>::NWIN;
}
double fb_slot_bytes(int wp) {
    return (double)sizeof(gp) * (double)fb_tab_entries(wp) + (double)sizeof(ge) * (fb_nwin(wp) + 1) + 8;
}

// table bytes held by all contexts of a device (the budget is per device)
std::mutex g_fb_bytes_mutex;
std::map<int, size_t> g_fb_bytes;
void fb_account(hd_ctx* ctx, size_t add, size_t sub) {
    std::lock_guard<std::mutex> lock(g_fb_bytes_mutex);
    size_t& d = g_fb_bytes[ctx->device];
    d = d + add - std::min(d, sub);
    ctx->fb->bytes = ctx->fb->bytes + add - std::min(ctx->fb->bytes, sub);
}
size_t fb_device_bytes(int device) {
    std::lock_guard<std::mutex> lock(g_fb_bytes_mutex);
    return g_fb_bytes[device];
}

void fb_free_tables(hd_ctx* ctx) {
    FbWork* f = ctx->fb;
    for (gp* c : f->chunks) (void)hipFree(c);
    f->chunks.clear();
    void* ptrs[] = {f->tabs, f->base, f->pub, f->state, f->list};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    f->tabs = nullptr;
    f->base = f->pub = nullptr;
    f->state = f->list = nullptr;
    f->nslots = 0;
    fb_account(ctx, 0, f->bytes);
}

// The per-slot arrays for max_slots slots (small: bases, keys, states, table
// pointers), once per table width; no table memory yet.
int fb_alloc_slots(hd_ctx* ctx) {
    FbWork* f = ctx->fb;
    const size_t m = f->max_slots, NWIN = (size_t)fb_nwin(f->wp);
    FBCHK(hipMalloc(&f->tabs, sizeof(gp*) * m), "fb table pointers");
    FBCHK(hipMalloc(&f->base, sizeof(ge) * NWIN * m), "fb bases");
    FBCHK(hipMalloc(&f->pub, sizeof(ge) * m), "fb keys");
    FBCHK(hipMalloc(&f->state, 4 * m), "fb state");
    FBCHK(hipMalloc(&f->list, 4 * m), "fb list");
    FBCHK(hipMemsetAsync(f->state, 0, 4 * m, ctx->stream), "fb state clear");
    FBCHK(hipMemsetAsync(f->tabs, 0, sizeof(gp*) * m, ctx->stream), "fb table pointers clear");
    FBCHK(hipStreamSynchronize(ctx->stream), "fb slot arrays");
    fb_account(ctx, (sizeof(gp*) + sizeof(ge) * (NWIN + 1) + 8) * m, 0);
    return HD_OK;
}

// Table chunks until `want` slots have tables (chunks never move: the slots
// already built keep their tables).
int fb_grow_slots(hd_ctx* ctx, uint32_t want) {
    FbWork* f = ctx->fb;
    want = std::min(want, f->max_slots);
    const size_t TAB = fb_tab_entries(f->wp);
    // test hook: HD_FB_FAIL_WIDTH=w fails every table allocation at width w
    // as the device would when another process took the memory
    // (tests/test_fastpath.py: the narrower-width retry of hd_fb_map_signatories)
    if (const char* fw = getenv("HD_FB_FAIL_WIDTH"))
        if (atoi(fw) == f->wp && f->nslots < want) return hd_ctx_fail(ctx, hipErrorOutOfMemory, "fb table chunk (HD_FB_FAIL_WIDTH)");
    while (f->nslots < want) {
        const uint32_t k = std::min<uint32_t>(HD_FB_CHUNK, f->max_slots - f->nslots);
        gp* c = nullptr;
        FBCHK(hipMalloc(&c, sizeof(gp) * TAB * k), "fb table chunk");
        f->chunks.push_back(c);
        std::vector<gp*> ptr(k);
        for (uint32_t j = 0; j < k; j++) ptr[j] = c + TAB * j;
        FBCHK(hipMemcpyAsync(f->tabs + f->nslots, ptr.data(), sizeof(gp*) * k, hipMemcpyHostToDevice, ctx->stream),
              "fb table pointers");
        FBCHK(hipStreamSynchronize(ctx->stream), "fb table pointers");
        f->nslots += k;
        fb_account(ctx, sizeof(gp) * TAB * k, 0);
    }
    return HD_OK;
}

// k_fb_runs grid (4 blocks per CU) and its z-ratio scratch
uint32_t fb_run_blocks(const hd_ctx* ctx) { return (uint32_t)std::max(ctx->n_cu, 1) * 4u; }
size_t fb_run_scratch_bytes(const hd_ctx* ctx) { return (size_t)HD_FB_RUN * 9 * 4 * 256 * fb_run_blocks(ctx); }

// build the tables of every LEARNED slot, stream-ordered (nothing to launch
// once every mapped key is READY)
// a foreign key claimed since the last build (HD_VAR_FOREIGN_KEYS)
static bool fb_foreign_pending(const FbWork* f) {
    return f->fcap && f->fpend_host && *(volatile uint32_t*)f->fpend_host != f->fseen;
}

int fb_learn(hd_ctx* ctx, hipStream_t s) {
    FbWork* f = ctx->fb;
    const bool fnew = fb_foreign_pending(f);
    if (f->nr_host && *(volatile uint32_t*)f->nr_host == 0 && !fnew && !f->fforce) return HD_OK;
    if (fnew) f->fseen = *(volatile uint32_t*)f->fpend_host;
    f->fforce = false;
    const uint32_t g = (uint32_t)std::max(ctx->n_cu, 1) * 4u;
    k_fb_list<<<1, 256, 0, s>>>(f->nslots, f->state, f->list, f->counts);
    if (f->wp == HD_FB_WX) {
        k_fb_bases<HD_FB_WX><<<g, 256, 0, s>>>(f->list, f->counts, f->pub, f->base);
        k_fb_runs<HD_FB_WX><<<fb_run_blocks(ctx), 256, 0, s>>>(f->list, f->counts, f->base, f->tabs, f->zr);
    } else if (f->wp == HD_FB_WW) {
        k_fb_bases<HD_FB_WW><<<g, 256, 0, s>>>(f->list, f->counts, f->pub, f->base);
        k_fb_runs<HD_FB_WW><<<fb_run_blocks(ctx), 256, 0, s>>>(f->list, f->counts, f->base, f->tabs, f->zr);
    } else if (f->wp == HD_FB_WN) {
        k_fb_bases<HD_FB_WN><<<g, 256, 0, s>>>(f->list, f->counts, f->pub, f->base);
        k_fb_runs<HD_FB_WN><<<fb_run_blocks(ctx), 256, 0, s>>>(f->list, f->counts, f->base, f->tabs, f->zr);
    } else {
        k_fb_bases<HD_FB_W><<<g, 256, 0, s>>>(f->list, f->counts, f->pub, f->base);
        k_fb_runs<HD_FB_W><<<fb_run_blocks(ctx), 256, 0, s>>>(f->list, f->counts, f->base, f->tabs, f->zr);
    }
    k_fb_ready<<<1, 256, 0, s>>>(f->list, f->counts, f->state, f->nr_dev, f->fbase, f->fbase + f->fres);
    FBCHK(hipGetLastError(), "fb table kernels");
    return HD_OK;
}

// the foreign block's host-side state after its dictionary was emptied
void fb_foreign_forget(FbWork* f) {
    ((volatile uint32_t*)f->fpend_host)[0] = 0;
    ((volatile uint32_t*)f->fpend_host)[1] = 0;
    f->fseen = 0;
    f->fwait = 1;
    f->fcalls = 0;
    f->fforce = false;
}

// Foreign-slot eviction.  The fcap foreign slots go to the first Froms whose
// NOT_ADMITTED recovery claims them; later Froms stay in the dictionary
// without a slot (key kept, recoveries counted).  While such recoveries are
// flagged, every fwait-th call (fwait doubling up to HD_FD_EVICT_WAIT_MAX
// while checks change nothing) waits for the context's calls to finish --
// nothing may read a table about to be re-keyed -- and reads the counters:
// the slotless Froms by recoveries since the last check, hottest first, take
// the slots of the READY foreign keys with the fewest known-key checks while
// hot >= 2 cold + 4 (hysteresis: two senders of similar rates do not trade
// places every check).  A demoted From keeps its key and may come back;
// slotless entries without a recovery since the last check leave the
// dictionary (throwaway Froms cannot fill its 128 buckets either).  The
// dictionary is rebuilt on the host and uploaded, the counters restart, and
// the promoted slots (state LEARNED) are built at this call's end
// (fforce).  Verdicts never depend on it: a slot that is not READY sends its
// messages to the full recovery.
#define HD_FD_EVICT_WAIT_MAX 1024u
int fb_evict(hd_ctx* ctx, bool* changed) {
    FbWork* f = ctx->fb;
    *changed = false;
    if (!f->fcap || !f->fhit || !f->fkey || !f->fdict) return HD_OK;
    volatile uint32_t* miss = (volatile uint32_t*)f->fpend_host + 1;
    if (*miss == 0) return HD_OK;
    if (++f->fcalls < f->fwait) return HD_OK;
    f->fcalls = 0;
    int rq = hd_fb_quiesce(ctx);
    if (rq) return rq;
    *miss = 0;
    f->evict_checks++;
    hipStream_t s = ctx->stream;
    const uint32_t B = HD_FD_BUCKETS, R = f->fres;
    std::vector<uint32_t> fd(HD_FD_WORDS), hit(64 + B), st(R);
    std::vector<ge> key(B), pub(R);
    FBCHK(hipMemcpyAsync(fd.data(), f->fdict, 4 * (size_t)HD_FD_WORDS, hipMemcpyDeviceToHost, s), "evict read");
    FBCHK(hipMemcpyAsync(hit.data(), f->fhit, 4 * hit.size(), hipMemcpyDeviceToHost, s), "evict read");
    FBCHK(hipMemcpyAsync(key.data(), f->fkey, sizeof(ge) * B, hipMemcpyDeviceToHost, s), "evict read");
    FBCHK(hipMemcpyAsync(pub.data(), f->pub + f->fbase, sizeof(ge) * R, hipMemcpyDeviceToHost, s), "evict read");
    FBCHK(hipMemcpyAsync(st.data(), f->state + f->fbase, 4 * (size_t)R, hipMemcpyDeviceToHost, s), "evict read");
    FBCHK(hipStreamSynchronize(s), "evict read");
    struct Ent {
        uint32_t from[8];
        uint32_t slot, hits;
        ge key;
        bool moved;
    };
    std::vector<Ent> held, loose;
    for (uint32_t b = 0; b < B; b++) {
        if (fd[b] != 2u) continue;
        Ent e;
        memcpy(e.from, &fd[2 * B + 8 * b], 32);
        e.slot = fd[B + b];
        e.moved = false;
        if (e.slot != 0xFFFFFFFFu && e.slot >= f->fbase && e.slot < f->fbase + R) {
            e.hits = hit[e.slot - f->fbase];
            e.key = pub[e.slot - f->fbase];
            held.push_back(e);
        } else {
            e.slot = 0xFFFFFFFFu;
            e.hits = hit[64 + b];
            e.key = key[b];
            loose.push_back(e);
        }
    }
    std::stable_sort(loose.begin(), loose.end(), [](const Ent& a, const Ent& b) { return a.hits > b.hits; });
    std::vector<Ent*> cold;
    for (Ent& e : held)
        if (st[e.slot - f->fbase] == HD_FB_READY) cold.push_back(&e);   // built slots only: a new one had no chance
    std::stable_sort(cold.begin(), cold.end(), [](const Ent* a, const Ent* b) { return a->hits < b->hits; });
    std::vector<Ent> promoted;
    size_t swaps = 0;
    while (swaps < loose.size() && swaps < cold.size() && loose[swaps].hits >= 2 * cold[swaps]->hits + 4) {
        Ent& hot = loose[swaps];
        Ent* old = cold[swaps];
        hot.slot = old->slot;
        hot.moved = true;
        old->slot = 0xFFFFFFFFu;
        old->moved = true;
        promoted.push_back(hot);
        swaps++;
    }
    // the new dictionary: slot holders first (they always fit: at most 64 of
    // 128 buckets), then the slotless Froms worth keeping
    std::vector<Ent> keep;
    for (const Ent& e : held) keep.push_back(e);
    for (const Ent& e : loose)
        if (e.moved || e.hits > 0) keep.push_back(e);
    std::stable_partition(keep.begin(), keep.end(), [](const Ent& e) { return e.slot != 0xFFFFFFFFu; });
    const bool dropped = keep.size() < held.size() + loose.size();
    if (swaps == 0 && !dropped) {
        f->fwait = std::min(2 * f->fwait, HD_FD_EVICT_WAIT_MAX);
        FBCHK(hipMemsetAsync(f->fhit, 0, 4 * hit.size(), s), "evict counters");
        FBCHK(hipStreamSynchronize(s), "evict counters");
        return HD_OK;
    }
    std::vector<uint32_t> nd(HD_FD_WORDS, 0u), efrom(8 * keep.size() + 8), eslot(keep.size() + 1);
    std::vector<int32_t> where(keep.size() + 1);
    for (size_t k = 0; k < keep.size(); k++) {
        memcpy(&efrom[8 * k], keep[k].from, 32);
        eslot[k] = keep[k].slot;
    }
    if (!fdict_rebuild(nd.data(), where.data(), efrom.data(), eslot.data(), (uint32_t)keep.size())) {
        // a slot holder would find no bucket: keep the old dictionary and
        // slots for this pass (fdict_rebuild)
        f->evict_aborts++;
        f->fwait = std::min(2 * f->fwait, HD_FD_EVICT_WAIT_MAX);
        FBCHK(hipMemsetAsync(f->fhit, 0, 4 * hit.size(), s), "evict counters");
        FBCHK(hipStreamSynchronize(s), "evict counters");
        return HD_OK;
    }
    std::vector<ge> nkey(B);
    for (size_t k = 0; k < keep.size(); k++)
        if (where[k] >= 0) nkey[where[k]] = keep[k].key;
    FBCHK(hipMemcpyAsync(f->fdict, nd.data(), 4 * (size_t)HD_FD_WORDS, hipMemcpyHostToDevice, s), "evict write");
    FBCHK(hipMemcpyAsync(f->fkey, nkey.data(), sizeof(ge) * B, hipMemcpyHostToDevice, s), "evict write");
    FBCHK(hipMemsetAsync(f->fhit, 0, 4 * hit.size(), s), "evict counters");
    const uint32_t learned = HD_FB_LEARNED;
    for (const Ent& e : promoted) {
        FBCHK(hipMemcpyAsync(f->pub + e.slot, &e.key, sizeof(ge), hipMemcpyHostToDevice, s), "evict key");
        FBCHK(hipMemcpyAsync(f->state + e.slot, &learned, 4, hipMemcpyHostToDevice, s), "evict state");
    }
    FBCHK(hipStreamSynchronize(s), "evict write");
    f->fwait = swaps ? 1u : std::min(2 * f->fwait, HD_FD_EVICT_WAIT_MAX);
    f->fforce = swaps > 0;
    f->evictions += (uint32_t)swaps;
    *changed = true;
    return HD_OK;
}

}  // namespace

// The G table (W = HD_FB_WG) is built once per device and process and shared
// by every context on that device.
static std::mutex g_fb_g_mutex;
static std::map<int, gp*> g_fb_g_tables;

static int fb_g_table(hd_ctx* ctx, const gp** out) {
    std::lock_guard<std::mutex> lock(g_fb_g_mutex);
    auto it = g_fb_g_tables.find(ctx->device);
    if (it != g_fb_g_tables.end()) {
        *out = it->second;
        return HD_OK;
    }
    ge g;
    const uint32_t GX[8] = {0x79BE667Eu, 0xF9DCBBACu, 0x55A06295u, 0xCE870B07u,
                            0x029BFCDBu, 0x2DCE28D9u, 0x59F2815Bu, 0x16F81798u};
    const uint32_t GY[8] = {0x483ADA77u, 0x26A3C465u, 0x5DA4FBFCu, 0x0E1108A8u,
                            0xFD17B448u, 0xA6855419u, 0x9C47D08Fu, 0xFB10D4B8u};
    fe_from_be(g.x, GX);
    fe_from_be(g.y, GY);
    gp* tab = nullptr;
    gp** tp = nullptr;       // the builder's table pointer array: {tab}
    ge *base = nullptr, *pub = nullptr;
    uint32_t* cl = nullptr;  // [0] = list {0}, [1] = count 1
    FBCHK(hipMalloc(&tab, sizeof(gp) * (size_t)FbL<HD_FB_WG>::TAB), "G table");
    FBCHK(hipMalloc(&tp, sizeof(gp*)), "G table pointer");
    FBCHK(hipMalloc(&base, sizeof(ge) * FbL<HD_FB_WG>::NWIN), "G bases");
    FBCHK(hipMalloc(&pub, sizeof(ge)), "G point");
    FBCHK(hipMalloc(&cl, 8), "G list");
    const uint32_t hl[2] = {0u, 1u};
    hipStream_t s = ctx->stream;
    FBCHK(hipMemcpyAsync(pub, &g, sizeof(ge), hipMemcpyHostToDevice, s), "G point");
    FBCHK(hipMemcpyAsync(cl, hl, 8, hipMemcpyHostToDevice, s), "G list");
    FBCHK(hipMemcpyAsync(tp, &tab, sizeof(gp*), hipMemcpyHostToDevice, s), "G table pointer");
    k_fb_bases<HD_FB_WG><<<1, 64, 0, s>>>(cl, cl + 1, pub, base);
    k_fb_runs<HD_FB_WG><<<fb_run_blocks(ctx), 256, 0, s>>>(cl, cl + 1, base, tp, ctx->fb->zr);
    FBCHK(hipGetLastError(), "G table kernels");
    FBCHK(hipStreamSynchronize(s), "G table build");
    (void)hipFree(base);
    (void)hipFree(pub);
    (void)hipFree(cl);
    (void)hipFree(tp);
    g_fb_g_tables[ctx->device] = tab;
    *out = tab;
    return HD_OK;
}

int hd_fb_init(hd_ctx* ctx) {
    if (ctx->fb) return HD_OK;
    ctx->fb = new (std::nothrow) FbWork();
    if (!ctx->fb) return HD_ENOMEM;
    FbWork* f = ctx->fb;
    // the device's table budget: HD_FB_MAX_BYTES, else 64 GiB -- room for
    // the headline's 100 signatories at 20 bits beside the G table and
    // everything else the process keeps resident (its batches, torch's
    // cache, more contexts).  A budget of 3/4 of the device (216 GB: 22-bit
    // tables for 100 keys, one addition fewer) measured the same headline
    // within noise and starved the process's other allocations; a replica
    // that owns its GPU may still set it.
    f->budget = 64.0 * (1ull << 30);
    if (const char* m = getenv("HD_FB_MAX_BYTES")) f->budget = atof(m);
    f->max_slots = (uint32_t)std::max(1.0, std::min(1e6, f->budget / fb_slot_bytes(f->wp)));
    FBCHK(hipMalloc(&f->counts, 8), "fb counts");
    FBCHK(hipMalloc(&f->zr, fb_run_scratch_bytes(ctx)), "fb builder scratch");
    FBCHK(hipHostMalloc((void**)&f->nr_host, 4, hipHostMallocMapped | hipHostMallocCoherent), "fb ready count");
    *f->nr_host = 0xFFFFFFFFu;
    FBCHK(hipHostGetDevicePointer((void**)&f->nr_dev, f->nr_host, 0), "fb ready count map");
    FBCHK(hipHostMalloc((void**)&f->est_host, 8, hipHostMallocMapped | hipHostMallocCoherent), "fb list estimate");
    f->est_host[0] = f->est_host[1] = 0xFFFFFFFFu;
    FBCHK(hipHostGetDevicePointer((void**)&f->est_dev, f->est_host, 0), "fb list estimate map");
    FBCHK(hipHostMalloc((void**)&f->fpend_host, 8, hipHostMallocMapped | hipHostMallocCoherent), "fb foreign claims");
    f->fpend_host[0] = f->fpend_host[1] = 0;
    FBCHK(hipHostGetDevicePointer((void**)&f->fpend_dev, f->fpend_host, 0), "fb foreign claims map");
    int rc = fb_alloc_slots(ctx);
    if (rc) return rc;
    return fb_g_table(ctx, &f->gtab);
}

const gp* hd_fb_gtab(const hd_ctx* ctx) { return ctx && ctx->fb ? ctx->fb->gtab : nullptr; }

void hd_fb_release(hd_ctx* ctx) {
    if (!ctx || !ctx->fb) return;
    FbWork* f = ctx->fb;
    fb_free_tables(ctx);
    if (f->done) (void)hipEventDestroy(f->done);
    for (hipEvent_t e : f->ev_call) (void)hipEventDestroy(e);
    for (hipEvent_t e : f->ev_sums) (void)hipEventDestroy(e);
    for (auto& sc : f->sc) {
        if (sc.done) (void)hipEventDestroy(sc.done);
        void* sp[] = {sc.rows, sc.slow, sc.count, sc.slow2};
        for (void* p : sp)
            if (p) (void)hipFree(p);
    }
    void* ptrs[] = {f->counts, f->adm_slot, f->zr, f->fdict, f->fnext, f->fhit, f->fkey};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (f->nr_host) (void)hipHostFree(f->nr_host);
    if (f->est_host) (void)hipHostFree(f->est_host);
    if (f->fpend_host) (void)hipHostFree(f->fpend_host);
    delete f;
    ctx->fb = nullptr;
}

// Messages per inversion of the known-key check (HD_VAR_SPLIT_K): 8 or 16;
// -1 (default) by batch size: 16 from 2^20 - 2^16 messages up (65,536 lanes,
// one wave per SIMD), else 8.  The inversion kernels are bound by their
// dependent ALU chains; halving the inversions outweighs the lost second wave
// per SIMD (1M C2 messages, one box, scalars and prefixes in registers:
// k_fast_sinv 102 -> 91 us, k_fast_zinv 91 -> 76 us from K = 8 to 16; with the
// rows in HBM between steps K = 4 / 8 / 16 gave 177 / 111 / 90 and 166 / 102
// / 85 us)
static int split_k_for(const hd_ctx* ctx, uint32_t n) {
    const int k = ctx->var[HD_VAR_SPLIT_K];
    if (k > 0) return k;
    return n >= (1u << 20) - (1u << 16) ? 16 : 8;
}

// Per-key window width for an admitted set of m: the widest tables
// (HD_FB_WX, 12 windows of u2, 1.48 GB per key) when all m keys and the
// foreign-key block fit the device's table budget next to what other contexts
// hold; else the wide ones (HD_FB_WW, 13 windows, 407 MB) when the m keys do;
// else the 16-bit
// ones (16 windows, 36 MB) when all m keys fit the context's budget; else the
// narrow ones (HD_FB_WN, 20 windows, 5 MB), so that thousands of signatories
// still take the known-key check instead of the full recovery (a key
// without a slot costs ~10x per message).  HD_VAR_KEY_WIDTH forces one.
// The table bytes the device can still give this context: its free memory
// (other processes' allocations included) plus what this context holds.
static double fb_free_cap(hd_ctx* ctx) {
    size_t fr = 0, tot = 0;
    (void)hipSetDevice(ctx->device);
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 1e300;
    return 0.9 * (double)fr + (double)ctx->fb->bytes;
}

// (cap: the widest width allowed, 0 = any; hd_fb_map_signatories narrows it
// when an allocation fails)
static int fb_pick_width(hd_ctx* ctx, uint32_t m, int cap) {
    if (ctx->var[HD_VAR_KEY_WIDTH]) return ctx->var[HD_VAR_KEY_WIDTH];
    FbWork* f = ctx->fb;
    const double others = (double)(fb_device_bytes(ctx->device) - std::min(fb_device_bytes(ctx->device), f->bytes));
    const double free_cap = fb_free_cap(ctx);
    const double shared = std::min(f->budget - others, free_cap);
    // (+ the foreign-key block's slots)
    const double slots = (double)m + 1 + (ctx->var[HD_VAR_FOREIGN_KEYS] > 0 ? ctx->var[HD_VAR_FOREIGN_KEYS] : 0);
    const auto allowed = [cap](int w) { return cap == 0 || w <= cap; };
    if (allowed(HD_FB_WX) && fb_slot_bytes(HD_FB_WX) * slots <= shared) return HD_FB_WX;
    if (allowed(HD_FB_WW) && fb_slot_bytes(HD_FB_WW) * ((double)m + 1) <= shared) return HD_FB_WW;
    if (allowed(HD_FB_W) && fb_slot_bytes(HD_FB_W) * slots <= std::min(f->budget, free_cap)) return HD_FB_W;
    return HD_FB_WN;
}

// mapped slots whose state is not READY (device idle: called after a sync)
static int fb_count_not_ready(hd_ctx* ctx) {
    FbWork* f = ctx->fb;
    uint32_t nr = 0;
    if (!f->slot_of.empty()) {
        std::vector<uint32_t> st(f->nslots);
        FBCHK(hipMemcpyAsync(st.data(), f->state, 4 * (size_t)f->nslots, hipMemcpyDeviceToHost, ctx->stream),
              "fb state read");
        FBCHK(hipStreamSynchronize(ctx->stream), "fb state read");
        for (const auto& kv : f->slot_of) nr += st[kv.second] != HD_FB_READY ? 1u : 0u;
    }
    *(volatile uint32_t*)f->nr_host = nr;
    return HD_OK;
}

static int fb_map(hd_ctx* ctx, const uint8_t* sorted, uint32_t m, int cap);

// HD_FB_TRACE=1: one stderr line per table-mapping attempt (debug aid)
static bool fb_trace() {
    static const bool on = getenv("HD_FB_TRACE") != nullptr;
    return on;
}

// One table mapping at a time per device: the width pick reads the bytes
// the device's other contexts hold and its free memory, so contexts mapping
// concurrently (hd_multi's per-device threads over one GPU) would each count
// the memory the others are about to take and oversubscribe the device.
static std::mutex g_fb_map_mutex[64];

// Map the admitted set to table slots.  A table allocation the device
// cannot serve (another process took the memory since the width was picked)
// retries at the next narrower width, down to 13 bits, instead of failing
// the set change.
int hd_fb_map_signatories(hd_ctx* ctx, const uint8_t* sorted, uint32_t m) {
    std::lock_guard<std::mutex> lock(g_fb_map_mutex[(unsigned)ctx->device % 64u]);
    int rc = HD_OK;
    for (int cap : {0, HD_FB_WW, HD_FB_W, HD_FB_WN}) {
        if (fb_trace()) {
            size_t fr = 0, tot = 0;
            (void)hipMemGetInfo(&fr, &tot);
            fprintf(stderr, "[fb] ctx %p m %u cap %d: wp %d nslots %u used %u max %u bytes %.2fG dev %.2fG free %.2fG\n",
                    (void*)ctx, m, cap, ctx->fb->wp, ctx->fb->nslots, ctx->fb->used, ctx->fb->max_slots,
                    ctx->fb->bytes / 1e9, fb_device_bytes(ctx->device) / 1e9, fr / 1e9);
        }
        rc = fb_map(ctx, sorted, m, cap);
        if (fb_trace())
            fprintf(stderr, "[fb] ctx %p -> rc %d wp %d nslots %u used %u %s\n", (void*)ctx, rc, ctx->fb->wp,
                    ctx->fb->nslots, ctx->fb->used, rc ? ctx->last_error.c_str() : "");
        if (rc != HD_ENOMEM || ctx->var[HD_VAR_KEY_WIDTH]) break;
        (void)hipGetLastError();   // the failed allocation must not surface in a later launch check
    }
    // a set change that failed here leaves slots mapped without tables (and
    // the device's slot map of the previous set): until a mapping succeeds,
    // every message takes the full recovery against the new admitted set
    ctx->fb->map_ok = rc == HD_OK;
    return rc;
}

static int fb_map(hd_ctx* ctx, const uint8_t* sorted, uint32_t m, int cap) {
    FbWork* f = ctx->fb;
    // no verify call of this context may still learn into a slot reassigned
    // here (hd_set_signatories quiesced the context already)
    int rq = hd_ctx_quiesce(ctx);
    if (rq) return rq;
    *(volatile uint32_t*)f->nr_host = 0xFFFFFFFFu;
    const int wp = fb_pick_width(ctx, m, cap);
    if (wp != f->wp || (cap && f->nslots < f->used)) {
        // another table width: every key is learned again (full recovery)
        fb_free_tables(ctx);
        f->slot_of.clear();
        f->free_slots.clear();
        f->used = 1;
        f->fcap = f->fres = 0;   // the foreign block goes with the tables
        f->wp = wp;
        f->max_slots =
            (uint32_t)std::max(1.0, std::min(1e6, std::min(f->budget, fb_free_cap(ctx)) / fb_slot_bytes(wp)));
        int ra = fb_alloc_slots(ctx);
        if (ra) return ra;
    }
    std::unordered_map<std::string, uint32_t> keep;
    std::vector<int32_t> adm_slot(std::max(m, 1u), -1);
    std::vector<uint32_t> fresh;
    for (uint32_t k = 0; k < m; k++) {
        std::string key(reinterpret_cast<const char*>(sorted + 32 * (size_t)k), 32);
        auto it = f->slot_of.find(key);
        if (it != f->slot_of.end()) {
            adm_slot[k] = (int32_t)it->second;
            keep.emplace(key, it->second);
            f->slot_of.erase(it);
        }
    }
    // signatories no longer admitted give their slots back
    for (auto& kv : f->slot_of) {
        f->free_slots.push_back(kv.second);
        fresh.push_back(kv.second);
    }
    f->slot_of.swap(keep);
    for (uint32_t k = 0; k < m; k++) {
        if (adm_slot[k] >= 0) continue;
        uint32_t slot;
        if (!f->free_slots.empty()) {
            slot = f->free_slots.back();
            f->free_slots.pop_back();
        } else if (f->used < f->max_slots) {
            slot = f->used++;
        } else {
            continue;  // over the slot cap: this signatory always takes the full recovery
        }
        adm_slot[k] = (int32_t)slot;
        f->slot_of.emplace(std::string(reinterpret_cast<const char*>(sorted + 32 * (size_t)k), 32), slot);
        fresh.push_back(slot);
    }
    // foreign keys: a block of slots reserved once, after the admitted ones
    // of the first set that asks for it; emptied (dictionary and states) on
    // every set change -- a From that leaves or joins the set is learned again
    const uint32_t want = (uint32_t)std::max(0, ctx->var[HD_VAR_FOREIGN_KEYS]);
    if (want && !f->fres && f->used + want <= f->max_slots) {
        f->fbase = f->used;
        f->fres = want;
        f->used += want;
    }
    f->fcap = std::min(want, f->fres);   // 0: no foreign learning until a set change asks again
    int rc = fb_grow_slots(ctx, f->used);
    if (rc) return rc;
    hipStream_t s = ctx->stream;
    for (uint32_t slot : fresh) FBCHK(hipMemsetAsync(f->state + slot, 0, 4, s), "fb slot reset");
    if (f->fres) {
        if (!f->fdict) FBCHK(hipMalloc(&f->fdict, 4 * (size_t)HD_FD_WORDS), "fb foreign dictionary");
        if (!f->fnext) FBCHK(hipMalloc(&f->fnext, 4), "fb foreign count");
        if (!f->fhit) FBCHK(hipMalloc(&f->fhit, 4 * (64 + (size_t)HD_FD_BUCKETS)), "fb foreign hits");
        if (!f->fkey) FBCHK(hipMalloc(&f->fkey, sizeof(ge) * HD_FD_BUCKETS), "fb foreign keys");
        FBCHK(hipMemsetAsync(f->fdict, 0, 4 * (size_t)HD_FD_WORDS, s), "fb foreign reset");
        FBCHK(hipMemsetAsync(f->fnext, 0, 4, s), "fb foreign reset");
        FBCHK(hipMemsetAsync(f->fhit, 0, 4 * (64 + (size_t)HD_FD_BUCKETS), s), "fb foreign reset");
        FBCHK(hipMemsetAsync(f->state + f->fbase, 0, 4 * (size_t)f->fres, s), "fb foreign reset");
        fb_foreign_forget(f);
    }
    rc = hd_dev_grow(ctx, (void**)&f->adm_slot, &f->cap_adm_slot, 4 * adm_slot.size());
    if (rc) return rc;
    FBCHK(hipMemcpyAsync(f->adm_slot, adm_slot.data(), 4 * adm_slot.size(), hipMemcpyHostToDevice, s), "fb adm_slot");
    FBCHK(hipStreamSynchronize(s), "fb map");
    return fb_count_not_ready(ctx);
}

int hd_fb_clear_keys(hd_ctx* ctx) {
    FbWork* f = ctx->fb;
    int rq = hd_ctx_quiesce(ctx);
    if (rq) return rq;
    if (f->nslots > 1) FBCHK(hipMemsetAsync(f->state + 1, 0, 4 * (size_t)(f->nslots - 1), ctx->stream), "fb clear");
    if (f->fres && f->fdict) {   // the foreign keys are learned again too
        FBCHK(hipMemsetAsync(f->fdict, 0, 4 * (size_t)HD_FD_WORDS, ctx->stream), "fb clear");
        FBCHK(hipMemsetAsync(f->fnext, 0, 4, ctx->stream), "fb clear");
        FBCHK(hipMemsetAsync(f->fhit, 0, 4 * (64 + (size_t)HD_FD_BUCKETS), ctx->stream), "fb clear");
    }
    FBCHK(hipStreamSynchronize(ctx->stream), "fb clear");
    if (f->fres) fb_foreign_forget(f);
    return fb_count_not_ready(ctx);
}

// the next free event pair of a profile record (created on first use), or
// NULL when profiling is off or the event could not be created
static hipEvent_t* fb_prof_pair(std::vector<hipEvent_t>& ev, size_t& used, bool on) {
    if (!on) return nullptr;
    if (2 * (used + 1) > ev.size()) {
        hipEvent_t a = nullptr, b = nullptr;
        if (hipEventCreate(&a) != hipSuccess) return nullptr;
        if (hipEventCreate(&b) != hipSuccess) {
            (void)hipEventDestroy(a);
            return nullptr;
        }
        ev.push_back(a);
        ev.push_back(b);
    }
    return &ev[2 * used++];
}

// Blocks of a grid-stride fallback kernel (k_slow_lift, k_verify over a
// list) for the latest list length seen (FbWork::est_host): 1.25x its
// blocks, at least 64 (a sudden burst of leftovers costs a few grid-stride
// rounds once), at most `full`.
static uint32_t fallback_blocks(uint32_t est, uint32_t full) {
    if (est == 0xFFFFFFFFu) return full;
    const uint64_t want = ((uint64_t)est * 5 / 4 + 255) / 256;
    return (uint32_t)std::min<uint64_t>(full, std::max<uint64_t>(want, std::min(64u, full)));
}

// k_fast_sums occupancy (HD_VAR_SUM_WAVES) and prefetch depth (HD_VAR_SUM_PREFETCH)
template <int WP>
static void launch_sums(const hd_ctx* ctx, uint32_t blocks, hipStream_t s, uint32_t n, const gp* gtab,
                        const gp* const* tab, const SplitRows& rows) {
    // 0 (the default): 4 waves per SIMD for a batch that fills fewer than two
    // rounds at 3 (C3's 128k messages: +5 %; measured 3 % slower per 1M, where
    // 3 waves keep the loaded-ahead table points)
    int w = ctx->var[HD_VAR_SUM_WAVES];
    const int pf = ctx->var[HD_VAR_SUM_PREFETCH];
    if (w == 0) w = (uint64_t)n < 2ull * 3 * 4 * 64 * (uint64_t)std::max(ctx->n_cu, 1) ? 4 : 3;
    if (pf == 2) {
        if (w == 2) k_fast_sums<2, WP, 2><<<blocks, 256, 0, s>>>(n, gtab, tab, rows);
        else k_fast_sums<3, WP, 2><<<blocks, 256, 0, s>>>(n, gtab, tab, rows);   // (no 4-wave form)
    } else {
        if (w == 2) k_fast_sums<2, WP, 1><<<blocks, 256, 0, s>>>(n, gtab, tab, rows);
        else if (w == 4) k_fast_sums<4, WP, 0><<<blocks, 256, 0, s>>>(n, gtab, tab, rows);
        else k_fast_sums<3, WP, 1><<<blocks, 256, 0, s>>>(n, gtab, tab, rows);
    }
}

template <int K, int WP>
static void launch_split(hd_ctx* ctx, const DevBatch& b, const uint8_t* d_digest, uint8_t* d_verdict,
                         uint8_t* d_rec32, int32_t* d_signer, uint32_t* d_bitmap, const SplitRows& rows,
                         const FbWork::Scratch& sc, hipStream_t s, bool auth) {
    FbWork* f = ctx->fb;
    const uint32_t n = b.n;
    // lanes of the K-per-lane kernels, a multiple of 64 (k_fast_final's bitmap words)
    const uint32_t T = ((n + (uint32_t)K - 1) / (uint32_t)K + 63u) & ~63u;
    const uint32_t tb = (T + 255) / 256, nb = (n + 255) / 256;
    k_fast_prep<<<nb, 256, 0, s>>>(b, d_digest, f->state, f->adm_slot, hd_adm_index(ctx), ctx->n_adm, rows,
                                   f->fcap ? f->fdict : nullptr, f->fhit, f->fbase);
    k_fast_sinv<K><<<tb, 256, 0, s>>>(n, T, rows);
    hipEvent_t* pe = fb_prof_pair(f->ev_sums, f->n_sums, f->prof);
    if (pe) (void)hipEventRecord(pe[0], s);
    launch_sums<WP>(ctx, nb, s, n, f->gtab, f->tabs, rows);
    if (pe) (void)hipEventRecord(pe[1], s);
    k_fast_zinv<K><<<tb, 256, 0, s>>>(n, T, rows);
    // whole blocks of 256: every wavefront's 64 messages are one bitmap word pair
    k_fast_cmp<<<nb, 256, 0, s>>>(b, rows, ctx->d_adm_perm, d_verdict, d_rec32, d_signer, sc.slow, sc.count,
                                  d_bitmap, auth);
}

static int fb_verify_impl(hd_ctx* ctx, const DevBatch& b, const uint8_t* d_digest, uint8_t* d_verdict,
                          uint8_t* d_rec32, int32_t* d_signer, uint32_t* d_bitmap, FbWork::Scratch& sc,
                          hipStream_t s, bool auth);

int hd_fb_verify(hd_ctx* ctx, const DevBatch& b, const uint8_t* d_digest, uint8_t* d_verdict, uint8_t* d_rec32,
                 int32_t* d_signer, uint32_t* d_bitmap, hipStream_t s, bool auth) {
    FbWork* f = ctx->fb;
    if (!f->done) FBCHK(hipEventCreateWithFlags(&f->done, hipEventDisableTiming), "fb event");
    const int j = f->next;
    f->next = (j + 1) % FbWork::NSCRATCH;
    FbWork::Scratch& sc = f->sc[j];
    if (!sc.done) FBCHK(hipEventCreateWithFlags(&sc.done, hipEventDisableTiming), "fb scratch event");
    if (!sc.count) FBCHK(hipMalloc(&sc.count, 8), "fb scratch count");
    // foreign slots re-keyed (fb_evict; it waited for every earlier call)
    bool evicted = false;
    int re = fb_evict(ctx, &evicted);
    if (re) return re;
    // see FbWork: in the steady state only this set's previous user orders
    // this call; otherwise the previous call does, on whatever stream
    const bool steady = !evicted && f->nr_host && *(volatile uint32_t*)f->nr_host == 0 && !fb_foreign_pending(f);
    if (sc.used && sc.stream != s) FBCHK(hipStreamWaitEvent(s, sc.done, 0), "fb scratch order");
    if (f->any && f->last != s && !(steady && f->steady)) FBCHK(hipStreamWaitEvent(s, f->done, 0), "fb stream order");
    hipEvent_t* pe = fb_prof_pair(f->ev_call, f->n_call, f->prof);
    if (pe) (void)hipEventRecord(pe[0], s);
    const int rc = fb_verify_impl(ctx, b, d_digest, d_verdict, d_rec32, d_signer, d_bitmap, sc, s, auth);
    if (pe) (void)hipEventRecord(pe[1], s);
    FBCHK(hipEventRecord(sc.done, s), "fb scratch record");
    FBCHK(hipEventRecord(f->done, s), "fb event record");
    sc.used = true;
    sc.stream = s;
    f->last_set = j;
    f->last = s;
    f->any = true;
    f->steady = steady;
    return rc;
}

// Every verify call of this context has finished (the host waits on the
// call events; other contexts and streams are not waited for).
int hd_fb_quiesce(hd_ctx* ctx) {
    FbWork* f = ctx->fb;
    if (!f) return HD_OK;
    for (auto& sc : f->sc)
        if (sc.used) FBCHK(hipEventSynchronize(sc.done), "fb quiesce");
    if (f->any) FBCHK(hipEventSynchronize(f->done), "fb quiesce");
    return HD_OK;
}

static int fb_verify_impl(hd_ctx* ctx, const DevBatch& b, const uint8_t* d_digest, uint8_t* d_verdict,
                          uint8_t* d_rec32, int32_t* d_signer, uint32_t* d_bitmap, FbWork::Scratch& sc,
                          hipStream_t s, bool auth) {
    FbWork* f = ctx->fb;
    int rc = hd_dev_grow(ctx, (void**)&sc.slow, &sc.cap_slow, 4 * (size_t)b.n);
    if (rc) return rc;
    const uint32_t blocks = (b.n + 255) / 256;
    rc = hd_dev_grow(ctx, (void**)&sc.slow2, &sc.cap_slow2, 4 * (size_t)b.n);
    if (rc) return rc;
    FBCHK(hipMemsetAsync(sc.count, 0, 8, s), "fb count reset");
    if (ctx->n_adm > 0 && f->adm_slot && f->map_ok) {
        const size_t row_words = 62;   // per message
        rc = hd_dev_grow(ctx, (void**)&sc.rows, &sc.cap_rows, 4 * row_words * (size_t)b.n);
        if (rc) return rc;
        const uint32_t n = b.n;
        SplitRows rows;
        rows.aux = sc.rows;
        rows.idx = (int32_t*)(sc.rows + (size_t)n);
        rows.u1 = sc.rows + 2 * (size_t)n;
        rows.u2 = sc.rows + 10 * (size_t)n;
        rows.s = sc.rows + 18 * (size_t)n;
        rows.pre = sc.rows + 26 * (size_t)n;
        rows.xyz = sc.rows + 35 * (size_t)n;
        rows.prio = ctx->var[HD_VAR_WAVE_PRIO];
        const int k = split_k_for(ctx, n);
        f->last_k = k;
#define HD_SPLIT(K, WP) launch_split<K, WP>(ctx, b, d_digest, d_verdict, d_rec32, d_signer, d_bitmap, rows, sc, s, auth)
        if (f->wp == HD_FB_WX) {
            if (k == 16) HD_SPLIT(16, HD_FB_WX);
            else HD_SPLIT(8, HD_FB_WX);
        } else if (f->wp == HD_FB_WW) {
            if (k == 16) HD_SPLIT(16, HD_FB_WW);
            else HD_SPLIT(8, HD_FB_WW);
        } else if (f->wp == HD_FB_WN) {
            if (k == 16) HD_SPLIT(16, HD_FB_WN);
            else HD_SPLIT(8, HD_FB_WN);
        } else {
            if (k == 16) HD_SPLIT(16, HD_FB_W);
            else HD_SPLIT(8, HD_FB_W);
        }
#undef HD_SPLIT
        FBCHK(hipGetLastError(), "split check launch");
        // k_fast_cmp wrote the valid bitmap; the slow path sets the bits of
        // its VALID messages
        const uint32_t full = std::min(blocks, (uint32_t)std::max(ctx->n_cu, 1) * 4u);
        // HD_VAR_SLOW_LIFT: the lift kernel first (its NO_POINT verdicts leave
        // the list), or k_verify over the whole leftover list (it lifts too).
        // A leftover list is usually under one wave per SIMD, so k_verify's
        // time is one recovery's latency whatever the list length, and the
        // separate lift only adds its own chain in series.
        const bool lift = ctx->var[HD_VAR_SLOW_LIFT] != 0;
        if (lift) {
            const uint32_t lift_blocks = fallback_blocks(f->est_host[0], full);
            k_slow_lift<<<lift_blocks, 256, 0, s>>>(b, sc.slow, sc.count, d_verdict, d_rec32, d_signer, sc.slow2,
                                                    sc.count + 1, ctx->var[HD_VAR_WAVE_PRIO], f->est_dev, rows,
                                                    f->gtab);
            FBCHK(hipGetLastError(), "k_slow_lift");
        }
        const SlowCtl ctl{lift ? sc.slow2 : sc.slow, lift ? sc.count + 1 : sc.count, f->adm_slot, f->state, f->pub,
                          d_bitmap, lift ? f->est_dev + 1 : f->est_dev, ctx->var[HD_VAR_WAVE_PRIO],
                          f->fcap ? f->fdict : nullptr, f->fnext, f->fbase, f->fcap, f->fpend_dev,
                          f->fcap ? f->fhit + 64 : nullptr, f->fkey, f->fpend_dev + 1};
        rc = hd_launch_slow(ctx, b, d_digest, d_verdict, d_rec32, d_signer, nullptr, ctl,
                            fallback_blocks(f->est_host[lift ? 1 : 0], full), s);
        if (rc) return rc;
        return fb_learn(ctx, s);
    }
    // no admitted set: every message takes the full recovery (it ends in
    // NOT_ADMITTED at best), nothing to learn
    const SlowCtl none{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, 0, 0, nullptr};
    return hd_launch_slow(ctx, b, d_digest, d_verdict, d_rec32, d_signer, d_bitmap, none, blocks, s);
}

extern "C" {

int hd_ctx_set_fastpath(hd_ctx* ctx, int enable) {
    if (!ctx) return HD_EINVAL;
    if (enable && !ctx->fb) {
        (void)hipSetDevice(ctx->device);
        int rc = hd_fb_init(ctx);
        if (rc) return rc;
        // map the current admitted set (sorted words -> bytes)
        if (ctx->n_adm) {
            std::vector<uint32_t> words(8 * (size_t)ctx->n_adm);
            FBCHK(hipMemcpy(words.data(), ctx->d_adm, 32 * (size_t)ctx->n_adm, hipMemcpyDeviceToHost), "adm read");
            std::vector<uint8_t> sorted(32 * (size_t)ctx->n_adm);
            for (size_t k = 0; k < words.size(); k++) store_be32(&sorted[4 * k], words[k]);
            rc = hd_fb_map_signatories(ctx, sorted.data(), ctx->n_adm);
            if (rc) return rc;
        }
    }
    ctx->fastpath = enable != 0;
    return HD_OK;
}

int hd_ctx_fastpath_geometry(hd_ctx* ctx, int* g_windows, int* key_windows, int* msgs_per_inversion) {
    if (!ctx) return HD_EINVAL;
    const int k = ctx->fb ? ctx->fb->last_k : 8;
    if (g_windows) *g_windows = FbL<HD_FB_WG>::NWIN;
    if (key_windows) *key_windows = fb_nwin(ctx->fb ? ctx->fb->wp : HD_FB_W);
    if (msgs_per_inversion) *msgs_per_inversion = k > 0 ? k : 2;
    return HD_OK;
}

int hd_ctx_profile(hd_ctx* ctx, int enable) {
    if (!ctx) return HD_EINVAL;
    if (!ctx->fb) return enable ? HD_EINVAL : HD_OK;   // the profile covers the known-key path's calls
    ctx->fb->prof = enable != 0;
    return HD_OK;
}

int hd_ctx_profile_read(hd_ctx* ctx, uint32_t* calls, double* verify_ms, uint32_t* sums_launches, double* sums_ms) {
    if (!ctx) return HD_EINVAL;
    double tc = 0, ts = 0;
    uint32_t nc = 0, ns = 0;
    if (ctx->fb) {
        FbWork* f = ctx->fb;
        (void)hipSetDevice(ctx->device);
        for (size_t k = 0; k < f->n_call; k++) {
            float ms = 0;
            FBCHK(hipEventSynchronize(f->ev_call[2 * k + 1]), "profile sync");
            FBCHK(hipEventElapsedTime(&ms, f->ev_call[2 * k], f->ev_call[2 * k + 1]), "profile read");
            tc += ms;
        }
        for (size_t k = 0; k < f->n_sums; k++) {
            float ms = 0;
            FBCHK(hipEventSynchronize(f->ev_sums[2 * k + 1]), "profile sync");
            FBCHK(hipEventElapsedTime(&ms, f->ev_sums[2 * k], f->ev_sums[2 * k + 1]), "profile read");
            ts += ms;
        }
        nc = (uint32_t)f->n_call;
        ns = (uint32_t)f->n_sums;
        f->n_call = f->n_sums = 0;
    }
    if (calls) *calls = nc;
    if (verify_ms) *verify_ms = tc;
    if (sums_launches) *sums_launches = ns;
    if (sums_ms) *sums_ms = ts;
    return HD_OK;
}

int hd_ctx_foreign_stats(hd_ctx* ctx, uint32_t* ready_slots, uint32_t* evictions, uint32_t* checks) {
    if (!ctx) return HD_EINVAL;
    if (ready_slots) *ready_slots = 0;
    if (evictions) *evictions = 0;
    if (checks) *checks = 0;
    if (!ctx->fb) return HD_OK;
    (void)hipSetDevice(ctx->device);
    FbWork* f = ctx->fb;
    int rq = hd_ctx_quiesce(ctx);
    if (rq) return rq;
    if (ready_slots && f->fres) {
        std::vector<uint32_t> st(f->fres);
        FBCHK(hipMemcpy(st.data(), f->state + f->fbase, 4 * (size_t)f->fres, hipMemcpyDeviceToHost), "state read");
        for (uint32_t v : st) *ready_slots += v == HD_FB_READY;
    }
    if (evictions) *evictions = f->evictions;
    if (checks) *checks = f->evict_checks;
    return HD_OK;
}

int hd_ctx_fastpath_stats(hd_ctx* ctx, uint32_t* known_keys, uint32_t* last_fallback) {
    if (!ctx) return HD_EINVAL;
    if (known_keys) *known_keys = 0;
    if (last_fallback) *last_fallback = 0;
    if (!ctx->fb) return HD_OK;
    (void)hipSetDevice(ctx->device);
    FbWork* f = ctx->fb;
    int rq = hd_ctx_quiesce(ctx);
    if (rq) return rq;
    if (known_keys && f->nslots > 1) {
        std::vector<uint32_t> st(f->nslots);
        FBCHK(hipMemcpy(st.data(), f->state, 4 * (size_t)f->nslots, hipMemcpyDeviceToHost), "state read");
        for (uint32_t k = 1; k < f->nslots; k++)   // admitted keys (not the foreign block)
            *known_keys += st[k] == HD_FB_READY && !(k >= f->fbase && k < f->fbase + f->fres);
    }
    if (last_fallback && f->last_set >= 0)
        FBCHK(hipMemcpy(last_fallback, f->sc[f->last_set].count, 4, hipMemcpyDeviceToHost), "fallback read");
    return HD_OK;
}

}  // extern "C"
