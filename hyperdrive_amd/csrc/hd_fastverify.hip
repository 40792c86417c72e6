// hd_fastverify.hip -- the known-key fast path of hd_verify_batch_device and
// the tables it runs on (hd_fixedbase.h).
//
// Per batch, stream-ordered, no host synchronisation:
//   k_verify_fast   one message per lane: a message whose claimed From is an
//                   admitted signatory with a known key is checked with two
//                   fixed-base multiplications (29 mixed additions, no
//                   doublings, no square root); VALID / early exact verdicts
//                   are final, everything else is appended to a list
//   k_verify        (hd_verify.hip) the full libsecp256k1-semantics recovery
//                   over that list only; VALID messages of signatories without
//                   a known key publish the recovered key to their slot
//   k_fb_bitmap     the valid bitmap from the final verdicts
//   k_fb_list / k_fb_bases / k_fb_entries / k_fb_ready
//                   build the tables of newly learned keys (HD_FB_NWIN window
//                   bases, then HD_FB_NWIN x HD_FB_N affine multiples, one per
//                   lane); with nothing learned each exits at once
// Table memory is capped by HD_FB_MAX_BYTES (default 64 GiB of the 288 GB):
// signatories beyond the cap always take the full recovery.
// G has one table with wider windows (HD_FB_WG bits: 13 additions for u1
// instead of 16), built once per device and process (fb_g_table).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/hd_verify.h"
#include "hd_fixedbase.h"
#include "hd_internal.h"
#include "hd_verify_msg.h"

using namespace hd;

struct FbWork {
    const ge* gtab = nullptr;   // the shared G table of the device (fb_g_table)
    uint32_t nslots = 0;        // allocated slots; slot 0 is unused
    uint32_t max_slots = 0;     // from HD_FB_MAX_BYTES (slot 0 included)
    ge* tab = nullptr;          // nslots x HD_FB_TAB
    ge* base = nullptr;         // nslots x HD_FB_NWIN window bases
    ge* pub = nullptr;          // nslots keys
    uint32_t* state = nullptr;  // nslots HD_FB_* states
    int32_t* adm_slot = nullptr;  // admitted sorted index -> slot
    size_t cap_adm_slot = 0;
    uint32_t* list = nullptr;     // slot work list (nslots)
    uint32_t* counts = nullptr;   // [0] slots to build, [1] messages for the slow path
    uint32_t* slow = nullptr;     // message index list
    size_t cap_slow = 0;
    std::unordered_map<std::string, uint32_t> slot_of;  // signatory -> slot
    std::vector<uint32_t> free_slots;
    uint32_t used = 1;            // slots handed out so far (slot 0 = G)
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
};

// Lane t checks messages 2t and 2t + 1 (verify_fast2: one inversion of each
// kind for the pair).
template <int WAVES>
__global__ __launch_bounds__(256, WAVES) void k_verify_fast(DevBatch b, const uint8_t* __restrict__ digest_in,
                                                     const ge* __restrict__ gtab, const ge* __restrict__ tab, const uint32_t* __restrict__ state,
                                                     const int32_t* __restrict__ adm_slot,
                                                     const uint32_t* __restrict__ adm, const int32_t* __restrict__ adm_perm,
                                                     uint32_t n_adm, int adm_steps, uint8_t* __restrict__ verdict,
                                                     uint8_t* __restrict__ rec32, int32_t* __restrict__ signer,
                                                     uint32_t* __restrict__ slow, uint32_t* __restrict__ n_slow) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    FastIn in[2];
    int32_t idx[2], slot[2];
    bool present[2], bad_type[2];
    HD_UNROLL for (int k = 0; k < 2; k++) {
        const uint32_t i = 2 * t + k;
        present[k] = i < b.n;
        bad_type[k] = false;
        idx[k] = -1;
        slot[k] = -1;
        HD_UNROLL for (int w = 0; w < 8; w++) in[k].digest_be[w] = in[k].r_be[w] = in[k].s_be[w] = 0u;
        in[k].v = 0;
        in[k].ready = false;
        if (!present[k]) continue;
        FastSrc src{b, i, digest_in};
        const uint32_t type = src.type();
        if (type < 1 || type > 3) {
            bad_type[k] = true;
            continue;
        }
        uint32_t from_be[8];
        HD_UNROLL for (int w = 0; w < 8; w++) from_be[w] = src.from(w);
        idx[k] = admitted_find(adm, n_adm, adm_steps, from_be);
        slot[k] = idx[k] >= 0 ? adm_slot[idx[k]] : -1;
        in[k].ready = slot[k] >= 0 && state[slot[k]] == HD_FB_READY;
        if (!in[k].ready) continue;
        if (digest_in) {
            HD_UNROLL for (int w = 0; w < 8; w++) in[k].digest_be[w] = load_be32(digest_in + 32 * (size_t)i + 4 * w);
        } else {
            uint32_t value_be[8];
            HD_UNROLL for (int w = 0; w < 8; w++) value_be[w] = src.value(w);
            if (type == T_PROPOSE)
                sha256_propose(in[k].digest_be, b.height[i], b.round[i], b.valid_round ? b.valid_round[i] : -1,
                               value_be);
            else
                sha256_vote(in[k].digest_be, b.height[i], b.round[i], value_be);
        }
        HD_UNROLL for (int w = 0; w < 8; w++) { in[k].r_be[w] = src.sig_r(w); in[k].s_be[w] = src.sig_s(w); }
        in[k].v = src.sig_v();
    }
    uint8_t v[2];
    __shared__ FastPark park[256];
    verify_fast2(v, in, gtab, tab + (size_t)(slot[0] > 0 ? slot[0] : 0) * HD_FB_TAB,
                 tab + (size_t)(slot[1] > 0 ? slot[1] : 0) * HD_FB_TAB, &park[threadIdx.x]);
    bool to_slow[2];
    HD_UNROLL for (int k = 0; k < 2; k++) {
        const uint32_t i = 2 * t + k;
        to_slow[k] = false;
        if (!present[k]) continue;
        if (bad_type[k]) v[k] = V_BAD_TYPE;
        if (v[k] == HD_NEEDS_SLOW) {
            to_slow[k] = true;
            continue;
        }
        // VALID: the recovered key is the signatory's, so the recovered
        // signatory is From; early verdicts recover nothing
        const bool ok = v[k] == V_VALID;
        verdict[i] = v[k];
        if (rec32) {
            uint8_t* o = rec32 + 32 * (size_t)i;
            const uint8_t* f = b.from32 + 32 * (size_t)i;
            HD_UNROLL for (int w = 0; w < 8; w++) store_be32(o + 4 * w, ok ? load_be32(f + 4 * w) : 0u);
        }
        if (signer) signer[i] = ok ? adm_perm[idx[k]] : -1;
    }
    // wave-aggregated append of the slow-path indices (order is irrelevant:
    // every message is verified on its own)
    HD_UNROLL for (int k = 0; k < 2; k++) {
        const unsigned long long bal = __ballot(to_slow[k]);
        if (bal) {
            const uint32_t lane = threadIdx.x & 63u;
            const uint32_t leader = (uint32_t)__ffsll((long long)bal) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(n_slow, (uint32_t)__popcll(bal));
            base = __shfl(base, (int)leader);
            if (to_slow[k]) slow[base + (uint32_t)__popcll(bal & ((1ull << lane) - 1))] = 2 * t + k;
        }
    }
}

__global__ void k_fb_bitmap(uint32_t n, const uint8_t* __restrict__ verdict, uint32_t* __restrict__ bitmap) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (32 * w >= n) return;
    uint32_t bits = 0;
    const uint32_t lim = min(32u, n - 32 * w);
    for (uint32_t k = 0; k < lim; k++) bits |= (uint32_t)(verdict[32 * w + k] == V_VALID) << k;
    bitmap[w] = bits;
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

template <int W>
__global__ __launch_bounds__(256) void k_fb_entries(const uint32_t* __restrict__ list,
                                                    const uint32_t* __restrict__ count, const ge* __restrict__ base,
                                                    ge* __restrict__ tab) {
    constexpr uint32_t TAB = FbL<W>::TAB;
    const uint64_t total = (uint64_t)*count * TAB;
    for (uint64_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t slot = list[t / TAB], e = (uint32_t)(t % TAB);
        int j;
        uint32_t d;
        fb_entry_pos<W>(e, j, d);
        ge o;
        fb_entry(o, base[(size_t)slot * FbL<W>::NWIN + j], d);
        tab[(size_t)slot * TAB + e] = o;
    }
}

__global__ void k_fb_ready(const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                           uint32_t* __restrict__ state) {
    for (uint32_t k = threadIdx.x; k < *count; k += blockDim.x) state[list[k]] = HD_FB_READY;
}

int fb_grow_slots(hd_ctx* ctx, uint32_t want) {
    FbWork* f = ctx->fb;
    if (want <= f->nslots) return HD_OK;
    const uint32_t n = std::min(f->max_slots, std::max(want, 2 * f->nslots));
    ge *tab = nullptr, *base = nullptr, *pub = nullptr;
    uint32_t *state = nullptr, *list = nullptr;
    FBCHK(hipMalloc(&tab, sizeof(ge) * HD_FB_TAB * (size_t)n), "fb tables");
    FBCHK(hipMalloc(&base, sizeof(ge) * HD_FB_NWIN * (size_t)n), "fb bases");
    FBCHK(hipMalloc(&pub, sizeof(ge) * (size_t)n), "fb keys");
    FBCHK(hipMalloc(&state, 4 * (size_t)n), "fb state");
    FBCHK(hipMalloc(&list, 4 * (size_t)n), "fb list");
    FBCHK(hipMemset(state, 0, 4 * (size_t)n), "fb state clear");
    if (f->nslots) {
        const size_t k = f->nslots;
        FBCHK(hipMemcpy(tab, f->tab, sizeof(ge) * HD_FB_TAB * k, hipMemcpyDeviceToDevice), "fb copy");
        FBCHK(hipMemcpy(base, f->base, sizeof(ge) * HD_FB_NWIN * k, hipMemcpyDeviceToDevice), "fb copy");
        FBCHK(hipMemcpy(pub, f->pub, sizeof(ge) * k, hipMemcpyDeviceToDevice), "fb copy");
        FBCHK(hipMemcpy(state, f->state, 4 * k, hipMemcpyDeviceToDevice), "fb copy");
        (void)hipFree(f->tab);
        (void)hipFree(f->base);
        (void)hipFree(f->pub);
        (void)hipFree(f->state);
        (void)hipFree(f->list);
    }
    f->tab = tab;
    f->base = base;
    f->pub = pub;
    f->state = state;
    f->list = list;
    f->nslots = n;
    return HD_OK;
}

// build the tables of every LEARNED slot, stream-ordered
int fb_learn(hd_ctx* ctx, hipStream_t s) {
    FbWork* f = ctx->fb;
    const uint32_t g = (uint32_t)std::max(ctx->n_cu, 1) * 4u;
    k_fb_list<<<1, 256, 0, s>>>(f->nslots, f->state, f->list, f->counts);
    k_fb_bases<HD_FB_W><<<g, 256, 0, s>>>(f->list, f->counts, f->pub, f->base);
    k_fb_entries<HD_FB_W><<<g * 2, 256, 0, s>>>(f->list, f->counts, f->base, f->tab);
    k_fb_ready<<<1, 256, 0, s>>>(f->list, f->counts, f->state);
    FBCHK(hipGetLastError(), "fb table kernels");
    return HD_OK;
}

}  // namespace

// The G table (W = HD_FB_WG) is built once per device and process and shared
// by every context on that device.
static std::mutex g_fb_g_mutex;
static std::map<int, ge*> g_fb_g_tables;

static int fb_g_table(hd_ctx* ctx, const ge** out) {
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
    ge *tab = nullptr, *base = nullptr, *pub = nullptr;
    uint32_t* cl = nullptr;  // [0] = list {0}, [1] = count 1
    FBCHK(hipMalloc(&tab, sizeof(ge) * (size_t)FbL<HD_FB_WG>::TAB), "G table");
    FBCHK(hipMalloc(&base, sizeof(ge) * FbL<HD_FB_WG>::NWIN), "G bases");
    FBCHK(hipMalloc(&pub, sizeof(ge)), "G point");
    FBCHK(hipMalloc(&cl, 8), "G list");
    const uint32_t hl[2] = {0u, 1u};
    FBCHK(hipMemcpy(pub, &g, sizeof(ge), hipMemcpyHostToDevice), "G point");
    FBCHK(hipMemcpy(cl, hl, 8, hipMemcpyHostToDevice), "G list");
    const uint32_t grid = (uint32_t)std::max(ctx->n_cu, 1) * 8u;
    k_fb_bases<HD_FB_WG><<<1, 64, 0, ctx->stream>>>(cl, cl + 1, pub, base);
    k_fb_entries<HD_FB_WG><<<grid, 256, 0, ctx->stream>>>(cl, cl + 1, base, tab);
    FBCHK(hipGetLastError(), "G table kernels");
    FBCHK(hipStreamSynchronize(ctx->stream), "G table build");
    (void)hipFree(base);
    (void)hipFree(pub);
    (void)hipFree(cl);
    g_fb_g_tables[ctx->device] = tab;
    *out = tab;
    return HD_OK;
}

int hd_fb_init(hd_ctx* ctx) {
    if (ctx->fb) return HD_OK;
    ctx->fb = new (std::nothrow) FbWork();
    if (!ctx->fb) return HD_ENOMEM;
    FbWork* f = ctx->fb;
    double budget = 64.0 * (1ull << 30);
    if (const char* m = getenv("HD_FB_MAX_BYTES")) budget = atof(m);
    const double per_slot = (double)sizeof(ge) * (HD_FB_TAB + HD_FB_NWIN + 1) + 8;
    f->max_slots = (uint32_t)std::max(1.0, std::min(1e6, budget / per_slot));
    FBCHK(hipMalloc(&f->counts, 8), "fb counts");
    int rc = fb_grow_slots(ctx, 1);
    if (rc) return rc;
    return fb_g_table(ctx, &f->gtab);
}

void hd_fb_release(hd_ctx* ctx) {
    if (!ctx || !ctx->fb) return;
    FbWork* f = ctx->fb;
    void* ptrs[] = {f->tab, f->base, f->pub, f->state, f->list, f->counts, f->slow, f->adm_slot};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    delete f;
    ctx->fb = nullptr;
}

int hd_fb_map_signatories(hd_ctx* ctx, const uint8_t* sorted, uint32_t m) {
    FbWork* f = ctx->fb;
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
    int rc = fb_grow_slots(ctx, f->used);
    if (rc) return rc;
    for (uint32_t slot : fresh) FBCHK(hipMemset(f->state + slot, 0, 4), "fb slot reset");
    rc = hd_dev_grow(ctx, (void**)&f->adm_slot, &f->cap_adm_slot, 4 * adm_slot.size());
    if (rc) return rc;
    FBCHK(hipMemcpy(f->adm_slot, adm_slot.data(), 4 * adm_slot.size(), hipMemcpyHostToDevice), "fb adm_slot");
    return HD_OK;
}

int hd_fb_clear_keys(hd_ctx* ctx) {
    FbWork* f = ctx->fb;
    FBCHK(hipDeviceSynchronize(), "fb clear sync");
    if (f->nslots > 1) FBCHK(hipMemset(f->state + 1, 0, 4 * (size_t)(f->nslots - 1)), "fb clear");
    return HD_OK;
}

int hd_fb_verify(hd_ctx* ctx, const DevBatch& b, const uint8_t* d_digest, uint8_t* d_verdict, uint8_t* d_rec32,
                 int32_t* d_signer, uint32_t* d_bitmap, hipStream_t s) {
    FbWork* f = ctx->fb;
    int rc = hd_dev_grow(ctx, (void**)&f->slow, &f->cap_slow, 4 * (size_t)b.n);
    if (rc) return rc;
    const uint32_t blocks = (b.n + 255) / 256;
    const uint32_t fast_blocks = ((b.n + 1) / 2 + 255) / 256;   // two messages per lane
    FBCHK(hipMemsetAsync(f->counts + 1, 0, 4, s), "fb count reset");
    if (ctx->n_adm > 0 && f->adm_slot) {
        static const int fw = getenv("HD_FAST_WAVES") ? atoi(getenv("HD_FAST_WAVES")) : 2;
#define HD_LAUNCH_FAST(W)                                                                                        \
    k_verify_fast<W><<<fast_blocks, 256, 0, s>>>(b, d_digest, f->gtab, f->tab, f->state, f->adm_slot, ctx->d_adm, ctx->d_adm_perm, \
                                            ctx->n_adm, ctx->adm_steps, d_verdict, d_rec32, d_signer, f->slow,       \
                                            f->counts + 1)
        if (fw == 2) HD_LAUNCH_FAST(2);
        else if (fw == 4) HD_LAUNCH_FAST(4);
        else if (fw == 5) HD_LAUNCH_FAST(5);
        else HD_LAUNCH_FAST(3);
#undef HD_LAUNCH_FAST
        FBCHK(hipGetLastError(), "k_verify_fast launch");
        // the fallback list is usually short (its length is only known on the
        // device): a grid of 4 blocks per CU walks it, instead of one block
        // per 256 messages that would mostly start and exit
        const SlowCtl ctl{f->slow, f->counts + 1, f->adm_slot, f->state, f->pub};
        const uint32_t slow_blocks = std::min(blocks, (uint32_t)std::max(ctx->n_cu, 1) * 4u);
        rc = hd_launch_slow(ctx, b, d_digest, d_verdict, d_rec32, d_signer, nullptr, ctl, slow_blocks, s);
        if (rc) return rc;
        if (d_bitmap) {
            k_fb_bitmap<<<((b.n + 31) / 32 + 255) / 256, 256, 0, s>>>(b.n, d_verdict, d_bitmap);
            FBCHK(hipGetLastError(), "k_fb_bitmap launch");
        }
        return fb_learn(ctx, s);
    }
    // no admitted set: every message takes the full recovery (it ends in
    // NOT_ADMITTED at best), nothing to learn
    const SlowCtl none{nullptr, nullptr, nullptr, nullptr, nullptr};
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

int hd_ctx_fastpath_stats(hd_ctx* ctx, uint32_t* known_keys, uint32_t* last_fallback) {
    if (!ctx) return HD_EINVAL;
    if (known_keys) *known_keys = 0;
    if (last_fallback) *last_fallback = 0;
    if (!ctx->fb) return HD_OK;
    (void)hipSetDevice(ctx->device);
    FbWork* f = ctx->fb;
    FBCHK(hipDeviceSynchronize(), "fastpath stats sync");
    if (known_keys && f->nslots > 1) {
        std::vector<uint32_t> st(f->nslots);
        FBCHK(hipMemcpy(st.data(), f->state, 4 * (size_t)f->nslots, hipMemcpyDeviceToHost), "state read");
        for (uint32_t k = 1; k < f->nslots; k++) *known_keys += st[k] == HD_FB_READY;
    }
    if (last_fallback) FBCHK(hipMemcpy(last_fallback, f->counts + 1, 4, hipMemcpyDeviceToHost), "fallback read");
    return HD_OK;
}

}  // extern "C"
