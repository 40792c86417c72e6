// hd_verify.hip -- gfx950 kernels and the C ABI (include/hd_verify.h) of the
// hyperdrive batch authenticator.
//
// Kernels
//   k_verify  one message per lane: digest -> secp256k1 recover -> signatory
//             -> Equal(From) -> admitted lookup.  INT32-VALU bound (no MFMA:
//             nothing here is a dense contraction).  The tables of
//             1G..2048G and lambda times those (288 KiB) are read
//             through the L2 by the 12-bit G windows; the admitted set
//             (sorted, 32 B entries) is read through L2.  A valid-bitmap word
//             pair per wavefront comes from one __ballot.
//   (k_gen / k_keys, the synthetic workload, live in hd_genk.hip)
//   tally kernels: see hd_tally.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hd_digest.h"
#include "../../include/hd_verify.h"
#include "hd_fixedbase.h"
#include "hd_verify_msg.h"
#include "hd_internal.h"

using namespace hd;

// ---------------------------------------------------------------- kernels
// Message i of a device batch, loaded field by field when the hot path needs
// it (see verify_msg_src).
struct DevSrc {
    const DevBatch& b;
    uint32_t i;
    const uint8_t* dg;  // caller-supplied digests (hd_verify_batch_digest_device) or NULL
    __device__ __forceinline__ uint32_t type() const { return b.type[i]; }
    __device__ __forceinline__ int64_t h() const { return b.height[i]; }
    __device__ __forceinline__ int64_t r() const { return b.round[i]; }
    __device__ __forceinline__ int64_t vr() const { return b.valid_round ? b.valid_round[i] : -1; }
    __device__ __forceinline__ uint32_t value(int w) const { return load_be32(b.value32 + 32 * (size_t)i + 4 * w); }
    __device__ __forceinline__ uint32_t from(int w) const { return load_be32(b.from32 + 32 * (size_t)i + 4 * w); }
    __device__ __forceinline__ uint32_t sig_r(int w) const { return load_be32(b.sig65 + 65 * (size_t)i + 4 * w); }
    __device__ __forceinline__ uint32_t sig_s(int w) const { return load_be32(b.sig65 + 65 * (size_t)i + 32 + 4 * w); }
    __device__ __forceinline__ uint32_t sig_v() const { return b.sig65[65 * (size_t)i + 64]; }
    __device__ __forceinline__ bool has_digest() const { return dg != nullptr; }
    __device__ __forceinline__ uint32_t digest(int w) const { return load_be32(dg + 32 * (size_t)i + 4 * w); }
};

// A NOT_ADMITTED recovery's key into the foreign-key dictionary (once per
// From; a bucket another lane is writing is left alone -- learning is only an
// optimisation) and, while reserved slots last, into its own table slot.  A
// From without a slot keeps its key in its bucket (fkey) and counts each
// further recovery (fbhit, and the host-mapped fmiss flag), so that the host
// can later hand it the slot of a colder key (fb_evict).
__device__ void fdict_learn(const SlowCtl& ctl, const uint32_t from_be[8], const ge& q) {
    uint32_t* fd = ctl.fdict;
    uint32_t b = fdict_bucket(from_be);
    for (int p = 0; p < 8; p++, b = (b + 1u) & (HD_FD_BUCKETS - 1u)) {
        const uint32_t c = atomicCAS(&fd[b], 0u, 1u);
        if (c == 0u) {
            const uint32_t j = atomicAdd(ctl.fnext, 1u);
            uint32_t slot = 0xFFFFFFFFu;
            if (j < ctl.fcap) {
                slot = ctl.fbase + j;
                ctl.fb_pub[slot] = q;
                __threadfence();
                atomicExch(&ctl.fb_state[slot], HD_FB_LEARNED);
            } else if (ctl.fkey) {
                ctl.fkey[b] = q;
            }
            HD_UNROLL for (int w = 0; w < 8; w++) fd[2u * HD_FD_BUCKETS + 8u * b + w] = from_be[w];
            fd[HD_FD_BUCKETS + b] = slot;
            __threadfence();
            atomicExch(&fd[b], 2u);
            if (slot != 0xFFFFFFFFu)
                __hip_atomic_store(ctl.fpend, j + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        if (c != 2u) return;
        // the bucket may have been written by a lane of this launch on another
        // XCD: read it with read-modify-write atomics, performed where the
        // writer's release made it visible (a plain load may hit this XCD's
        // L2 line from before the write -- the From would not match, claim a
        // second bucket and a second slot).  Rare: the full recovery's leftovers.
        uint32_t diff = 0;
        HD_UNROLL for (int w = 0; w < 8; w++) diff |= atomicAdd(&fd[2u * HD_FD_BUCKETS + 8u * b + w], 0u) ^ from_be[w];
        if (!diff) {
            const uint32_t sl = atomicAdd(&fd[HD_FD_BUCKETS + b], 0u);
            if (ctl.fbhit && sl == 0xFFFFFFFFu) {   // known, without a slot
                atomicAdd(&ctl.fbhit[b], 1u);
                __hip_atomic_store(ctl.fmiss, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            return;
        }
    }
}

// With ctl.list, lane p verifies message ctl.list[p] for p < *ctl.count (the
// known-key fast path's leftovers); with ctl.adm_slot, a VALID message whose
// signatory has no known key yet publishes its recovered key to the
// signatory's table slot (first writer wins, hd_fixedbase.h states).
template <int PKFMT, int WAVES>
__global__ __launch_bounds__(256, WAVES) void k_verify(DevBatch b, const ge* __restrict__ gtab_g,
                                                const uint32_t* __restrict__ adm, const int32_t* __restrict__ adm_perm,
                                                uint32_t n_adm, int adm_steps, uint8_t* __restrict__ verdict,
                                                uint8_t* __restrict__ rec32, int32_t* __restrict__ signer,
                                                uint32_t* __restrict__ bitmap, const uint8_t* __restrict__ digest_in,
                                                SlowCtl ctl, const gp* __restrict__ fbg) {
    // s_setprio takes an immediate: a uniform branch per level
    if (ctl.prio == 1) __builtin_amdgcn_s_setprio(1);
    else if (ctl.prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (ctl.prio >= 3) __builtin_amdgcn_s_setprio(3);
    const uint32_t stride = gridDim.x * blockDim.x;
    const uint32_t total = ctl.list ? *ctl.count : b.n;
    if (ctl.est_out && blockIdx.x == 0 && threadIdx.x == 0) ctl.est_out[0] = total;
    for (uint32_t base = blockIdx.x * blockDim.x; base < total; base += stride) {
        const uint32_t p = base + threadIdx.x;
        const bool active = p < total;
        uint8_t v = 0xFF;
        if (active) {
            const uint32_t i = ctl.list ? ctl.list[p] : p;
            DevSrc src{b, i, digest_in};
            uint32_t rec[8];
            int32_t s;
            ge q;
            v = verify_msg_src(src, gtab_g, adm, n_adm, adm_steps, PKFMT, rec, s, ctl.adm_slot ? &q : nullptr, fbg);
            verdict[i] = v;
            if (rec32) {
                uint8_t* o = rec32 + 32 * (size_t)i;
                HD_UNROLL for (int w = 0; w < 8; w++) store_be32(o + 4 * w, rec[w]);
            }
            if (signer) signer[i] = s >= 0 ? adm_perm[s] : -1;
            if (ctl.bitmap_or && v == V_VALID) atomicOr(&ctl.bitmap_or[i >> 5], 1u << (i & 31));
            if (ctl.fdict && v == V_NOT_ADMITTED) {
                uint32_t from_be[8];
                HD_UNROLL for (int w = 0; w < 8; w++) from_be[w] = src.from(w);
                fdict_learn(ctl, from_be, q);
            }
            if (ctl.adm_slot && v == V_VALID) {
                const int32_t slot = ctl.adm_slot[s];
                if (slot >= 0 && ctl.fb_state[slot] == HD_FB_EMPTY &&
                    atomicCAS(&ctl.fb_state[slot], HD_FB_EMPTY, HD_FB_CLAIMED) == HD_FB_EMPTY) {
                    ctl.fb_pub[slot] = q;
                    __threadfence();
                    atomicExch(&ctl.fb_state[slot], HD_FB_LEARNED);
                }
            }
        }
        if (bitmap) {
            const unsigned long long bal = __ballot(active && v == V_VALID);
            const uint32_t wave_base = base + (threadIdx.x & ~63u);
            if ((threadIdx.x & 63u) == 0 && wave_base < b.n) {
                bitmap[wave_base / 32] = (uint32_t)bal;
                if (wave_base + 32 < b.n) bitmap[wave_base / 32 + 1] = (uint32_t)(bal >> 32);
            }
        }
    }
}

// ---------------------------------------------------------------- host side
namespace {
const char* const kErr[] = {"ok", "invalid argument", "out of memory", "device error", "tally capacity too small",
                            "more tally groups than staged (run the synchronous tally)"};
}

int hd_ctx_fail(hd_ctx* ctx, hipError_t e, const char* what) {
    if (ctx) {
        char buf[256];
        snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
        ctx->last_error = buf;
    }
    return e == hipErrorOutOfMemory ? HD_ENOMEM : HD_EDEVICE;
}

int hd_ctx_note_stream(hd_ctx* ctx, hipStream_t s) {
    if (!s || s == ctx->stream) return HD_OK;
    hipEvent_t ev = nullptr;
    for (auto& se : ctx->caller_ev)
        if (se.first == s) ev = se.second;
    if (!ev) {
        // a new caller stream: first forget the streams whose last recorded
        // work has completed (destroy has nothing to wait for there), so a
        // caller making a stream per call does not grow the list.  The event
        // is re-recorded on the handle's current stream at every call, so a
        // reused handle is ordered correctly either way.
        auto& L = ctx->caller_ev;
        for (size_t k = 0; k < L.size();) {
            if (hipEventQuery(L[k].second) == hipSuccess) {
                (void)hipEventDestroy(L[k].second);
                L[k] = L.back();
                L.pop_back();
            } else {
                k++;
            }
        }
        hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) return hd_ctx_fail(ctx, e, "caller stream event");
        ctx->caller_ev.emplace_back(s, ev);
    }
    hipError_t e = hipEventRecord(ev, s);
    return e == hipSuccess ? HD_OK : hd_ctx_fail(ctx, e, "caller stream event record");
}

int hd_dev_grow(hd_ctx* ctx, void** p, size_t* cap, size_t need) {
    if (need <= *cap) return HD_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    // 1/8 slack: batches of nearly the same size (the two halves of a wire
    // push, a partition's candidates) then share a buffer.  A regrow frees the
    // old buffer, and hipFree waits for the whole device: in the ingress push
    // it serialised the two concurrent verify calls until every scratch set
    // had seen the larger half (profiles/round5: 0.23 ms host gap per push).
    size_t want = std::max(need + need / 8, (size_t)4096);
    hipError_t e = hipMalloc(p, want);
    if (e != hipSuccess) return hd_ctx_fail(ctx, e, "hipMalloc");
    *cap = want;
    return HD_OK;
}

extern "C" {

int hd_abi_version(void) { return 2; }

const char* hd_strerror(int code) {
    int k = -code;
    if (k < 0 || k > 5) return "unknown error";
    return kErr[k];
}

const char* hd_ctx_last_error(hd_ctx* ctx) { return ctx ? ctx->last_error.c_str() : ""; }

int hd_ctx_create(int device, hd_ctx** out) {
    if (!out) return HD_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return HD_EDEVICE;
    hd_ctx* ctx = new (std::nothrow) hd_ctx();
    if (!ctx) return HD_ENOMEM;
    ctx->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        int rc = hd_ctx_fail(ctx, e, "hipStreamCreate");
        delete ctx;
        return rc;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) ctx->n_cu = prop.multiProcessorCount;
    // variant defaults from the environment (hd_ctx_set_variant)
    struct { int key; const char* env; } envs[] = {
        {HD_VAR_VERIFY_WAVES, "HD_VERIFY_WAVES"}, {HD_VAR_SUM_WAVES, "HD_SUM_WAVES"},
        {HD_VAR_SUM_PREFETCH, "HD_SUM_PF"},       {HD_VAR_SPLIT_K, "HD_FAST_K"},
        {HD_VAR_KEY_WIDTH, "HD_FB_PW"},           {HD_VAR_WAVE_PRIO, "HD_WAVE_PRIO"},
        {HD_VAR_FOREIGN_KEYS, "HD_FOREIGN_KEYS"}, {HD_VAR_SLOW_LIFT, "HD_SLOW_LIFT"},
    };
    for (auto& ev : envs)
        if (const char* e = getenv(ev.env)) (void)hd_ctx_set_variant(ctx, ev.key, atoi(e));
    if (getenv("HD_RECOVER_GLV_G")) (void)hd_ctx_set_variant(ctx, HD_VAR_RECOVER_G, 1);
    if (const char* f = getenv("HD_VERIFY_FASTPATH")) ctx->fastpath = atoi(f) != 0;
    // G tables (1G..2048G and lambda*(1G..2048G), affine), built once on the
    // host with the same code the device runs, then uploaded.
    static std::once_flag once;
    static std::vector<ge> host_tab(2 * HD_GLV_GTAB_N);
    std::call_once(once, [] { build_gtab_glv(host_tab.data()); });
    e = hipMalloc(&ctx->d_gtab, sizeof(ge) * 2 * HD_GLV_GTAB_N);
    if (e == hipSuccess)
        e = hipMemcpy(ctx->d_gtab, host_tab.data(), sizeof(ge) * 2 * HD_GLV_GTAB_N, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        int rc = hd_ctx_fail(ctx, e, "gtab upload");
        hd_ctx_destroy(ctx);
        return rc;
    }
    if (ctx->fastpath) {
        const int rc = hd_fb_init(ctx);
        if (rc) {
            hd_ctx_destroy(ctx);
            return rc;
        }
    }
    *out = ctx;
    return HD_OK;
}

int hd_ctx_destroy(hd_ctx* ctx) {
    if (!ctx) return HD_EINVAL;
    (void)hipSetDevice(ctx->device);
    (void)hd_ctx_quiesce(ctx);
    // work the caller queued on its own streams may still read or write this
    // context's scratch (a route's k_route_write, an async tally): nothing is
    // freed before the last such work of every stream has finished (other
    // contexts' and streams' work is not waited for)
    for (auto& se : ctx->caller_ev) {
        (void)hipEventSynchronize(se.second);
        (void)hipEventDestroy(se.second);
    }
    ctx->caller_ev.clear();
    if (ctx->ev_slow) (void)hipEventDestroy(ctx->ev_slow);
    void* ptrs[] = {ctx->d_gtab, ctx->d_adm, ctx->d_adm_perm, ctx->d_sig_caller, ctx->d_adm_ix};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (auto& b : ctx->bufs)
        if (b.p) (void)hipFree(b.p);
    hd_host_release(ctx);
    hd_tally_release(ctx);
    hd_fb_release(ctx);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return HD_OK;
}

int hd_ctx_set_variant(hd_ctx* ctx, int which, int value) {
    if (!ctx || which < 0 || which >= HD_VAR__COUNT) return HD_EINVAL;
    bool ok = false;
    switch (which) {
        case HD_VAR_VERIFY_WAVES: ok = value >= 2 && value <= 4; break;
        case HD_VAR_SUM_WAVES: ok = value == 0 || (value >= 2 && value <= 4); break;
        case HD_VAR_SUM_PREFETCH: ok = value == 1 || value == 2; break;
        case HD_VAR_RECOVER_G: case HD_VAR_SLOW_LIFT: ok = value == 0 || value == 1; break;
        case HD_VAR_SPLIT_K: ok = value == -1 || value == 8 || value == 16; break;
        case HD_VAR_KEY_WIDTH:
            ok = value == 0 || value == HD_FB_W || value == HD_FB_WW || value == HD_FB_WN || value == HD_FB_WX;
            break;
        case HD_VAR_WAVE_PRIO: ok = value >= 0 && value <= 3; break;
        case HD_VAR_FOREIGN_KEYS: ok = value >= 0 && value <= 64; break;
        default: ok = false;   // a key of a variant removed in round 5 (measured without gain)
    }
    if (!ok) return HD_EINVAL;
    ctx->var[which] = value;
    if (which == HD_VAR_VERIFY_WAVES) ctx->verify_waves = value;
    return HD_OK;
}

int hd_ctx_get_variant(hd_ctx* ctx, int which, int* value) {
    if (!ctx || !value || which < 0 || which >= HD_VAR__COUNT) return HD_EINVAL;
    *value = ctx->var[which];
    return HD_OK;
}

int hd_ctx_set_pubkey_format(hd_ctx* ctx, int format) {
    if (!ctx || format < HD_PUBKEY_UNCOMPRESSED || format > HD_PUBKEY_XY_STRIPPED) return HD_EINVAL;
    if (format != ctx->pkfmt) {
        ctx->pkfmt = format;
        // keys were learned under the other signatory derivation
        if (ctx->fb) return hd_fb_clear_keys(ctx);
    }
    return HD_OK;
}

int hd_set_signatories(hd_ctx* ctx, const uint8_t* sigs32, uint32_t n) {
    if (!ctx || (n && !sigs32)) return HD_EINVAL;
    (void)hipSetDevice(ctx->device);
    // kernels of earlier calls of this context (any stream) may still read
    // the admitted tables
    int rq = hd_ctx_quiesce(ctx);
    if (rq) return rq;
    // sort (stable on the original index so duplicates map to the first)
    std::vector<uint32_t> order(n);
    for (uint32_t i = 0; i < n; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(),
                     [&](uint32_t a, uint32_t b) { return memcmp(sigs32 + 32 * (size_t)a, sigs32 + 32 * (size_t)b, 32) < 0; });
    std::vector<uint32_t> words;
    std::vector<int32_t> perm;
    words.reserve(8 * (size_t)n);
    for (uint32_t k = 0; k < n; k++) {
        const uint8_t* s = sigs32 + 32 * (size_t)order[k];
        if (!perm.empty() && memcmp(s, sigs32 + 32 * (size_t)perm.back(), 32) == 0) continue;  // dedup
        for (int w = 0; w < 8; w++) words.push_back(load_be32(s + 4 * w));
        perm.push_back((int32_t)order[k]);
    }
    uint32_t m = (uint32_t)perm.size();
    const uint32_t ix_slots = adm_index_slots(m);
    std::vector<uint32_t> ix(ix_slots);
    adm_index_build(words.data(), m, ix.data(), ix_slots);
    size_t cap_a = ctx->cap_adm, cap_p = ctx->cap_adm_perm;
    int rc = hd_dev_grow(ctx, (void**)&ctx->d_adm, &cap_a, 32 * (size_t)std::max(m, 1u));
    if (rc) return rc;
    ctx->cap_adm = cap_a;
    rc = hd_dev_grow(ctx, (void**)&ctx->d_adm_perm, &cap_p, 4 * (size_t)std::max(m, 1u));
    if (rc) return rc;
    ctx->cap_adm_perm = cap_p;
    rc = hd_dev_grow(ctx, (void**)&ctx->d_adm_ix, &ctx->cap_adm_ix, 4 * (size_t)ix_slots);
    if (rc) return rc;
    rc = hd_dev_grow(ctx, (void**)&ctx->d_sig_caller, &ctx->cap_sig_caller, 32 * (size_t)std::max(n, 1u));
    if (rc) return rc;
    hipError_t e = hipSuccess;
    if (m) {
        e = hipMemcpyAsync(ctx->d_adm, words.data(), 32 * (size_t)m, hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(ctx->d_adm_perm, perm.data(), 4 * (size_t)m, hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(ctx->d_sig_caller, sigs32, 32 * (size_t)n, hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(ctx->d_adm_ix, ix.data(), 4 * (size_t)ix_slots, hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    }
    if (e != hipSuccess) return hd_ctx_fail(ctx, e, "set_signatories upload");
    ctx->n_adm = m;
    ctx->adm_ver++;
    ctx->adm_ix_mask = ix_slots - 1;
    ctx->n_sig_caller = n;
    int steps = 0;
    while ((1u << steps) < m) steps++;
    ctx->adm_steps = steps;
    if (ctx->fb) {
        std::vector<uint8_t> sorted(32 * (size_t)m);
        for (uint32_t k = 0; k < m; k++) memcpy(&sorted[32 * (size_t)k], sigs32 + 32 * (size_t)perm[k], 32);
        return hd_fb_map_signatories(ctx, sorted.data(), m);
    }
    return HD_OK;
}

}  // extern "C"

int hd_launch_slow(hd_ctx* ctx, const DevBatch& b, const uint8_t* d_digest, uint8_t* d_verdict, uint8_t* d_rec32,
                   int32_t* d_signer, uint32_t* d_bitmap, const SlowCtl& ctl, uint32_t blocks, hipStream_t s) {
#define HD_LAUNCH_VERIFY(C, W)                                                                                    \
    k_verify<C, W><<<blocks, 256, 0, s>>>(b, ctx->d_gtab, ctx->d_adm, ctx->d_adm_perm, ctx->n_adm, ctx->adm_steps, \
                                          d_verdict, d_rec32, d_signer, d_bitmap, d_digest, ctl, fbg)
    // waves/SIMD the kernel is register-allocated for (HD_VAR_VERIFY_WAVES 2 / 3 / 4,
    // default 3; the other pubkey formats are compiled for 3 only)
    const int w = ctx->verify_waves;
    // the fixed-base G table, when the context has one (HD_VAR_RECOVER_G 0)
    const gp* fbg = ctx->var[HD_VAR_RECOVER_G] ? nullptr : hd_fb_gtab(ctx);
    if (ctx->pkfmt == HD_PUBKEY_COMPRESSED) {
        if (w == 2) HD_LAUNCH_VERIFY(1, 2);
        else if (w == 4) HD_LAUNCH_VERIFY(1, 4);
        else HD_LAUNCH_VERIFY(1, 3);
    } else if (ctx->pkfmt == HD_PUBKEY_RAW64) {
        HD_LAUNCH_VERIFY(2, 3);
    } else if (ctx->pkfmt == HD_PUBKEY_XY_STRIPPED) {
        HD_LAUNCH_VERIFY(3, 3);
    } else {
        HD_LAUNCH_VERIFY(0, 3);
    }
#undef HD_LAUNCH_VERIFY
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hd_ctx_fail(ctx, e, "k_verify launch");
    return HD_OK;
}

namespace {
int launch_verify(hd_ctx* ctx, const hd_batch* db, const uint8_t* d_digest, uint8_t* d_verdict, uint8_t* d_recovered32,
                  int32_t* d_signer, uint32_t* d_valid_bitmap, void* stream, bool auth = false) {
    (void)hipSetDevice(ctx->device);
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    DevBatch b{db->n, db->type, db->height, db->round, db->valid_round, db->value32, db->from32, db->sig65};
    if (ctx->fastpath && ctx->fb)
        return hd_fb_verify(ctx, b, d_digest, d_verdict, d_recovered32, d_signer, d_valid_bitmap, s, auth);
    // one block per 256 messages, no grid-stride: the dispatcher hands a CU a
    // new block whenever one retires, which balances the last round better
    // than a resident-sized grid looping over the batch (measured on 1M:
    // 13.2 ms vs 13.5 ms at 2x resident blocks, 14.3 ms at 1x)
    const uint32_t blocks = (db->n + 255) / 256;
    const SlowCtl none{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, 0, 0, nullptr};
    const int rc = hd_launch_slow(ctx, b, d_digest, d_verdict, d_recovered32, d_signer, d_valid_bitmap, none, blocks, s);
    if (rc) return rc;
    hipError_t e = ctx->ev_slow ? hipSuccess : hipEventCreateWithFlags(&ctx->ev_slow, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ctx->ev_slow, s);
    return e == hipSuccess ? HD_OK : hd_ctx_fail(ctx, e, "verify event");
}
}  // namespace

int hd_ctx_quiesce(hd_ctx* ctx) {
    hipError_t e = ctx->stream ? hipStreamSynchronize(ctx->stream) : hipSuccess;
    if (e == hipSuccess && ctx->ev_slow) e = hipEventSynchronize(ctx->ev_slow);
    if (e != hipSuccess) return hd_ctx_fail(ctx, e, "quiesce");
    return ctx->fb ? hd_fb_quiesce(ctx) : HD_OK;
}

extern "C" {

int hd_verify_batch_device(hd_ctx* ctx, const hd_batch* db, uint8_t* d_verdict, uint8_t* d_recovered32,
                           int32_t* d_signer, uint32_t* d_valid_bitmap, void* stream) {
    if (!ctx || !db) return HD_EINVAL;
    if (db->n == 0) return HD_OK;  // empty device tensors may have NULL data pointers
    if (!d_verdict) return HD_EINVAL;
    if (!db->type || !db->height || !db->round || !db->value32 || !db->from32 || !db->sig65) return HD_EINVAL;
    return launch_verify(ctx, db, nullptr, d_verdict, d_recovered32, d_signer, d_valid_bitmap, stream);
}

int hd_authenticate_batch_device(hd_ctx* ctx, const hd_batch* db, uint8_t* d_verdict, void* stream) {
    if (!ctx || !db) return HD_EINVAL;
    if (db->n == 0) return HD_OK;
    if (!d_verdict) return HD_EINVAL;
    if (!db->type || !db->height || !db->round || !db->value32 || !db->from32 || !db->sig65) return HD_EINVAL;
    return launch_verify(ctx, db, nullptr, d_verdict, nullptr, nullptr, nullptr, stream, true);
}

int hd_verify_batch_digest_device(hd_ctx* ctx, const hd_batch* db, const uint8_t* d_digest32, uint8_t* d_verdict,
                                  uint8_t* d_recovered32, int32_t* d_signer, uint32_t* d_valid_bitmap, void* stream) {
    if (!ctx || !db) return HD_EINVAL;
    if (db->n == 0) return HD_OK;
    if (!d_verdict || !d_digest32) return HD_EINVAL;
    if (!db->type || !db->from32 || !db->sig65) return HD_EINVAL;
    return launch_verify(ctx, db, d_digest32, d_verdict, d_recovered32, d_signer, d_valid_bitmap, stream);
}

}  // extern "C"

int hd_upload_batch(hd_ctx* ctx, const hd_batch* hb, hd_batch* db) {
    const uint32_t n = hb->n;
    struct F { const void* src; size_t sz; int slot; } f[] = {
        {hb->type, (size_t)n, BUF_TYPE},
        {hb->height, 8 * (size_t)n, BUF_HEIGHT},
        {hb->round, 8 * (size_t)n, BUF_ROUND},
        {hb->valid_round, 8 * (size_t)n, BUF_VROUND},
        {hb->value32, 32 * (size_t)n, BUF_VALUE},
        {hb->from32, 32 * (size_t)n, BUF_FROM},
        {hb->sig65, 65 * (size_t)n, BUF_SIG},
    };
    void* dst[7];
    for (int k = 0; k < 7; k++) {
        if (!f[k].src) { dst[k] = nullptr; continue; }
        int rc = hd_dev_grow(ctx, &ctx->bufs[f[k].slot].p, &ctx->bufs[f[k].slot].cap, f[k].sz);
        if (rc) return rc;
        dst[k] = ctx->bufs[f[k].slot].p;
        hipError_t e = hipMemcpyAsync(dst[k], f[k].src, f[k].sz, hipMemcpyHostToDevice, ctx->stream);
        if (e != hipSuccess) return hd_ctx_fail(ctx, e, "batch upload");
    }
    db->n = n;
    db->type = (const uint8_t*)dst[0];
    db->height = (const int64_t*)dst[1];
    db->round = (const int64_t*)dst[2];
    db->valid_round = (const int64_t*)dst[3];
    db->value32 = (const uint8_t*)dst[4];
    db->from32 = (const uint8_t*)dst[5];
    db->sig65 = (const uint8_t*)dst[6];
    return HD_OK;
}

int hd_verify_uploaded(hd_ctx* ctx, const hd_batch* db, uint8_t* verdict, uint8_t* recovered32, uint32_t* valid_bitmap) {
    const uint32_t n = db->n;
    int rc = hd_dev_grow(ctx, &ctx->bufs[BUF_VERDICT].p, &ctx->bufs[BUF_VERDICT].cap, n);
    if (!rc) rc = hd_dev_grow(ctx, &ctx->bufs[BUF_SIGNER].p, &ctx->bufs[BUF_SIGNER].cap, 4 * (size_t)n);
    if (!rc && recovered32) rc = hd_dev_grow(ctx, &ctx->bufs[BUF_REC].p, &ctx->bufs[BUF_REC].cap, 32 * (size_t)n);
    size_t nwords = (n + 31) / 32;
    if (!rc && valid_bitmap) rc = hd_dev_grow(ctx, &ctx->bufs[BUF_BITMAP].p, &ctx->bufs[BUF_BITMAP].cap, 4 * nwords);
    if (rc) return rc;
    uint8_t* d_v = (uint8_t*)ctx->bufs[BUF_VERDICT].p;
    uint8_t* d_r = recovered32 ? (uint8_t*)ctx->bufs[BUF_REC].p : nullptr;
    uint32_t* d_b = valid_bitmap ? (uint32_t*)ctx->bufs[BUF_BITMAP].p : nullptr;
    int32_t* d_s = (int32_t*)ctx->bufs[BUF_SIGNER].p;
    rc = hd_verify_batch_device(ctx, db, d_v, d_r, d_s, d_b, ctx->stream);
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(verdict, d_v, n, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && d_r) e = hipMemcpyAsync(recovered32, d_r, 32 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess && d_b) e = hipMemcpyAsync(valid_bitmap, d_b, 4 * nwords, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hd_ctx_fail(ctx, e, "verify");
    return HD_OK;
}

extern "C" {

int hd_verify_batch(hd_ctx* ctx, const hd_batch* batch, uint8_t* verdict, uint8_t* recovered32, uint32_t* valid_bitmap) {
    if (!ctx || !batch || !verdict) return HD_EINVAL;
    if (batch->n == 0) return HD_OK;
    if (!batch->type || !batch->height || !batch->round || !batch->value32 || !batch->from32 || !batch->sig65)
        return HD_EINVAL;
    (void)hipSetDevice(ctx->device);
    hd_batch db;
    int rc = hd_upload_batch(ctx, batch, &db);
    if (rc) return rc;
    return hd_verify_uploaded(ctx, &db, verdict, recovered32, valid_bitmap);
}

}  // extern "C"
