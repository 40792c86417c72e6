// hd_tally.hip -- GPU tally of authenticated votes: the first-wins vote logs
// of process/process.go:823-892 and the counts the 2f+1 / f+1 rules read
// (process.go:486-494, 534, 574-582, 626-632, 658, 696-702, 751), for every
// (height, round) in a batch at once.
//
// Candidates are VALID Prevotes / Precommits.  The tally is three group-bys,
// done with open-addressing hash tables in HBM rather than sorts (a sort of
// 1M 64-bit keys is ~0.2 ms per radix pass; a probe is a few L2 accesses):
//
//   G  (h, r)                 one slot per round: distinct prevote and
//                             precommit signers, signers with both
//   D  (h, r, type, From)     first-wins logs (process.go:834-847)
//   C  (G slot, type, value)  count of first-wins votes per value
//                             (process.go:574-579 and the other count loops)
//
// A slot's `claim` word holds the LOWEST batch index of its key: a new key
// claims an empty slot by CAS, an equal key with a lower index lowers it by
// atomicMin.  Keys are never copied -- a probe compares against the
// claimer's fields in the (immutable) batch, so there is no torn-key window.
// Device-scope atomics execute at the memory side on gfx950 (tens of ns, ~11
// ns per op on one word), so everything else is read-only probing and
// wavefront-aggregated adds: the distinct signers of a round over both types
// (TraceLogs[r] restricted to votes, process.go:744-754) are prevotes +
// precommits - signers with both, found by probing D for the opposite type.
// Counts are integer atomics, hence deterministic; outputs are ordered by the
// batch index of each group's first message.
// Non-winners compare their value with the winner's: identical -> dropped
// silently, different -> the double vote handed to Catcher.CatchDouble*
// (process.go:838-843, 875-880).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "hd_internal.h"
#include "hd_verify_msg.h"

using namespace hd;

static const uint32_t kEmpty = 0xFFFFFFFFu;

struct TallyWork {
    DevBuf b[12];
};
enum TSlot { T_G, T_D, T_C, T_GSLOT, T_DSLOT, T_NSEL, T_SEL, T_SORTK, T_SORTV, T_TMP, T_DUP };

// table layouts (structure of arrays inside one allocation, capacity cap)
struct GTab {   // (h, r)
    uint32_t* claim;
    uint32_t* nprev;
    uint32_t* nprec;
    uint32_t* nboth;
};
struct CTab {   // (G slot, type, value)
    uint32_t* claim;
    uint32_t* n;
};

HD uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

HD uint64_t hash_hr(int64_t h, int64_t r) {
    return mix64((uint64_t)h * 0x9E3779B97F4A7C15ull ^ mix64((uint64_t)r));
}
// partition of a round among nparts (the high half of its hash; the table
// probes use the low bits)
HD uint32_t part_of(uint64_t hhr, uint32_t nparts) { return nparts > 1 ? (uint32_t)((hhr >> 32) % nparts) : 0u; }

struct Part {
    uint32_t part, nparts;
};

__device__ __forceinline__ bool candidate(const DevBatch& b, const uint8_t* verdict, const uint32_t* bitmap,
                                          uint32_t i, Part p) {
    const uint8_t t = b.type[i];
    if (t != T_PREVOTE && t != T_PRECOMMIT) return false;
    if (!(verdict ? verdict[i] == V_VALID : ((bitmap[i >> 5] >> (i & 31)) & 1u))) return false;
    return p.nparts <= 1 || part_of(hash_hr(b.height[i], b.round[i]), p.nparts) == p.part;
}

// candidates of the partition (sizes the hash tables): a wavefront sum,
// then one global atomic per wavefront (a shared-memory atomic from every
// lane serialises the block: measured 114 us per 1M messages)
__global__ __launch_bounds__(256) void k_tally_count(DevBatch b, const uint8_t* __restrict__ verdict,
                                                     const uint32_t* __restrict__ bitmap, Part p,
                                                     uint32_t* __restrict__ count) {
    uint32_t mine = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += gridDim.x * blockDim.x)
        mine += candidate(b, verdict, bitmap, i, p) ? 1u : 0u;
    HD_UNROLL for (int off = 32; off > 0; off >>= 1) mine += (uint32_t)__shfl_xor((int)mine, off, 64);
    if ((threadIdx.x & 63) == 0 && mine) atomicAdd(count, mine);
}

__device__ __forceinline__ bool eq32(const uint8_t* a, const uint8_t* b) {
    const uint4* x = reinterpret_cast<const uint4*>(a);
    const uint4* y = reinterpret_cast<const uint4*>(b);
    const uint4 x0 = x[0], x1 = x[1], y0 = y[0], y1 = y[1];
    return ((x0.x ^ y0.x) | (x0.y ^ y0.y) | (x0.z ^ y0.z) | (x0.w ^ y0.w) | (x1.x ^ y1.x) | (x1.y ^ y1.y) |
            (x1.z ^ y1.z) | (x1.w ^ y1.w)) == 0;
}

// Claim-or-find.  Returns the slot and whether this call created it; the
// slot's claim word ends up holding the lowest index of its key.
template <typename Eq>
__device__ __forceinline__ uint32_t probe(uint32_t* claim, uint32_t mask, uint64_t hash, uint32_t i, Eq eq,
                                          bool& created) {
    uint32_t s = (uint32_t)hash & mask;
    while (true) {
        uint32_t c = claim[s];
        if (c == kEmpty) {
            c = atomicCAS(&claim[s], kEmpty, i);
            if (c == kEmpty) {
                created = true;
                return s;
            }
        }
        if (eq(c)) {
            if (i < c) atomicMin(&claim[s], i);
            created = false;
            return s;
        }
        s = (s + 1) & mask;
    }
}
// Read-only lookup (the table is complete): the slot of a key that exists.
template <typename Eq>
__device__ __forceinline__ uint32_t find(const uint32_t* claim, uint32_t mask, uint64_t hash, Eq eq) {
    uint32_t s = (uint32_t)hash & mask;
    while (true) {
        const uint32_t c = claim[s];
        if (c == kEmpty) return kEmpty;
        if (eq(c)) return s;
        s = (s + 1) & mask;
    }
}

// Adds one wavefront's 0/1 increments to a counter array.  Lanes of a
// wavefront usually share their slot (batches arrive in height order), so
// the lanes whose slot equals the first active lane's add with one atomic
// (ballot + popcount over the active lanes only); the others fall back to
// their own.
__device__ __forceinline__ void wave_add(uint32_t* ctr, uint32_t slot, bool inc) {
    const unsigned long long act = __ballot(true);
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)act) - 1;
    const uint32_t s0 = __shfl(slot, leader, 64);
    const bool mine = slot == s0;
    const uint32_t v = (uint32_t)__popcll(__ballot(mine && inc));
    if (lane == leader && v) atomicAdd(&ctr[s0], v);
    if (!mine && inc) atomicAdd(&ctr[slot], 1u);
}

// Lanes of a wavefront usually share their round (batches arrive in height
// order): the first active lane -- the lowest batch index among them -- probes
// for every lane whose key equals its key and broadcasts the slot; the
// others probe on their own.  Skipping the followers' probes keeps the
// first-wins claim exact: their indices are higher than the leader's.  This
// turns up to 64 same-address CAS / atomicMin per wavefront into one.
__device__ __forceinline__ int first_active_lane() {
    return __ffsll((long long)__ballot(true)) - 1;
}
__device__ __forceinline__ int64_t shfl64(int64_t v, int src) {
    const int lo = __shfl((int)(uint32_t)v, src, 64), hi = __shfl((int)(uint32_t)((uint64_t)v >> 32), src, 64);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

__device__ __forceinline__ uint64_t hash_log(uint64_t hhr, const uint8_t* from, uint32_t t) {
    return mix64(hhr ^ *reinterpret_cast<const uint64_t*>(from) ^ (uint64_t)t);
}

// pass 1: every candidate -> its round (G) and its log entry (D, first-wins:
// the lowest index of the key); a new D slot counts a distinct signer of
// that type in the round.
__global__ void k_tally_logs(DevBatch b, const uint8_t* __restrict__ verdict, const uint32_t* __restrict__ bitmap,
                             Part p, GTab G, uint32_t* __restrict__ D, uint32_t mask, uint32_t* __restrict__ gslot,
                             uint32_t* __restrict__ dslot, uint8_t* __restrict__ dup) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += stride) {
        if (!candidate(b, verdict, bitmap, i, p)) {
            if (dup) dup[i] = 3;
            gslot[i] = kEmpty;
            continue;
        }
        const int64_t h = b.height[i], r = b.round[i];
        const uint8_t t = b.type[i];
        const uint8_t* from = b.from32 + 32 * (size_t)i;
        const uint64_t hhr = hash_hr(h, r);
        bool created;
        const int lead = first_active_lane();
        const bool follower = shfl64(h, lead) == h && shfl64(r, lead) == r && (int)(threadIdx.x & 63) != lead;
        uint32_t g = kEmpty;
        if (!follower)
            g = probe(G.claim, mask, hhr, i, [&](uint32_t c) { return b.height[c] == h && b.round[c] == r; },
                      created);
        {
            const uint32_t gl = (uint32_t)__shfl((int)g, lead, 64);
            if (follower) g = gl;
        }
        const uint32_t d = probe(D, mask, hash_log(hhr, from, t), i,
                                 [&](uint32_t c) {
                                     return b.type[c] == t && b.height[c] == h && b.round[c] == r &&
                                            eq32(b.from32 + 32 * (size_t)c, from);
                                 },
                                 created);
        wave_add(G.nprev, g, created && t == T_PREVOTE);
        wave_add(G.nprec, g, created && t == T_PRECOMMIT);
        gslot[i] = g;
        dslot[i] = d;
    }
}

// pass 2: winners count their value (C) and, for prevotes, whether the same
// signer also has a precommit log in the round; the rest are classified
// against the winner's value.
__global__ void k_tally_values(DevBatch b, const uint32_t* __restrict__ D, GTab G, CTab C, uint32_t mask,
                               const uint32_t* __restrict__ gslot, const uint32_t* __restrict__ dslot,
                               uint8_t* __restrict__ dup) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += stride) {
        const uint32_t g = gslot[i];
        if (g == kEmpty) continue;
        const uint32_t w = D[dslot[i]];
        const uint8_t* value = b.value32 + 32 * (size_t)i;
        if (w != i) {
            if (dup) dup[i] = eq32(b.value32 + 32 * (size_t)w, value) ? 1 : 2;
            continue;
        }
        if (dup) dup[i] = 0;
        const uint8_t t = b.type[i];
        const int64_t h = b.height[i], r = b.round[i];
        const uint8_t* from = b.from32 + 32 * (size_t)i;
        bool both = false;
        if (t == T_PREVOTE) {
            const uint32_t o = find(D, mask, hash_log(hash_hr(h, r), from, T_PRECOMMIT), [&](uint32_t c) {
                return b.type[c] == T_PRECOMMIT && b.height[c] == h && b.round[c] == r &&
                       eq32(b.from32 + 32 * (size_t)c, from);
            });
            both = o != kEmpty;
        }
        wave_add(G.nboth, g, both);
        const uint64_t hv = *reinterpret_cast<const uint64_t*>(value) ^ *reinterpret_cast<const uint64_t*>(value + 8);
        bool created;
        // same (round, type, value) as the wave's first active winner: share its slot
        const int lead = first_active_lane();
        const uint4* vw = reinterpret_cast<const uint4*>(value);
        const uint4 v0 = vw[0], v1 = vw[1];
        uint32_t diff = (uint32_t)__shfl((int)g, lead, 64) ^ g;
        diff |= (uint32_t)__shfl((int)t, lead, 64) ^ t;
        diff |= (uint32_t)__shfl((int)v0.x, lead, 64) ^ v0.x;
        diff |= (uint32_t)__shfl((int)v0.y, lead, 64) ^ v0.y;
        diff |= (uint32_t)__shfl((int)v0.z, lead, 64) ^ v0.z;
        diff |= (uint32_t)__shfl((int)v0.w, lead, 64) ^ v0.w;
        diff |= (uint32_t)__shfl((int)v1.x, lead, 64) ^ v1.x;
        diff |= (uint32_t)__shfl((int)v1.y, lead, 64) ^ v1.y;
        diff |= (uint32_t)__shfl((int)v1.z, lead, 64) ^ v1.z;
        diff |= (uint32_t)__shfl((int)v1.w, lead, 64) ^ v1.w;
        const bool follower = diff == 0 && (int)(threadIdx.x & 63) != lead;
        uint32_t c = kEmpty;
        if (!follower)
            c = probe(C.claim, mask, mix64(hv ^ ((uint64_t)g << 1 | (t & 1u))), i,
                      [&](uint32_t o) {
                          return gslot[o] == g && b.type[o] == t && eq32(b.value32 + 32 * (size_t)o, value);
                      },
                      created);
        {
            const uint32_t cl = (uint32_t)__shfl((int)c, lead, 64);
            if (follower) c = cl;
        }
        wave_add(C.n, c, true);
    }
}

// occupied slots -> (lowest index, slot) pairs.  Each block compacts a
// chunk of HD_USED_CHUNK slots in order and reserves its output range with
// ONE atomic (same-word atomics serialise at the memory side).
#define HD_USED_CHUNK 8192
__global__ __launch_bounds__(256) void k_tally_used(uint32_t cap, const uint32_t* __restrict__ claim,
                                                    uint32_t* __restrict__ key, uint32_t* __restrict__ val,
                                                    uint32_t* __restrict__ count) {
    typedef hipcub::BlockScan<uint32_t, 256> Scan;
    __shared__ typename Scan::TempStorage ts;
    __shared__ uint32_t base;
    const uint32_t lo = blockIdx.x * HD_USED_CHUNK;
    const int per = HD_USED_CHUNK / 256;  // contiguous slots per thread
    const uint32_t s0 = lo + threadIdx.x * per;
    uint32_t mine = 0;
    for (int k = 0; k < per; k++) mine += (s0 + k < cap && claim[s0 + k] != kEmpty) ? 1u : 0u;
    uint32_t off = 0, total = 0;
    Scan(ts).ExclusiveSum(mine, off, total);
    if (threadIdx.x == 0) base = total ? atomicAdd(count, total) : 0u;
    __syncthreads();
    uint32_t o = base + off;
    for (int k = 0; k < per && mine; k++) {
        const uint32_t s = s0 + k;
        if (s < cap) {
            const uint32_t c = claim[s];
            if (c != kEmpty) {
                key[o] = c;
                val[o] = s;
                o++;
            }
        }
    }
}

__global__ void k_tally_emit_hr(uint32_t n_hr, const uint32_t* __restrict__ slot, GTab G, const int64_t* __restrict__ h,
                                const int64_t* __restrict__ r, int64_t* __restrict__ oh, int64_t* __restrict__ orr,
                                uint32_t* __restrict__ oprev, uint32_t* __restrict__ oprec, uint32_t* __restrict__ oany,
                                uint32_t* __restrict__ orep) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_hr) return;
    const uint32_t s = slot[k], i = G.claim[s];
    orep[k] = i;
    oh[k] = h[i];
    orr[k] = r[i];
    oprev[k] = G.nprev[s];
    oprec[k] = G.nprec[s];
    oany[k] = G.nprev[s] + G.nprec[s] - G.nboth[s];
}

__global__ void k_tally_emit_counts(uint32_t n_c, const uint32_t* __restrict__ slot, CTab C, const int64_t* __restrict__ h,
                                    const int64_t* __restrict__ r, const uint8_t* __restrict__ type,
                                    int64_t* __restrict__ oh, int64_t* __restrict__ orr, uint8_t* __restrict__ ot,
                                    uint32_t* __restrict__ orep, uint32_t* __restrict__ on) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_c) return;
    const uint32_t s = slot[k], i = C.claim[s];
    oh[k] = h[i];
    orr[k] = r[i];
    ot[k] = type[i];
    orep[k] = i;
    on[k] = C.n[s];
}

// ---------------------------------------------------------------- host side
#define TCHK(expr, what)                                         \
    do {                                                         \
        hipError_t _e = (expr);                                  \
        if (_e != hipSuccess) return hd_ctx_fail(ctx, _e, what); \
    } while (0)

static void* tbuf(hd_ctx* ctx, int slot, size_t bytes, int* rc) {
    DevBuf& b = ctx->tally->b[slot];
    int r = hd_dev_grow(ctx, &b.p, &b.cap, bytes);
    if (r) {
        *rc = r;
        return nullptr;
    }
    return b.p;
}

void hd_tally_release(hd_ctx* ctx) {
    if (!ctx || !ctx->tally) return;
    for (auto& b : ctx->tally->b)
        if (b.p) (void)hipFree(b.p);
    delete ctx->tally;
    ctx->tally = nullptr;
}

static inline uint32_t nblk(uint32_t n) { return (n + 255) / 256; }

// Sort the occupied slots of a table by their group's first batch index.
// Returns the number of groups in *n_out (host) and the slot order in *order.
static int used_sorted(hd_ctx* ctx, uint32_t cap, const uint32_t* claim, uint32_t** order, uint32_t* n_out,
                       hipStream_t s) {
    int rc = 0;
    uint32_t* cnt = (uint32_t*)tbuf(ctx, T_NSEL, 64, &rc);
    uint32_t* key = (uint32_t*)tbuf(ctx, T_SORTK, 8 * (size_t)cap, &rc);
    uint32_t* val = (uint32_t*)tbuf(ctx, T_SORTV, 8 * (size_t)cap, &rc);
    if (rc) return rc;
    TCHK(hipMemsetAsync(cnt, 0, 4, s), "memset count");
    k_tally_used<<<(cap + HD_USED_CHUNK - 1) / HD_USED_CHUNK, 256, 0, s>>>(cap, claim, key, val, cnt);
    uint32_t n = 0;
    TCHK(hipMemcpyAsync(&n, cnt, 4, hipMemcpyDeviceToHost, s), "group count");
    TCHK(hipStreamSynchronize(s), "group count sync");
    *n_out = n;
    if (n == 0) {
        *order = val;
        return HD_OK;
    }
    hipcub::DoubleBuffer<uint32_t> kk(key, key + cap), vv(val, val + cap);
    size_t need = 0;
    TCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, need, kk, vv, n, 0, 32, s), "sort size");
    void* tmp = tbuf(ctx, T_TMP, need, &rc);
    if (rc) return rc;
    TCHK(hipcub::DeviceRadixSort::SortPairs(tmp, need, kk, vv, n, 0, 32, s), "sort groups");
    *order = vv.Current();
    return HD_OK;
}

static int tally_device(hd_ctx* ctx, const hd_batch* hb, const uint8_t* d_verdict, const uint32_t* d_bitmap,
                        Part part, hd_tally_out* out, hipStream_t s) {
    const uint32_t n = hb->n;
    if (!ctx->tally) ctx->tally = new TallyWork();
    DevBatch b{n, hb->type, hb->height, hb->round, hb->valid_round, hb->value32, hb->from32, hb->sig65};
    int rc = 0;
    const uint32_t grid = std::min<uint32_t>(nblk(n), (uint32_t)ctx->n_cu * 16u);
    // the tables hold at most one key per candidate: size them by this
    // partition's candidates (one counting pass), load factor <= 1/2 so
    // probes terminate
    uint32_t n_cand = n;
    {
        uint32_t* cnt = (uint32_t*)tbuf(ctx, T_NSEL, 64, &rc);
        if (rc) return rc;
        TCHK(hipMemsetAsync(cnt + 1, 0, 4, s), "clear candidate count");
        k_tally_count<<<grid, 256, 0, s>>>(b, d_verdict, d_bitmap, part, cnt + 1);
        TCHK(hipMemcpyAsync(&n_cand, cnt + 1, 4, hipMemcpyDeviceToHost, s), "candidate count");
        TCHK(hipStreamSynchronize(s), "candidate count sync");
    }
    uint32_t cap = 1024;
    while (cap < 2 * n_cand) cap <<= 1;
    const uint32_t mask = cap - 1;
    uint32_t* g = (uint32_t*)tbuf(ctx, T_G, 20 * (size_t)cap, &rc);  // 16 B used; staging for the outputs
    uint32_t* d = (uint32_t*)tbuf(ctx, T_D, 4 * (size_t)cap, &rc);
    uint32_t* c = (uint32_t*)tbuf(ctx, T_C, 8 * (size_t)cap, &rc);
    uint32_t* gslot = (uint32_t*)tbuf(ctx, T_GSLOT, 4 * (size_t)n, &rc);
    uint32_t* dslot = (uint32_t*)tbuf(ctx, T_DSLOT, 4 * (size_t)n, &rc);
    uint8_t* d_dup = out->dup ? (uint8_t*)tbuf(ctx, T_DUP, n, &rc) : nullptr;
    if (rc) return rc;
    if (n_cand == 0) {   // nothing to tally here (dup: every message 3)
        out->n_hr = out->n_counts = 0;
        if (out->dup) memset(out->dup, 3, n);
        return HD_OK;
    }
    GTab G{g, g + cap, g + 2 * (size_t)cap, g + 3 * (size_t)cap};
    CTab C{c, c + cap};
    // claim words := empty; counters := 0
    TCHK(hipMemsetAsync(g, 0xFF, 4 * (size_t)cap, s), "clear G");
    TCHK(hipMemsetAsync(G.nprev, 0, 12 * (size_t)cap, s), "clear G counters");
    TCHK(hipMemsetAsync(d, 0xFF, 4 * (size_t)cap, s), "clear D");
    TCHK(hipMemsetAsync(c, 0xFF, 4 * (size_t)cap, s), "clear C");
    TCHK(hipMemsetAsync(C.n, 0, 4 * (size_t)cap, s), "clear C counters");
    k_tally_logs<<<grid, 256, 0, s>>>(b, d_verdict, d_bitmap, part, G, d, mask, gslot, dslot, d_dup);
    k_tally_values<<<grid, 256, 0, s>>>(b, d, G, C, mask, gslot, dslot, d_dup);
    TCHK(hipGetLastError(), "tally kernels");

    uint32_t n_hr = 0, n_cnt = 0;
    uint32_t* order = nullptr;
    rc = used_sorted(ctx, cap, G.claim, &order, &n_hr, s);
    if (rc) return rc;
    out->n_hr = n_hr;
    if (n_hr && n_hr <= out->cap_hr) {
        char* st = (char*)tbuf(ctx, T_SEL, 32 * (size_t)n_hr, &rc);
        if (rc) return rc;
        int64_t* o_h = reinterpret_cast<int64_t*>(st);
        int64_t* o_r = o_h + n_hr;
        uint32_t* o_prev = reinterpret_cast<uint32_t*>(o_r + n_hr);
        uint32_t* o_prec = o_prev + n_hr;
        uint32_t* o_any = o_prec + n_hr;
        uint32_t* o_rep = o_any + n_hr;
        k_tally_emit_hr<<<nblk(n_hr), 256, 0, s>>>(n_hr, order, G, b.height, b.round, o_h, o_r, o_prev, o_prec, o_any,
                                                   o_rep);
        struct Cp { void* dst; const void* src; size_t sz; } cp[] = {
            {out->hr_height, o_h, 8 * (size_t)n_hr},     {out->hr_round, o_r, 8 * (size_t)n_hr},
            {out->hr_prevotes, o_prev, 4 * (size_t)n_hr}, {out->hr_precommits, o_prec, 4 * (size_t)n_hr},
            {out->hr_any, o_any, 4 * (size_t)n_hr},       {out->hr_rep, o_rep, 4 * (size_t)n_hr},
        };
        for (auto& x : cp)
            if (x.dst) TCHK(hipMemcpyAsync(x.dst, x.src, x.sz, hipMemcpyDeviceToHost, s), "hr download");
    }
    // (the count sort below reuses the sort buffers: same stream, so the
    // per-round emit above has consumed `order` before they are rewritten)
    rc = used_sorted(ctx, cap, C.claim, &order, &n_cnt, s);
    if (rc) return rc;
    out->n_counts = n_cnt;
    if (n_hr > out->cap_hr || n_cnt > out->cap_counts) {
        TCHK(hipStreamSynchronize(s), "sync");
        return HD_ECAP;
    }
    if (n_cnt) {
        // staging for the counts: the G table (20 B x cap, cap >= 2 n_cnt) is
        // no longer read once the per-round outputs are downloaded
        TCHK(hipStreamSynchronize(s), "hr sync");
        int64_t* c_h = reinterpret_cast<int64_t*>(g);
        int64_t* c_r = c_h + n_cnt;
        uint32_t* c_rep = reinterpret_cast<uint32_t*>(c_r + n_cnt);
        uint32_t* c_n = c_rep + n_cnt;
        uint8_t* c_t = reinterpret_cast<uint8_t*>(c_n + n_cnt);
        k_tally_emit_counts<<<nblk(n_cnt), 256, 0, s>>>(n_cnt, order, C, b.height, b.round, b.type, c_h, c_r, c_t,
                                                        c_rep, c_n);
        struct Cp { void* dst; const void* src; size_t sz; } cp[] = {
            {out->count_height, c_h, 8 * (size_t)n_cnt}, {out->count_round, c_r, 8 * (size_t)n_cnt},
            {out->count_type, c_t, (size_t)n_cnt},       {out->count_rep, c_rep, 4 * (size_t)n_cnt},
            {out->count_n, c_n, 4 * (size_t)n_cnt},
        };
        for (auto& x : cp) TCHK(hipMemcpyAsync(x.dst, x.src, x.sz, hipMemcpyDeviceToHost, s), "count download");
    }
    if (out->dup) TCHK(hipMemcpyAsync(out->dup, d_dup, (size_t)n, hipMemcpyDeviceToHost, s), "dup download");
    TCHK(hipStreamSynchronize(s), "tally sync");
    return HD_OK;
}

static bool tally_out_ok(const hd_tally_out* o) {
    return o && o->count_height && o->count_round && o->count_type && o->count_rep && o->count_n && o->hr_height &&
           o->hr_round && o->hr_prevotes && o->hr_precommits && o->hr_any;
}

extern "C" {

int hd_tally(hd_ctx* ctx, const hd_batch* batch, const uint8_t* verdict, hd_tally_out* out) {
    if (!ctx || !batch || !verdict || !tally_out_ok(out)) return HD_EINVAL;
    if (!batch->type || !batch->height || !batch->round || !batch->value32 || !batch->from32) return HD_EINVAL;
    out->n_counts = out->n_hr = 0;
    if (batch->n == 0) return HD_OK;
    (void)hipSetDevice(ctx->device);
    hd_batch hb = *batch;
    hb.sig65 = nullptr;  // not needed
    hb.valid_round = nullptr;
    hd_batch db;
    int rc = hd_upload_batch(ctx, &hb, &db);
    if (rc) return rc;
    rc = hd_dev_grow(ctx, &ctx->bufs[BUF_VERDICT].p, &ctx->bufs[BUF_VERDICT].cap, batch->n);
    if (rc) return rc;
    uint8_t* d_v = (uint8_t*)ctx->bufs[BUF_VERDICT].p;
    TCHK(hipMemcpyAsync(d_v, verdict, batch->n, hipMemcpyHostToDevice, ctx->stream), "verdict upload");
    return tally_device(ctx, &db, d_v, nullptr, Part{0, 1}, out, ctx->stream);
}

int hd_tally_device(hd_ctx* ctx, const hd_batch* dbatch, const uint8_t* d_verdict, hd_tally_out* out, void* stream) {
    if (!ctx || !dbatch || !tally_out_ok(out)) return HD_EINVAL;
    if (dbatch->n && !d_verdict) return HD_EINVAL;
    out->n_counts = out->n_hr = 0;
    if (dbatch->n == 0) return HD_OK;
    (void)hipSetDevice(ctx->device);
    return tally_device(ctx, dbatch, d_verdict, nullptr, Part{0, 1}, out, stream ? (hipStream_t)stream : ctx->stream);
}

int hd_tally_device_bitmap(hd_ctx* ctx, const hd_batch* dbatch, const uint32_t* d_valid_bitmap, hd_tally_out* out,
                           void* stream) {
    return hd_tally_device_bitmap_part(ctx, dbatch, d_valid_bitmap, 0, 1, out, stream);
}

int hd_tally_device_bitmap_part(hd_ctx* ctx, const hd_batch* dbatch, const uint32_t* d_valid_bitmap, uint32_t part,
                                uint32_t nparts, hd_tally_out* out, void* stream) {
    if (!ctx || !dbatch || !tally_out_ok(out) || nparts == 0 || part >= nparts) return HD_EINVAL;
    if (dbatch->n && !d_valid_bitmap) return HD_EINVAL;
    out->n_counts = out->n_hr = 0;
    if (dbatch->n == 0) return HD_OK;
    (void)hipSetDevice(ctx->device);
    return tally_device(ctx, dbatch, nullptr, d_valid_bitmap, Part{part, nparts}, out,
                        stream ? (hipStream_t)stream : ctx->stream);
}

uint32_t hd_tally_partition_of(int64_t height, int64_t round, uint32_t nparts) {
    return part_of(hash_hr(height, round), nparts);
}

int hd_process_batch(hd_ctx* ctx, const hd_batch* batch, uint8_t* verdict, uint8_t* recovered32,
                     uint32_t* valid_bitmap, hd_tally_out* tally) {
    if (!ctx || !batch || !verdict || !tally_out_ok(tally)) return HD_EINVAL;
    tally->n_counts = tally->n_hr = 0;
    if (batch->n == 0) return HD_OK;
    (void)hipSetDevice(ctx->device);
    hd_batch db;
    int rc = hd_upload_batch(ctx, batch, &db);
    if (rc) return rc;
    rc = hd_verify_uploaded(ctx, &db, verdict, recovered32, valid_bitmap);
    if (rc) return rc;
    return tally_device(ctx, &db, (const uint8_t*)ctx->bufs[BUF_VERDICT].p, nullptr, Part{0, 1}, tally, ctx->stream);
}

}  // extern "C"
