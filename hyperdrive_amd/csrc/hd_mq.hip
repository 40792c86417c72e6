// hd_mq.hip -- bulk MessageQueue (include/hd_mq.h; mq/mq.go:19-143).
//
// Senders.  mq.go keys its queues by the message's From (a 32-byte
// id.Signatory, mq.go:107-113).  The queue interns every From it sees into a
// dense sender id, assigned in order of first insertion and never reused: a
// device hash table (id per slot, keys compared against the interned 32-byte
// Froms) plus the array of interned Froms.  A batch looks its Froms up
// read-only; the Froms it introduces are deduplicated in a batch-local table
// (the slot's claim word keeps the lowest batch position, compared against
// the batch's own bytes), numbered in batch order and inserted into the hash
// table with one CAS each (they are distinct and new, so no comparison is
// needed there).
//
// Messages.  The queue is one SoA pool of messages kept sorted by (sender id,
// height, round, arrival).  A batch insert appends the batch's messages after
// the pool (so arrival order == position for equal keys), re-sorts with
// stable LSD radix passes over (round, height, sender) -- keys rebased to the
// batch's min and cut to their significant bits, so a typical insert costs a
// handful of 8-bit digit passes -- and keeps each sender's first max_capacity
// elements: exactly the result of inserting one message at a time with
// mq.go:133-142's truncation.  Consume(h) and DropMessagesBelowHeight(h)
// remove a prefix of every sender's run (mq.go:38-41, 70-83), so they only
// move per-sender head offsets: one single-block kernel binary-searches each
// run for the cut and scans the delivered counts, one kernel gathers the
// delivered prefixes (of senders in procsAllowed, mq.go:49-51, evaluated
// against the set given at that call) into a packed stage that comes back in
// ONE copy.  The consumed prefixes are compacted away lazily, by the next
// insert, which rebuilds the pool anyway -- a consume costs two host syncs
// and no pass over the pool.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <new>

#include "../../include/hd_mq.h"
#include "../../include/hd_votes.h"
#include "hd_internal.h"

using namespace hd;

namespace {

static const uint32_t kEmpty = 0xFFFFFFFFu;

struct Pool {
    uint32_t n = 0, cap = 0;
    int32_t* sender = nullptr;
    uint8_t* type = nullptr;
    int64_t* h = nullptr;
    int64_t* r = nullptr;
    int64_t* vr = nullptr;
    uint8_t* value = nullptr;
    uint8_t* from = nullptr;
    uint8_t* sig = nullptr;
    void* base = nullptr;
};

// one allocation per pool: 4 + 1 + 8 + 8 + 8 + 32 + 32 + 65 = 158 B / message
int pool_reserve(hd_ctx* ctx, Pool& p, uint32_t need) {
    if (need <= p.cap) return HD_OK;
    uint32_t cap = std::max<uint32_t>(need, std::max<uint32_t>(1024u, p.cap + p.cap / 2));
    cap = (cap + 15u) & ~15u;  // every field array 16-byte aligned (uint4 copies)
    const size_t c = cap;
    const size_t bytes = c * (8 + 8 + 8 + 32 + 32 + 65 + 4 + 1) + 64;
    void* base = nullptr;
    hipError_t e = hipMalloc(&base, bytes);
    if (e != hipSuccess) return hd_ctx_fail(ctx, e, "hipMalloc mq pool");
    if (p.base) (void)hipFree(p.base);
    char* b = (char*)base;
    p.h = (int64_t*)b;
    p.r = p.h + c;
    p.vr = p.r + c;
    p.value = (uint8_t*)(p.vr + c);
    p.from = p.value + 32 * c;
    p.sig = p.from + 32 * c;
    p.sender = (int32_t*)(((uintptr_t)(p.sig + 65 * c) + 15) & ~(uintptr_t)15);
    p.type = (uint8_t*)(p.sender + c);
    p.base = base;
    p.cap = cap;
    return HD_OK;
}

// the Pool field layout inside a region of pool_bytes(cap) bytes at base
size_t pool_bytes(uint32_t cap) { return (size_t)cap * (8 + 8 + 8 + 32 + 32 + 65 + 4 + 1) + 64; }
Pool pool_view(void* base, uint32_t cap) {
    Pool p;
    const size_t c = cap;
    char* b = (char*)base;
    p.h = (int64_t*)b;
    p.r = p.h + c;
    p.vr = p.r + c;
    p.value = (uint8_t*)(p.vr + c);
    p.from = p.value + 32 * c;
    p.sig = p.from + 32 * c;
    p.sender = (int32_t*)(((uintptr_t)(p.sig + 65 * c) + 15) & ~(uintptr_t)15);
    p.type = (uint8_t*)(p.sender + c);
    p.base = base;
    p.cap = cap;
    p.n = 0;
    return p;
}

// ---------------------------------------------------------------- senders
// The interned Froms (8 little-endian words each, the bytes as given) and
// the hash table of their ids.
struct Dict {
    const uint32_t* keys;
    const uint32_t* slots;
    uint32_t mask;
    uint64_t seed;
};

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}
// From is a SHA-256 output, but the seed (per queue) keeps crafted signatories
// from lining up in one probe chain
__device__ __forceinline__ uint32_t key_hash(const uint4& a, const uint4& b, uint64_t seed) {
    const uint64_t x = ((uint64_t)a.y << 32 | a.x) ^ mix64(((uint64_t)a.w << 32 | a.z) ^ seed) ^
                       ((uint64_t)b.y << 32 | b.x) * 0x9E3779B97F4A7C15ull ^ ((uint64_t)b.w << 32 | b.z);
    return (uint32_t)mix64(x ^ seed);
}
__device__ __forceinline__ bool key_eq(const uint4& a, const uint4& b, const uint32_t* k) {
    const uint4 c = reinterpret_cast<const uint4*>(k)[0], d = reinterpret_cast<const uint4*>(k)[1];
    return ((a.x ^ c.x) | (a.y ^ c.y) | (a.z ^ c.z) | (a.w ^ c.w) | (b.x ^ d.x) | (b.y ^ d.y) | (b.z ^ d.z) |
            (b.w ^ d.w)) == 0;
}
__device__ __forceinline__ void load_key(const uint8_t* p, uint4& a, uint4& b) {
    a = reinterpret_cast<const uint4*>(p)[0];
    b = reinterpret_cast<const uint4*>(p)[1];
}
// id of an interned From, or kEmpty
__device__ __forceinline__ uint32_t dict_find(const Dict& d, const uint4& a, const uint4& b) {
    uint32_t s = key_hash(a, b, d.seed) & d.mask;
    while (true) {
        const uint32_t id = d.slots[s];
        if (id == kEmpty || key_eq(a, b, d.keys + 8 * (size_t)id)) return id;
        s = (s + 1) & d.mask;
    }
}
// put a From known to be absent into the table (the keys are distinct)
__device__ __forceinline__ void dict_put(uint32_t* slots, uint32_t mask, uint64_t seed, const uint4& a, const uint4& b,
                                         uint32_t id) {
    uint32_t s = key_hash(a, b, seed) & mask;
    while (atomicCAS(&slots[s], kEmpty, id) != kEmpty) s = (s + 1) & mask;
}

// insert flag of a verified message: authenticated (recovered == From: VALID
// or NOT_ADMITTED) and filterHeight (replica.go:247-249)
__global__ void k_mq_ingress(uint32_t n, const uint8_t* __restrict__ verdict, const int64_t* __restrict__ height,
                             int64_t min_height, uint8_t* __restrict__ flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint8_t v = verdict[i];
        flag[i] = (v == HD_VERDICT_VALID || v == HD_VERDICT_NOT_ADMITTED) && height[i] >= min_height;
    }
}
__global__ void k_mq_flag_nz(uint32_t n, const uint8_t* __restrict__ in, uint8_t* __restrict__ flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = in ? in[i] != 0 : 1;
}

// Sender of each insertable message (position e of newidx): an interned id,
// or -- for a From the queue has not seen -- a slot of the batch-local table
// whose claim word ends as the lowest position with that From.
__global__ void k_mq_lookup(uint32_t m, const uint32_t* __restrict__ newidx, const uint8_t* __restrict__ from32,
                            Dict d, uint32_t* __restrict__ lclaim, uint32_t lmask, uint32_t* __restrict__ sid,
                            uint32_t* __restrict__ lslot) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    uint4 a, b;
    load_key(from32 + 32 * (size_t)newidx[e], a, b);
    const uint32_t id = dict_find(d, a, b);
    sid[e] = id;
    if (id != kEmpty) {
        lslot[e] = kEmpty;
        return;
    }
    uint32_t s = key_hash(a, b, d.seed ^ 0x5A5A5A5Aull) & lmask;
    while (true) {
        uint32_t c = lclaim[s];
        if (c == kEmpty) {
            c = atomicCAS(&lclaim[s], kEmpty, e);
            if (c == kEmpty) break;
        }
        uint4 x, y;
        load_key(from32 + 32 * (size_t)newidx[c], x, y);
        if (((a.x ^ x.x) | (a.y ^ x.y) | (a.z ^ x.z) | (a.w ^ x.w) | (b.x ^ y.x) | (b.y ^ y.y) | (b.z ^ y.z) |
             (b.w ^ y.w)) == 0) {
            if (e < c) atomicMin(&lclaim[s], e);
            break;
        }
        s = (s + 1) & lmask;
    }
    lslot[e] = s;
}
// first occurrence of a new From in the batch
__global__ void k_mq_newflag(uint32_t m, const uint32_t* __restrict__ lslot, const uint32_t* __restrict__ lclaim,
                             uint8_t* __restrict__ flag) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < m) flag[e] = lslot[e] != kEmpty && lclaim[lslot[e]] == e;
}
// new sender k (batch order) gets id base + k
__global__ void k_mq_assign(const uint32_t* __restrict__ r_dev, const uint32_t* __restrict__ reps,
                            const uint32_t* __restrict__ newidx,
                            const uint8_t* __restrict__ from32, uint32_t base, uint32_t* __restrict__ keys,
                            uint32_t* __restrict__ slots, uint32_t mask, uint64_t seed,
                            const uint32_t* __restrict__ lslot, uint32_t* __restrict__ lid) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= *r_dev) return;
    const uint32_t e = reps[k], id = base + k;
    uint4 a, b;
    load_key(from32 + 32 * (size_t)newidx[e], a, b);
    reinterpret_cast<uint4*>(keys + 8 * (size_t)id)[0] = a;
    reinterpret_cast<uint4*>(keys + 8 * (size_t)id)[1] = b;
    dict_put(slots, mask, seed, a, b, id);
    lid[lslot[e]] = id;
}
__global__ void k_mq_sid(uint32_t m, const uint32_t* __restrict__ lslot, const uint32_t* __restrict__ lid,
                         uint32_t* __restrict__ sid) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < m && lslot[e] != kEmpty) sid[e] = lid[lslot[e]];
}
// rebuild the hash table at a new capacity from the interned keys
__global__ void k_mq_rehash(uint32_t n, const uint32_t* __restrict__ keys, uint32_t* __restrict__ slots, uint32_t mask,
                            uint64_t seed) {
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= n) return;
    const uint4 a = reinterpret_cast<const uint4*>(keys + 8 * (size_t)id)[0];
    const uint4 b = reinterpret_cast<const uint4*>(keys + 8 * (size_t)id)[1];
    dict_put(slots, mask, seed, a, b, id);
}
// procsAllowed -> allow[id] for the interned senders.  The list is raw
// 32-byte signatories, or (be_words) the ctx's admitted table of 8 big-endian
// words per signatory.
__global__ void k_mq_allow(uint32_t na, const uint32_t* __restrict__ list, int be_words, Dict d,
                           uint8_t* __restrict__ allow) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= na) return;
    uint32_t w[8];
    for (int j = 0; j < 8; j++) {
        const uint32_t x = list[8 * (size_t)k + j];
        w[j] = be_words ? __builtin_bswap32(x) : x;
    }
    const uint4 a = make_uint4(w[0], w[1], w[2], w[3]), b = make_uint4(w[4], w[5], w[6], w[7]);
    const uint32_t id = dict_find(d, a, b);
    if (id != kEmpty) allow[id] = 1;
}

// element e of the merged sequence: e < M -> pool[e]; else batch[newidx[e - M]]
// with sender nsid[e - M]
struct MqSrc {
    Pool p;
    DevBatch b;
    const uint32_t* newidx;
    const uint32_t* nsid;
    uint32_t M;
};

__device__ __forceinline__ void src_keys(const MqSrc& s, uint32_t e, uint32_t& snd, int64_t& h, int64_t& r) {
    if (e < s.M) {
        snd = (uint32_t)s.p.sender[e];
        h = s.p.h[e];
        r = s.p.r[e];
    } else {
        const uint32_t i = s.newidx[e - s.M];
        snd = s.nsid[e - s.M];
        h = s.b.height[i];
        r = s.b.round[i];
    }
}

__global__ void k_mq_keys(MqSrc s, uint32_t T, int64_t* __restrict__ hk, int64_t* __restrict__ rk,
                          uint32_t* __restrict__ sk, uint32_t* __restrict__ iota,
                          unsigned long long* __restrict__ red) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < 5) red[e] = ~0ull;   // k_mq_minmax3's identities (the next launch)
    if (e >= T) return;
    uint32_t snd;
    int64_t h, r;
    src_keys(s, e, snd, h, r);
    hk[e] = h;
    rk[e] = r;
    sk[e] = snd;
    iota[e] = e;
}

// 64-bit sort key of element perm[k]: field - min, as unsigned
__global__ void k_mq_rekey64(uint32_t T, const uint32_t* __restrict__ perm, const int64_t* __restrict__ field,
                             int64_t minv, uint64_t* __restrict__ key) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < T) key[k] = (uint64_t)field[perm[k]] - (uint64_t)minv;
}
__global__ void k_mq_rekey32(uint32_t T, const uint32_t* __restrict__ perm, const uint32_t* __restrict__ field,
                             uint32_t* __restrict__ key) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < T) key[k] = field[perm[k]];
}

// one sort key for (sender, height, round), each rebased to its minimum and
// packed high to low, when the three ranges fit 64 bits together (element e
// in the merged sequence's order: the sort is stable, so ties keep arrival)
__global__ void k_mq_combine(uint32_t T, const int64_t* __restrict__ rk, const int64_t* __restrict__ hk,
                             const uint32_t* __restrict__ sk, int64_t rmn, int64_t hmn, int rb, int hb,
                             uint64_t* __restrict__ key) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= T) return;
    const uint64_t r = (uint64_t)rk[e] - (uint64_t)rmn, h = (uint64_t)hk[e] - (uint64_t)hmn;
    key[e] = ((((uint64_t)sk[e] << hb) | h) << rb) | r;
}

// position of each sorted element's sender run start (inclusive max-scan input)
__global__ void k_mq_heads(uint32_t T, const uint32_t* __restrict__ perm, const uint32_t* __restrict__ sk,
                           uint32_t* __restrict__ head) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= T) return;
    head[k] = (k == 0 || sk[perm[k]] != sk[perm[k - 1]]) ? k : 0u;
}
__global__ void k_mq_keep(uint32_t T, const uint32_t* __restrict__ seg, uint32_t cap, uint8_t* __restrict__ keep) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < T) keep[k] = (k - seg[k]) < cap;
}

// dst[k] := element sel[k] of the merged sequence.  A block's 256 signature
// rows are one contiguous, 4-byte aligned range of d.sig (65 B x 256 = 16,640
// B per block): each lane stages its source row in LDS as aligned dwords, and
// the block then writes the range as whole dwords assembled from LDS bytes --
// ~37 global accesses per message instead of 130 byte loads and stores.
__device__ __forceinline__ uint32_t ld_bytes(const uint8_t* p, uint32_t lo, uint32_t hi) {
    // bytes p[lo .. hi) into a dword at byte positions lo .. hi - 1 (the rest 0)
    uint32_t v = 0;
    for (uint32_t t = lo; t < hi; t++) v |= (uint32_t)p[t] << (8 * t);
    return v;
}
__global__ __launch_bounds__(256) void k_mq_gather(MqSrc s, uint32_t n, const uint32_t* __restrict__ sel, Pool d,
                                                   const uint32_t* __restrict__ n_dev = nullptr) {
    if (n_dev) n = *n_dev;   // the count on the device (the grid covers an upper bound)
    __shared__ uint32_t rows_lds[256 * 17];
    __shared__ uint8_t off_lds[256];
    const uint32_t tid = threadIdx.x;
    const uint32_t k = blockIdx.x * 256u + tid;
    const uint8_t* sg = nullptr;   // this lane's source signature row (nullptr: zeros)
    if (k < n) {
        const uint32_t e = sel[k];
        if (e < s.M) {
            d.sender[k] = s.p.sender[e];
            d.type[k] = s.p.type[e];
            d.h[k] = s.p.h[e];
            d.r[k] = s.p.r[e];
            d.vr[k] = s.p.vr[e];
            for (int w = 0; w < 2; w++) {
                reinterpret_cast<uint4*>(d.value + 32 * (size_t)k)[w] = reinterpret_cast<const uint4*>(s.p.value + 32 * (size_t)e)[w];
                reinterpret_cast<uint4*>(d.from + 32 * (size_t)k)[w] = reinterpret_cast<const uint4*>(s.p.from + 32 * (size_t)e)[w];
            }
            sg = s.p.sig + 65 * (size_t)e;
        } else {
            const uint32_t i = s.newidx[e - s.M];
            d.sender[k] = (int32_t)s.nsid[e - s.M];
            d.type[k] = s.b.type[i];
            d.h[k] = s.b.height[i];
            d.r[k] = s.b.round[i];
            d.vr[k] = s.b.valid_round ? s.b.valid_round[i] : -1;
            if ((((uintptr_t)s.b.value32 | (uintptr_t)s.b.from32) & 15) == 0) {
                for (int w = 0; w < 2; w++) {
                    reinterpret_cast<uint4*>(d.value + 32 * (size_t)k)[w] = reinterpret_cast<const uint4*>(s.b.value32 + 32 * (size_t)i)[w];
                    reinterpret_cast<uint4*>(d.from + 32 * (size_t)k)[w] = reinterpret_cast<const uint4*>(s.b.from32 + 32 * (size_t)i)[w];
                }
            } else {
                for (int w = 0; w < 32; w++) {
                    d.value[32 * (size_t)k + w] = s.b.value32[32 * (size_t)i + w];
                    d.from[32 * (size_t)k + w] = s.b.from32[32 * (size_t)i + w];
                }
            }
            if (s.b.sig65) sg = s.b.sig65 + 65 * (size_t)i;
        }
    }
    // stage: the 17 aligned dwords that cover the row; the first and the last
    // are assembled from byte loads, so nothing outside the row is read
    uint32_t* my = rows_lds + 17 * tid;
    uint32_t off = 0;
    if (sg) {
        off = (uint32_t)((uintptr_t)sg & 3u);
        const uint8_t* a0 = sg - off;
        my[0] = ld_bytes(a0, off, 4);
        const uint32_t* w32 = reinterpret_cast<const uint32_t*>(a0);
        for (int j = 1; j < 16; j++) my[j] = w32[j];
        my[16] = ld_bytes(a0 + 64, 0, off + 1);
    } else {
        for (int j = 0; j < 17; j++) my[j] = 0;
    }
    off_lds[tid] = (uint8_t)off;
    __syncthreads();
    const uint32_t k0 = blockIdx.x * 256u;
    if (k0 >= n) return;
    const uint32_t nb = n - k0 < 256u ? n - k0 : 256u;
    const uint32_t bytes = 65u * nb, full = bytes >> 2;
    const uint8_t* lb = reinterpret_cast<const uint8_t*>(rows_lds);
    uint32_t* dst = reinterpret_cast<uint32_t*>(d.sig + 65 * (size_t)k0);
    for (uint32_t D = tid; D < full; D += 256u) {
        uint32_t v = 0;
        for (uint32_t t = 0; t < 4; t++) {
            const uint32_t b = 4 * D + t, row = b / 65u, col = b - 65u * row;
            v |= (uint32_t)lb[68 * row + off_lds[row] + col] << (8 * t);
        }
        dst[D] = v;
    }
    if (tid == 0) {   // the last block's trailing bytes (65 nb is not a multiple of 4)
        for (uint32_t b = 4 * full; b < bytes; b++) {
            const uint32_t row = b / 65u, col = b - 65u * row;
            d.sig[65 * (size_t)k0 + b] = lb[68 * row + off_lds[row] + col];
        }
    }
}

// (also clears the ns-entry head / send arrays k_mq_runs fills two launches
// later, in place of two memsets)
__global__ void k_mq_compose(uint32_t n, const uint32_t* __restrict__ perm, const uint32_t* __restrict__ sel,
                             uint32_t* __restrict__ ids, const uint32_t* __restrict__ n_dev, uint32_t ns,
                             uint32_t* __restrict__ head, uint32_t* __restrict__ send) {
    if (n_dev) n = *n_dev;
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    for (uint32_t i = k; i < ns; i += gridDim.x * blockDim.x) head[i] = send[i] = 0;
    if (k < n) ids[k] = perm[sel[k]];
}

// partition predicates over the pool.  Consume (strict = 0): removed = height
// <= h, delivered = removed and the sender allowed (allow may be NULL: all);
// drop (strict = 1): removed = height < h.  inv = kept.
__global__ void k_mq_pred(uint32_t n, const int64_t* __restrict__ ph, const int32_t* __restrict__ psnd, int64_t h,
                          int strict, const uint8_t* __restrict__ allow, uint8_t* __restrict__ removed,
                          uint8_t* __restrict__ deliver, uint8_t* __restrict__ inv) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const bool f = strict ? ph[e] < h : ph[e] <= h;
    removed[e] = f;
    if (deliver) deliver[e] = f && (!allow || allow[psnd[e]]);
    inv[e] = !f;
}

// per sender run of a freshly sorted pool: head = its first index, send = one
// past its last (senders without messages keep 0, 0)
__global__ void k_mq_runs(uint32_t M, const int32_t* __restrict__ snd, uint32_t* __restrict__ head,
                          uint32_t* __restrict__ send, const uint32_t* __restrict__ M_dev = nullptr) {
    if (M_dev) M = *M_dev;
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= M) return;
    const int32_t s = snd[k];
    if (k == 0 || snd[k - 1] != s) head[s] = k;
    if (k == M - 1 || snd[k + 1] != s) send[s] = k + 1;
}

// Consume / DropMessagesBelowHeight plan, one block: for each sender the cut
// of its live run [head, send) -- the first message with height > h (consume)
// or >= h (drop, strict) -- by binary search (a run is sorted by height);
// removed = cut - head; delivered = removed for allowed senders (allow NULL:
// none delivered); off = exclusive scan of delivered; totals = {delivered,
// removed}; newhead = cut (committed by the caller once the outputs fit).
__global__ __launch_bounds__(1024) void k_mq_plan(uint32_t nsend, const int64_t* __restrict__ ph,
                                                  const uint32_t* __restrict__ head, const uint32_t* __restrict__ send,
                                                  int64_t h, int strict, const uint8_t* __restrict__ allow,
                                                  uint32_t* __restrict__ newhead, uint32_t* __restrict__ off,
                                                  uint32_t* __restrict__ totals) {
    typedef hipcub::BlockScan<uint32_t, 1024> Scan;
    typedef hipcub::BlockReduce<uint32_t, 1024> Red;
    __shared__ typename Scan::TempStorage ts;
    __shared__ typename Red::TempStorage rs;
    __shared__ uint32_t carry_d, carry_r;
    if (threadIdx.x == 0) carry_d = carry_r = 0;
    __syncthreads();
    for (uint32_t base = 0; base < nsend; base += 1024) {
        const uint32_t s = base + threadIdx.x;
        uint32_t rem = 0, del = 0;
        if (s < nsend) {
            uint32_t lo = head[s], hi = send[s];
            const uint32_t h0 = lo;
            while (lo < hi) {   // first index with the height past the cut
                const uint32_t mid = lo + (hi - lo) / 2;
                const bool in = strict ? ph[mid] < h : ph[mid] <= h;
                if (in) lo = mid + 1;
                else hi = mid;
            }
            rem = lo - h0;
            del = allow && allow[s] ? rem : 0u;
            newhead[s] = lo;
        }
        uint32_t o = 0, agg = 0;
        Scan(ts).ExclusiveSum(del, o, agg);
        const uint32_t rsum = Red(rs).Sum(rem);
        if (s < nsend) off[s] = carry_d + o;
        __syncthreads();
        if (threadIdx.x == 0) {
            carry_d += agg;
            carry_r += rsum;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        totals[0] = carry_d;
        totals[1] = carry_r;
    }
}

// the delivered prefixes into the packed stage: block s copies sender s's
// (rows at or past cap are not written: the consume then fails with HD_ECAP)
__global__ __launch_bounds__(256) void k_mq_take(Pool p, const uint32_t* __restrict__ head,
                                                 const uint32_t* __restrict__ newhead, const uint32_t* __restrict__ off,
                                                 const uint8_t* __restrict__ allow, uint32_t cap, Pool d) {
    const uint32_t s = blockIdx.x;
    if (!allow[s]) return;
    const uint32_t lo = head[s], n = newhead[s] - lo, o = off[s];
    for (uint32_t j = threadIdx.x; j < n && o + j < cap; j += blockDim.x) {
        const uint32_t e = lo + j, k = o + j;
        d.sender[k] = p.sender[e];
        d.type[k] = p.type[e];
        d.h[k] = p.h[e];
        d.r[k] = p.r[e];
        d.vr[k] = p.vr[e];
        for (int w = 0; w < 2; w++) {
            reinterpret_cast<uint4*>(d.value + 32 * (size_t)k)[w] = reinterpret_cast<const uint4*>(p.value + 32 * (size_t)e)[w];
            reinterpret_cast<uint4*>(d.from + 32 * (size_t)k)[w] = reinterpret_cast<const uint4*>(p.from + 32 * (size_t)e)[w];
        }
        for (int w = 0; w < 65; w++) d.sig[65 * (size_t)k + w] = p.sig[65 * (size_t)e + w];
    }
}

// the plan's heads become the queue's unless its delivered count exceeds cap
__global__ void k_mq_commit(uint32_t nsend, const uint32_t* __restrict__ newhead, const uint32_t* __restrict__ totals,
                            uint32_t cap, uint32_t* __restrict__ head) {
    if (totals[0] > cap) return;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nsend; s += gridDim.x * blockDim.x) head[s] = newhead[s];
}

// A consume in one launch, for queues of at most 1024 senders (the usual
// case: one queue per validator): procsAllowed flags in LDS (the dict looked
// up for each allowed signatory), the plan (k_mq_plan's cut per sender and the
// scan of the delivered counts), the delivered rows packed into the stage as
// 160-byte records in delivery order (so the host downloads only a prefix),
// and the heads committed when the delivery fits `cap`.  The stage starts
// with a 64-byte header: {delivered, removed}.
#define HD_MQ_ROW 160
#define HD_MQ_HDR 64
__device__ __forceinline__ void mq_row_put(uint8_t* __restrict__ row, const Pool& p, uint32_t e, uint32_t allowed) {
    // whole dwords only (the stage may be mapped host memory: one PCIe write
    // per dword instead of per byte); bytes 152..155 = sig[64], type, allowed
    // (a prefetched row: its sender was in procsAllowed), 0
    uint32_t* o = reinterpret_cast<uint32_t*>(row);
    const uint64_t hv = (uint64_t)p.h[e], rv = (uint64_t)p.r[e], vv = (uint64_t)p.vr[e];
    o[0] = (uint32_t)hv;
    o[1] = (uint32_t)(hv >> 32);
    o[2] = (uint32_t)rv;
    o[3] = (uint32_t)(rv >> 32);
    o[4] = (uint32_t)vv;
    o[5] = (uint32_t)(vv >> 32);
    const uint32_t* val = reinterpret_cast<const uint32_t*>(p.value + 32 * (size_t)e);
    const uint32_t* frm = reinterpret_cast<const uint32_t*>(p.from + 32 * (size_t)e);
    for (int j = 0; j < 8; j++) o[6 + j] = val[j];
    for (int j = 0; j < 8; j++) o[14 + j] = frm[j];
    const uint8_t* sg = p.sig + 65 * (size_t)e;
    for (int j = 0; j < 16; j++)
        o[22 + j] = (uint32_t)sg[4 * j] | ((uint32_t)sg[4 * j + 1] << 8) | ((uint32_t)sg[4 * j + 2] << 16) |
                    ((uint32_t)sg[4 * j + 3] << 24);
    o[38] = (uint32_t)sg[64] | ((uint32_t)p.type[e] << 8) | (allowed << 16);
    o[39] = (uint32_t)p.sender[e];
}
// Prefetch (hpf > h): the same launch also stages every message of the
// heights (h, hpf] -- allowed or not, flagged in byte 154 -- after the
// delivered rows, in queue order, when they fit `pf_rows`; the host then
// serves the consumes of those heights without the device (hd_mq pf_*).  The
// heads are committed through h only.  Header words: {delivered, removed,
// seq, staged window rows, window: 1 staged / 2 over pf_rows / 0 none}.
__global__ __launch_bounds__(1024) void k_mq_consume1(uint32_t nsend, Pool p, uint32_t* __restrict__ head,
                                                      const uint32_t* __restrict__ send, int64_t h, uint32_t na,
                                                      const uint32_t* __restrict__ list, int be_words, Dict d,
                                                      uint32_t rows, uint32_t cap, uint8_t* __restrict__ stage,
                                                      uint32_t seq, int64_t hpf, uint32_t pf_rows,
                                                      uint32_t* __restrict__ win_meta) {
    typedef hipcub::BlockScan<uint32_t, 1024> Scan;
    typedef hipcub::BlockReduce<uint32_t, 1024> Red;
    __shared__ typename Scan::TempStorage ts;
    __shared__ typename Red::TempStorage rs;
    __shared__ uint8_t allow[1024];
    __shared__ uint32_t off[1024], lo_of[1024], off2[1024], cut_of[1024];
    __shared__ uint32_t tot_d, tot_p;
    const uint32_t t = threadIdx.x;
    allow[t] = 0;
    __syncthreads();
    for (uint32_t k = t; k < na; k += 1024) {
        uint32_t w[8];
        for (int j = 0; j < 8; j++) {
            const uint32_t x = list[8 * (size_t)k + j];
            w[j] = be_words ? __builtin_bswap32(x) : x;
        }
        const uint32_t id = dict_find(d, make_uint4(w[0], w[1], w[2], w[3]), make_uint4(w[4], w[5], w[6], w[7]));
        if (id != kEmpty) allow[id] = 1;
    }
    __syncthreads();
    uint32_t rem = 0, del = 0, cut = 0, h0 = 0, pre = 0;
    if (t < nsend) {
        uint32_t lo = head[t], hi = send[t];
        const uint32_t end = hi;
        h0 = lo;
        // a flush per height cuts a few messages off each run's front: look at
        // the first four at once (independent loads), search only past them
        {
            uint32_t c = 0;
            bool past = false;
            HD_UNROLL for (uint32_t j = 0; j < 4; j++) {
                const bool in = lo + j < hi;
                const int64_t hv = in ? p.h[lo + j] : 0;
                const bool le = in && hv <= h;
                c += (!past && le) ? 1u : 0u;
                past = past || !le;
            }
            if (past) hi = lo + c;   // the cut is within the first four
            lo += c;
        }
        while (lo < hi) {   // first index with the height past the cut
            const uint32_t mid = lo + (hi - lo) / 2;
            if (p.h[mid] <= h) lo = mid + 1;
            else hi = mid;
        }
        cut = lo;
        rem = lo - h0;
        del = allow[t] ? rem : 0u;
        if (hpf > h) {   // the window's end, searched past the consume's cut
            hi = end;
            while (lo < hi) {
                const uint32_t mid = lo + (hi - lo) / 2;
                if (p.h[mid] <= hpf) lo = mid + 1;
                else hi = mid;
            }
            pre = lo - cut;
        }
    }
    uint32_t o = 0, agg = 0;
    Scan(ts).ExclusiveSum(del, o, agg);
    const uint32_t rsum = Red(rs).Sum(rem);
    off[t] = t < nsend ? o : agg;       // entries past nsend sort after every row
    lo_of[t] = h0;
    cut_of[t] = cut;
    __syncthreads();                    // the scan storage is reused
    uint32_t o2 = 0, agg2 = 0;
    Scan(ts).ExclusiveSum(pre, o2, agg2);
    off2[t] = t < nsend ? o2 : agg2;
    if (t == 0) {
        const bool staged = hpf > h && agg <= rows && agg <= cap && agg2 <= pf_rows;
        tot_d = agg;
        tot_p = staged ? agg2 : 0u;
        reinterpret_cast<uint32_t*>(stage)[0] = agg;
        reinterpret_cast<uint32_t*>(stage)[1] = rsum;
        reinterpret_cast<uint32_t*>(stage)[3] = tot_p;
        reinterpret_cast<uint32_t*>(stage)[4] = staged ? 1u : (hpf > h && agg2 > pf_rows ? 2u : 0u);
    }
    __syncthreads();
    const uint32_t total = tot_d, nw = total < rows ? total : rows, np = tot_p;
    uint8_t* out = stage + HD_MQ_HDR;
    for (uint32_t k = t; k < nw; k += 1024) {
        // the sender of delivered row k: the last s with off[s] <= k whose run is non-empty
        uint32_t a = 0, b = nsend;      // off is non-decreasing over [0, nsend)
        while (b - a > 1) {
            const uint32_t m = (a + b) / 2;
            if (off[m] <= k) a = m;
            else b = m;
        }
        mq_row_put(out + (size_t)HD_MQ_ROW * k, p, lo_of[a] + (k - off[a]), 1u);
    }
    if (win_meta) {   // the window's rows are written by k_mq_window_rows (many blocks)
        if (t == 0) {
            win_meta[0] = np;
            win_meta[1] = nw;
        }
        if (t < nsend) {
            win_meta[2 + t] = off2[t];
            win_meta[2 + 1024 + t] = cut_of[t];
            win_meta[2 + 2048 + t] = allow[t];
        }
    }
    if (total <= cap && t < nsend) head[t] = cut;
    if (seq || win_meta) {
        // mapped host stage: every row and the header reach host memory
        // before the sequence word the host spins on (written here, or by
        // k_mq_signal after the window's rows)
        __threadfence_system();
        __syncthreads();
        if (seq && t == 0)
            __hip_atomic_store(reinterpret_cast<uint32_t*>(stage) + 2, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The prefetch window's rows (k_mq_consume1's plan in win_meta: count,
// delivered rows before them, and per sender the window's offset, start and
// allow flag), after the delivered rows of the stage; a grid of blocks, so
// the 160-byte rows cross PCIe from many CUs instead of one.  A block builds
// its 256 consecutive rows in LDS and then writes them as one contiguous
// 40 KB range of 16-byte stores (consecutive lanes, consecutive addresses):
// the stage is mapped host memory, and a lane writing its own row dword by
// dword sent every dword as its own PCIe write.
__global__ __launch_bounds__(256) void k_mq_window_rows(uint32_t nsend, Pool p, const uint32_t* __restrict__ win_meta,
                                                        uint8_t* __restrict__ stage) {
    __shared__ uint32_t o2[1024], co[1024], al[1024];
    __shared__ uint4 rows_lds[256 * HD_MQ_ROW / 16];
    const uint32_t np = win_meta[0], nw = win_meta[1];
    if (np == 0) return;
    for (uint32_t t = threadIdx.x; t < nsend; t += blockDim.x) {
        o2[t] = win_meta[2 + t];
        co[t] = win_meta[2 + 1024 + t];
        al[t] = win_meta[2 + 2048 + t];
    }
    __syncthreads();
    // 64 + 160 nw: 16-byte aligned in the (page-aligned) stage
    uint4* win = reinterpret_cast<uint4*>(stage + HD_MQ_HDR + (size_t)HD_MQ_ROW * nw);
    constexpr uint32_t Q = HD_MQ_ROW / 16;   // 16-byte words per row
    for (uint32_t base = blockIdx.x * 256u; base < np; base += gridDim.x * 256u) {
        const uint32_t k = base + threadIdx.x;
        if (k < np) {
            uint32_t a = 0, b = nsend;
            while (b - a > 1) {
                const uint32_t m = (a + b) / 2;
                if (o2[m] <= k) a = m;
                else b = m;
            }
            mq_row_put(reinterpret_cast<uint8_t*>(rows_lds + Q * threadIdx.x), p, co[a] + (k - o2[a]), al[a]);
        }
        __syncthreads();
        const uint32_t nq = Q * min(256u, np - base);
        uint4* dst = win + (size_t)Q * base;
        for (uint32_t i = threadIdx.x; i < nq; i += 256u) dst[i] = rows_lds[i];
        __syncthreads();
    }
    __threadfence_system();
}

// the mapped stage's sequence word, after every row of the consume (stream order)
__global__ void k_mq_signal(uint8_t* __restrict__ stage, uint32_t seq) {
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(reinterpret_cast<uint32_t*>(stage) + 2, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// live pool entries (not in a consumed / dropped prefix)
__global__ void k_mq_live(uint32_t M, const int32_t* __restrict__ snd, const uint32_t* __restrict__ head,
                          uint8_t* __restrict__ keep) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < M) keep[e] = e >= head[snd[e]];
}

// min and max of the three sort keys in one pass: out[0..4] = min of
// (rk, ~rk, hk, ~hk, ~sk) in the order-preserving unsigned form (signed x ->
// x ^ 2^63), all initialised to ~0; max(x) = ~min(~x)
__device__ __forceinline__ uint64_t mq_ord(int64_t x) { return (uint64_t)x ^ 0x8000000000000000ull; }
__global__ __launch_bounds__(256) void k_mq_minmax3(uint32_t T, const int64_t* __restrict__ rk,
                                                   const int64_t* __restrict__ hk, const uint32_t* __restrict__ sk,
                                                   unsigned long long* __restrict__ out) {
    uint64_t m[5] = {~0ull, ~0ull, ~0ull, ~0ull, ~0ull};
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < T; e += gridDim.x * blockDim.x) {
        const uint64_t r = mq_ord(rk[e]), hh = mq_ord(hk[e]), ss = ~(uint64_t)sk[e];
        m[0] = r < m[0] ? r : m[0];
        m[1] = ~r < m[1] ? ~r : m[1];
        m[2] = hh < m[2] ? hh : m[2];
        m[3] = ~hh < m[3] ? ~hh : m[3];
        m[4] = ss < m[4] ? ss : m[4];
    }
    // wavefront, then block minima; one atomic per block and field
    __shared__ uint64_t part[4][5];
    for (int k = 0; k < 5; k++) {
        uint64_t x = m[k];
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t y = __shfl_xor(x, o);
            x = y < x ? y : x;
        }
        if ((threadIdx.x & 63u) == 0) part[threadIdx.x >> 6][k] = x;
    }
    __syncthreads();
    if (threadIdx.x < 5) {
        uint64_t x = part[0][threadIdx.x];
        for (int w = 1; w < 4; w++) x = part[w][threadIdx.x] < x ? part[w][threadIdx.x] : x;
        atomicMin(out + threadIdx.x, (unsigned long long)x);
    }
}

// Stable select of the set flags' indices in two dependent launches: block
// b counts the flags of its 4,096-element tile; then block b sums the counts
// of the tiles before it, scans its own tile and writes the indices in
// order, and the last block writes the total.  rocprim's select takes four
// launches (a fill, a look-back init, the partition and a transform), each
// at the ~5 us floor of a dependent launch in the insert's trace.
#define HD_SEL_TILE 4096u        // 256 threads x 16 flags (one 16-byte load)
#define HD_SEL_MAX_TILES 1024u   // larger inputs take rocprim's select
__device__ __forceinline__ uint32_t sel_load16(const uint8_t* __restrict__ flag, uint32_t n, uint32_t i0) {
    // bit j = flag[i0 + j] != 0, for the indices below n
    uint32_t m = 0;
    if (i0 + 16 <= n) {
        const uint4 v = *reinterpret_cast<const uint4*>(flag + i0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        for (int q = 0; q < 4; q++)
            for (int b = 0; b < 4; b++) m |= (uint32_t)(((w[q] >> (8 * b)) & 0xFFu) != 0) << (4 * q + b);
    } else {
        for (uint32_t j = 0; j < 16; j++) m |= (uint32_t)(i0 + j < n && flag[i0 + j] != 0) << j;
    }
    return m;
}
__global__ __launch_bounds__(256) void k_sel_count(uint32_t n, const uint8_t* __restrict__ flag,
                                                   uint32_t* __restrict__ tile_count) {
    typedef hipcub::BlockReduce<uint32_t, 256> Red;
    __shared__ typename Red::TempStorage tmp;
    const uint32_t c = __popc(sel_load16(flag, n, blockIdx.x * HD_SEL_TILE + 16 * threadIdx.x));
    const uint32_t sum = Red(tmp).Sum(c);
    if (threadIdx.x == 0) tile_count[blockIdx.x] = sum;
}
__global__ __launch_bounds__(256) void k_sel_scatter(uint32_t n, const uint8_t* __restrict__ flag,
                                                     const uint32_t* __restrict__ tile_count,
                                                     uint32_t* __restrict__ out, uint32_t* __restrict__ count) {
    typedef hipcub::BlockReduce<uint32_t, 256> Red;
    typedef hipcub::BlockScan<uint32_t, 256> Scan;
    __shared__ union {
        typename Red::TempStorage red;
        typename Scan::TempStorage scan;
    } tmp;
    __shared__ uint32_t base_s;
    uint32_t pre = 0;
    for (uint32_t j = threadIdx.x; j < blockIdx.x; j += 256u) pre += tile_count[j];
    pre = Red(tmp.red).Sum(pre);
    if (threadIdx.x == 0) base_s = pre;
    __syncthreads();
    const uint32_t base = base_s;
    const uint32_t i0 = blockIdx.x * HD_SEL_TILE + 16 * threadIdx.x;
    uint32_t m = sel_load16(flag, n, i0);
    uint32_t off, tot;
    Scan(tmp.scan).ExclusiveSum((uint32_t)__popc(m), off, tot);
    uint32_t o = base + off;
    while (m) {
        const uint32_t j = __ffs(m) - 1;
        out[o++] = i0 + j;
        m &= m - 1;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *count = base + tot;
}

inline uint32_t nblk(uint32_t n) { return (n + 255) / 256; }

int bits_of(uint64_t range) {
    int b = 0;
    while (b < 64 && (range >> b)) b++;
    return b;
}

}  // namespace

enum MqSlot { MQ_FLAG, MQ_NEWIDX, MQ_NSEL, MQ_HK, MQ_RK, MQ_SK, MQ_PERM0, MQ_PERM1, MQ_K64A, MQ_K64B, MQ_K32A, MQ_K32B,
              MQ_HEAD, MQ_KEEP, MQ_SEL, MQ_RED, MQ_TMP, MQ_SID, MQ_LSLOT, MQ_LCLAIM, MQ_LID, MQ_REPS, MQ_ALLOW,
              MQ_LIST, MQ_DELIV, MQ_SEL2, MQ_HEADS, MQ_SEND, MQ_NEWHEAD, MQ_OFF, MQ_TOT, MQ_STAGE, MQ_WIN, MQ_SELCNT, MQ__N };

struct hd_mq {
    hd_ctx* ctx = nullptr;
    // an insert failed after it had started changing the queue's device state
    // (new senders interned, the pool swapped): the host's view (pool.n,
    // nsend) may no longer match it, so every later call is refused
    bool failed = false;
    // an insert on a caller's stream waits for the context stream's queue
    // work (a drop's or consume's head commits are queued there unsynchronised)
    hipEvent_t order_ev = nullptr;
    uint32_t max_cap = 1000;
    Pool pool, spare;
    DevBuf buf[MQ__N];
    // sender dictionary
    uint32_t nsend = 0;
    uint32_t* keys = nullptr;   // kcap x 8 words
    size_t kcap_bytes = 0;
    uint32_t* slots = nullptr;  // tcap ids
    uint32_t tcap = 0;
    uint64_t seed = 0;
    // live messages; consumed / dropped prefixes not yet compacted away
    uint64_t live = 0;
    bool dead = false;
    uint32_t runs_for = 0;      // senders the head / send arrays hold
    // pinned host stage of consume (the packed outputs + the plan totals)
    void* hstage = nullptr;
    size_t hstage_cap = 0;
    uint32_t last_deliv = 0;    // the previous consume's delivery: sizes the next one's first download
    // mapped (device-written) host stage of the fused consume: no download,
    // the host spins on a sequence word (HD_MQ_MAPPED=0: the download path)
    void* mstage = nullptr;
    uint8_t* mstage_dev = nullptr;
    size_t mstage_cap = 0;
    uint32_t seq = 0;
    bool mapped = true;
    // mapped reply block of the insert's host round trips (mq_reply): word 0
    // is the sequence word, the values follow
    uint32_t* rep = nullptr;
    uint32_t* rep_dev = nullptr;
    uint32_t rep_seq = 0;
    // Consume prefetch (mapped path): a consume of height h also stages the
    // rows of the heights (h, h + pf_win] (k_mq_consume1); while nothing is
    // inserted, the admitted set stays and the consumes stay inside that
    // window, they are served from the stage by the host alone.  The device
    // heads stay at pf_dev until pf_sync commits them through pf_done.
    bool pf = false;
    int64_t pf_dev = 0;        // heads committed on the device through this height
    int64_t pf_done = 0;       // consumed (or dropped) through this height
    int64_t pf_max = 0;        // the staged window ends here
    uint32_t pf_adm_ver = 0;   // the admitted set the allow flags were read against
    int pf_win = 64;           // window heights (halved when a window overflows the stage)
    const uint8_t* pf_base = nullptr;     // first window row in the stage
    std::vector<uint32_t> pf_start;       // rows of height pf_dev + 1 + j: pf_idx[pf_start[j] .. pf_start[j + 1])
    std::vector<uint32_t> pf_idx;
};

#define QCHK(expr, what)                                           \
    do {                                                           \
        hipError_t _e = (expr);                                    \
        if (_e != hipSuccess) return hd_ctx_fail(q->ctx, _e, what); \
    } while (0)

static void* qbuf(hd_mq* q, int slot, size_t bytes, int* rc) {
    DevBuf& b = q->buf[slot];
    int r = hd_dev_grow(q->ctx, &b.p, &b.cap, std::max<size_t>(bytes, 64));
    if (r) {
        *rc = r;
        return nullptr;
    }
    return b.p;
}

static Dict dict_of(const hd_mq* q) { return Dict{q->keys, q->slots, q->tcap - 1, q->seed}; }

// select-flagged over [0, n) -> out indices, returns count (synchronises)
// Indices of the set flags, in order.  The count lands in *count after a
// stream sync when wait is set; with wait unset it is only queued (the caller
// syncs before reading it), and with count == nullptr it is not downloaded
// (a caller that knows it).  Counts queued together use different slots.
// The insert's host round trips (the insertable count; the key ranges with
// the new senders; the kept count).  One thread per word copies device words
// into the mapped reply block, then the sequence word follows (system fence,
// release store), and the host spins on it.  In the C5 insert trace each
// round trip through a download into host memory and hipStreamSynchronize
// left the stream idle ~40 us (the copy, the host's wake-up, the next launch).
#define HD_MQ_REPLY_WORDS 16
struct ReplySrc {
    const uint32_t* p[HD_MQ_REPLY_WORDS];
    uint32_t n;
};
__global__ void k_mq_reply(ReplySrc src, uint32_t* __restrict__ rep, uint32_t seq) {
    const uint32_t t = threadIdx.x;
    const uint32_t* w = nullptr;
#pragma unroll
    for (uint32_t k = 0; k < HD_MQ_REPLY_WORDS; k++)
        if (t == k) w = src.p[k];
    // the words were written by earlier kernels of this stream, some by
    // device-scope atomics (the key ranges): plain loads see them -- the
    // kernel boundary orders them (scripts/visibility_probe.hip: 20 rounds x
    // 2,048 reader blocks on all 8 XCDs after atomics from 8,192 blocks, 0
    // stale words; profiles/round6/visibility_probe.log)
    if (t < src.n) rep[1 + t] = *w;
    __threadfence_system();
    __syncthreads();
    if (t == 0) __hip_atomic_store(rep, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Queue the reply of n device words (stream order) and wait for it; out[k] =
// *words[k].  Past ~0.2 s the stream is synchronised (a fault surfaces there).
static int mq_reply(hd_mq* q, hipStream_t s, const uint32_t* const* words, uint32_t n, uint32_t* out) {
    if (!q->rep) {
        void* h = nullptr;
        QCHK(hipHostMalloc(&h, 4 * (1 + HD_MQ_REPLY_WORDS) + 64, hipHostMallocMapped | hipHostMallocCoherent),
             "mq reply block");
        q->rep = (uint32_t*)h;
        void* d = nullptr;
        QCHK(hipHostGetDevicePointer(&d, h, 0), "mq reply pointer");
        q->rep_dev = (uint32_t*)d;
        q->rep[0] = 0;
    }
    ReplySrc src{};
    for (uint32_t k = 0; k < n; k++) src.p[k] = words[k];
    src.n = n;
    const uint32_t seq = ++q->rep_seq ? q->rep_seq : ++q->rep_seq;   // never 0
    k_mq_reply<<<1, 64, 0, s>>>(src, q->rep_dev, seq);
    QCHK(hipGetLastError(), "k_mq_reply");
    volatile uint32_t* word = q->rep;
    const auto t0 = std::chrono::steady_clock::now();
    while (*word != seq) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
            QCHK(hipStreamSynchronize(s), "mq reply sync");
            if (*word != seq) return hd_ctx_fail(q->ctx, hipErrorUnknown, "mq reply signal");
            break;
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    for (uint32_t k = 0; k < n; k++) out[k] = ((volatile uint32_t*)q->rep)[1 + k];
    return HD_OK;
}

static int select_idx(hd_mq* q, const uint8_t* flag, uint32_t n, uint32_t* out, uint32_t* count, hipStream_t s,
                      int slot = 0, bool wait = true, uint32_t** count_dev = nullptr) {
    int rc = 0;
    uint32_t* nsel = (uint32_t*)qbuf(q, MQ_NSEL, 64, &rc);
    if (rc) return rc;
    nsel += slot;
    if (count_dev) *count_dev = nsel;
    const uint32_t tiles = std::max((n + HD_SEL_TILE - 1) / HD_SEL_TILE, 1u);
    if (tiles <= HD_SEL_MAX_TILES && ((uintptr_t)flag & 15) == 0) {
        uint32_t* tc = (uint32_t*)qbuf(q, MQ_SELCNT, 4 * (size_t)HD_SEL_MAX_TILES, &rc);
        if (rc) return rc;
        k_sel_count<<<tiles, 256, 0, s>>>(n, flag, tc);
        k_sel_scatter<<<tiles, 256, 0, s>>>(n, flag, tc, out, nsel);
        QCHK(hipGetLastError(), "select");
    } else {
        hipcub::CountingInputIterator<uint32_t> iota(0);
        size_t need = 0;
        QCHK(hipcub::DeviceSelect::Flagged(nullptr, need, iota, flag, out, nsel, n, s), "select size");
        void* tmp = qbuf(q, MQ_TMP, need, &rc);
        if (rc) return rc;
        QCHK(hipcub::DeviceSelect::Flagged(tmp, need, iota, flag, out, nsel, n, s), "select");
    }
    if (count && wait) {
        const uint32_t* w[1] = {nsel};
        return mq_reply(q, s, w, 1, count);
    }
    if (count) QCHK(hipMemcpyAsync(count, nsel, 4, hipMemcpyDeviceToHost, s), "select count");
    return HD_OK;
}

// min / max of the three sort keys (k_mq_minmax3) into the device words
// red[0..4] (set to ~0 by k_mq_keys, the launch before); key_ranges_read
// brings them back with counts queued meanwhile
static int key_ranges_launch(hd_mq* q, uint32_t T, const int64_t* rk, const int64_t* hk, const uint32_t* sk,
                             hipStream_t s, unsigned long long* red) {
    const uint32_t blocks = std::min(nblk(T), 256u);
    k_mq_minmax3<<<blocks, 256, 0, s>>>(T, rk, hk, sk, red);
    QCHK(hipGetLastError(), "k_mq_minmax3");
    return HD_OK;
}

// the key ranges and n_extra device counts queued earlier (the new senders,
// the prefilter's survivors) in one round trip
static int key_ranges_read(hd_mq* q, const unsigned long long* red, hipStream_t s, int64_t* rmn, int64_t* rmx,
                           int64_t* hmn, int64_t* hmx, uint32_t* smx, const uint32_t* const* extra_dev,
                           uint32_t n_extra, uint32_t* extra) {
    // the five 64-bit reductions as ten words, then the counts
    const uint32_t* w[HD_MQ_REPLY_WORDS];
    for (int k = 0; k < 10; k++) w[k] = (const uint32_t*)red + k;
    for (uint32_t k = 0; k < n_extra; k++) w[10 + k] = extra_dev[k];
    uint32_t got[HD_MQ_REPLY_WORDS];
    const int rc = mq_reply(q, s, w, 10 + n_extra, got);
    if (rc) return rc;
    uint64_t host[5];
    memcpy(host, got, sizeof(host));
    for (uint32_t k = 0; k < n_extra; k++) extra[k] = got[10 + k];
    const uint64_t sign = 0x8000000000000000ull;
    *rmn = (int64_t)(host[0] ^ sign);
    *rmx = (int64_t)(~host[1] ^ sign);
    *hmn = (int64_t)(host[2] ^ sign);
    *hmx = (int64_t)(~host[3] ^ sign);
    *smx = (uint32_t)~host[4];
    return HD_OK;
}

// Stable radix sort of (key, perm) pairs on bits [0, bits) of the key.
// rocprim's default dispatch takes its merge-sort path up to 2^20 items, and
// that path ignores the bit range: ~10 block-merge rounds of two kernels each
// (~210 us for a C5 insert of 855k pairs).  A merge-sort limit of 0 sends
// every size above one block to the onesweep path, which sorts only the
// digits the range covers (a 20-bit (sender, height, round) key: 3 passes).
typedef rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>
    OnesweepSort;
template <class K>
static hipError_t sort_pairs_bits(void* tmp, size_t& need, hipcub::DoubleBuffer<K>& keys,
                                  hipcub::DoubleBuffer<uint32_t>& perm, uint32_t n, int bits, hipStream_t s) {
    rocprim::double_buffer<K> k(keys.Current(), keys.Alternate());
    rocprim::double_buffer<uint32_t> v(perm.Current(), perm.Alternate());
    const hipError_t e = rocprim::radix_sort_pairs<OnesweepSort>(tmp, need, k, v, n, 0u, (unsigned)bits, s);
    if (tmp && e == hipSuccess) {
        if (k.current() != keys.Current()) keys.selector ^= 1;
        if (v.current() != perm.Current()) perm.selector ^= 1;
    }
    return e;
}

// stable sort of perm (DoubleBuffer) by a 64-bit field rebased to its min
static int sort_pass64(hd_mq* q, hipcub::DoubleBuffer<uint32_t>& perm, const int64_t* field, uint32_t T, hipStream_t s,
                       int64_t mn, int64_t mx) {
    int rc = 0;
    const int bits = bits_of((uint64_t)mx - (uint64_t)mn);
    if (bits == 0) return HD_OK;
    uint64_t* ka = (uint64_t*)qbuf(q, MQ_K64A, 8 * (size_t)T, &rc);
    uint64_t* kb = (uint64_t*)qbuf(q, MQ_K64B, 8 * (size_t)T, &rc);
    if (rc) return rc;
    k_mq_rekey64<<<nblk(T), 256, 0, s>>>(T, perm.Current(), field, mn, ka);
    hipcub::DoubleBuffer<uint64_t> keys(ka, kb);
    size_t need = 0;
    QCHK(sort_pairs_bits(nullptr, need, keys, perm, T, bits, s), "sort size");
    void* tmp = qbuf(q, MQ_TMP, need, &rc);
    if (rc) return rc;
    QCHK(sort_pairs_bits(tmp, need, keys, perm, T, bits, s), "sort 64");
    return HD_OK;
}

static int sort_pass32(hd_mq* q, hipcub::DoubleBuffer<uint32_t>& perm, const uint32_t* field, uint32_t T,
                       hipStream_t s, uint32_t mx) {
    int rc = 0;
    const int bits = bits_of(mx);
    if (bits == 0) return HD_OK;
    uint32_t* ka = (uint32_t*)qbuf(q, MQ_K32A, 4 * (size_t)T, &rc);
    uint32_t* kb = (uint32_t*)qbuf(q, MQ_K32B, 4 * (size_t)T, &rc);
    if (rc) return rc;
    k_mq_rekey32<<<nblk(T), 256, 0, s>>>(T, perm.Current(), field, ka);
    hipcub::DoubleBuffer<uint32_t> keys(ka, kb);
    size_t need = 0;
    QCHK(sort_pairs_bits(nullptr, need, keys, perm, T, bits, s), "sort size");
    void* tmp = qbuf(q, MQ_TMP, need, &rc);
    if (rc) return rc;
    QCHK(sort_pairs_bits(tmp, need, keys, perm, T, bits, s), "sort 32");
    return HD_OK;
}

// keep the pool elements whose flag is set, in order
// Keep the pool entries whose keep flag is set; `kept` = their number when
// the caller knows it (saves the count download), else -1.
static int pool_filter(hd_mq* q, const uint8_t* keep, hipStream_t s, int64_t kept = -1) {
    int rc = 0;
    const uint32_t M = q->pool.n;
    uint32_t* sel = (uint32_t*)qbuf(q, MQ_SEL, 4 * (size_t)M, &rc);
    if (rc) return rc;
    uint32_t n = kept >= 0 ? (uint32_t)kept : 0;
    rc = select_idx(q, keep, M, sel, kept >= 0 ? nullptr : &n, s, 2);
    if (rc) return rc;
    rc = pool_reserve(q->ctx, q->spare, std::max(n, 1u));
    if (rc) return rc;
    MqSrc src{q->pool, DevBatch{}, nullptr, nullptr, M};
    if (n) k_mq_gather<<<nblk(n), 256, 0, s>>>(src, n, sel, q->spare);
    QCHK(hipGetLastError(), "mq gather");
    std::swap(q->pool, q->spare);
    q->pool.n = n;
    return HD_OK;
}

// the hash table holds at least 2 (nsend + more) slots (load <= 1/2)
static int dict_reserve(hd_mq* q, uint32_t more, hipStream_t s) {
    const uint64_t want = 2 * ((uint64_t)q->nsend + more);
    if (want > (1ull << 31)) return HD_EINVAL;
    if (q->tcap >= want && q->slots) return HD_OK;
    uint32_t cap = std::max<uint32_t>(q->tcap, 1024u);
    while (cap < want) cap <<= 1;
    uint32_t* slots = nullptr;
    QCHK(hipMalloc(&slots, 4 * (size_t)cap), "hipMalloc mq senders");
    QCHK(hipMemsetAsync(slots, 0xFF, 4 * (size_t)cap, s), "clear mq senders");
    if (q->nsend) k_mq_rehash<<<nblk(q->nsend), 256, 0, s>>>(q->nsend, q->keys, slots, cap - 1, q->seed);
    QCHK(hipGetLastError(), "mq rehash");
    QCHK(hipStreamSynchronize(s), "mq rehash sync");
    if (q->slots) (void)hipFree(q->slots);
    q->slots = slots;
    q->tcap = cap;
    return HD_OK;
}

// interned key storage for `n` senders (contents kept)
static int keys_reserve(hd_mq* q, uint32_t n, hipStream_t s) {
    const size_t need = 32 * (size_t)std::max(n, 1u);
    if (need <= q->kcap_bytes) return HD_OK;
    const size_t cap = std::max(need, 2 * q->kcap_bytes);
    uint32_t* k = nullptr;
    QCHK(hipMalloc(&k, cap), "hipMalloc mq keys");
    if (q->nsend) QCHK(hipMemcpyAsync(k, q->keys, 32 * (size_t)q->nsend, hipMemcpyDeviceToDevice, s), "mq keys copy");
    QCHK(hipStreamSynchronize(s), "mq keys sync");
    if (q->keys) (void)hipFree(q->keys);
    q->keys = k;
    q->kcap_bytes = cap;
    return HD_OK;
}

// sender ids of the m insertable messages (newidx), interning new Froms in
// batch order
// Sender ids of the m insertable messages (newidx), interning new Froms in
// batch order.  The number of new senders stays on the device (*r_dev): the
// caller reads it with its next download and then adds it to q->nsend (the
// ids and keys are written for it here, with room for m new senders).
static int intern_senders(hd_mq* q, const hd_batch* b, const uint32_t* newidx, uint32_t m, uint32_t** sid_out,
                          uint32_t** r_dev, hipStream_t s) {
    int rc = dict_reserve(q, m, s);
    if (rc) return rc;
    uint32_t lcap = 1024;
    while (lcap < 2 * m) lcap <<= 1;
    uint32_t* sid = (uint32_t*)qbuf(q, MQ_SID, 4 * (size_t)m, &rc);
    uint32_t* lslot = (uint32_t*)qbuf(q, MQ_LSLOT, 4 * (size_t)m, &rc);
    uint32_t* lclaim = (uint32_t*)qbuf(q, MQ_LCLAIM, 4 * (size_t)lcap, &rc);
    uint32_t* lid = (uint32_t*)qbuf(q, MQ_LID, 4 * (size_t)lcap, &rc);
    uint8_t* nflag = (uint8_t*)qbuf(q, MQ_KEEP, m, &rc);
    uint32_t* reps = (uint32_t*)qbuf(q, MQ_REPS, 4 * (size_t)m, &rc);
    if (rc) return rc;
    QCHK(hipMemsetAsync(lclaim, 0xFF, 4 * (size_t)lcap, s), "clear batch senders");
    k_mq_lookup<<<nblk(m), 256, 0, s>>>(m, newidx, b->from32, dict_of(q), lclaim, lcap - 1, sid, lslot);
    k_mq_newflag<<<nblk(m), 256, 0, s>>>(m, lslot, lclaim, nflag);
    QCHK(hipGetLastError(), "mq lookup");
    rc = select_idx(q, nflag, m, reps, nullptr, s, 1, false, r_dev);
    if (rc) return rc;
    rc = keys_reserve(q, q->nsend + m, s);
    if (rc) return rc;
    k_mq_assign<<<nblk(m), 256, 0, s>>>(*r_dev, reps, newidx, b->from32, q->nsend, q->keys, q->slots, q->tcap - 1,
                                        q->seed, lslot, lid);
    k_mq_sid<<<nblk(m), 256, 0, s>>>(m, lslot, lid, sid);
    QCHK(hipGetLastError(), "mq assign");
    *sid_out = sid;
    return HD_OK;
}

// drop the consumed prefixes from the pool (the live count is known)
static int mq_compact(hd_mq* q, hipStream_t s) {
    if (!q->dead) return HD_OK;
    const uint32_t M = q->pool.n;
    int rc = 0;
    uint8_t* keep = (uint8_t*)qbuf(q, MQ_KEEP, M, &rc);
    if (rc) return rc;
    k_mq_live<<<nblk(M), 256, 0, s>>>(M, q->pool.sender, (const uint32_t*)q->buf[MQ_HEADS].p, keep);
    QCHK(hipGetLastError(), "k_mq_live");
    rc = pool_filter(q, keep, s, (int64_t)q->live);
    if (rc) return rc;
    q->dead = false;
    return HD_OK;
}

// per-sender runs of the (freshly sorted, compact) pool
// (n_dev: the pool's size is still on the device, at most q->pool.n)
// (head / send: the MQ_HEADS / MQ_SEND buffers of ns entries, already
// cleared in stream order by k_mq_compose)
static int mq_runs(hd_mq* q, hipStream_t s, const uint32_t* n_dev) {
    uint32_t* head = (uint32_t*)q->buf[MQ_HEADS].p;
    uint32_t* send = (uint32_t*)q->buf[MQ_SEND].p;
    if (q->pool.n) k_mq_runs<<<nblk(q->pool.n), 256, 0, s>>>(q->pool.n, q->pool.sender, head, send, n_dev);
    QCHK(hipGetLastError(), "k_mq_runs");
    q->runs_for = q->nsend;
    q->live = q->pool.n;
    q->dead = false;
    return HD_OK;
}

static int pf_sync(hd_mq* q);   // the consume prefetch (below)

static int mq_insert_flagged_impl(hd_mq* q, const hd_batch* d_batch, const uint8_t* flag, hipStream_t s,
                                  bool* dirty);

// An insert that fails once it has begun to change the device state (new
// senders interned into the dictionary, the pool swapped) leaves the host's
// view of the queue (pool.n, nsend) out of step with it: the queue is then
// marked failed and refuses every later call.
static int mq_insert_flagged(hd_mq* q, const hd_batch* d_batch, const uint8_t* flag, hipStream_t s) {
    bool dirty = false;
    const int rc = mq_insert_flagged_impl(q, d_batch, flag, s, &dirty);
    if (rc && dirty) {
        q->failed = true;
        q->ctx->last_error += " (message queue state lost: the queue refuses further calls)";
    }
    return rc;
}

static int mq_insert_flagged_impl(hd_mq* q, const hd_batch* d_batch, const uint8_t* flag, hipStream_t s,
                                  bool* dirty) {
    const uint32_t nb = d_batch->n;
    int rc = mq_compact(q, s);
    if (rc) return rc;
    // 1. the batch's insertable messages, in batch order
    uint32_t* newidx = (uint32_t*)qbuf(q, MQ_NEWIDX, 4 * (size_t)nb, &rc);
    if (rc) return rc;
    uint32_t m = 0;
    rc = select_idx(q, flag, nb, newidx, &m, s);
    if (rc || m == 0) return rc;
    // 2. their sender queues (the From of each message)
    uint32_t* nsid = nullptr;
    uint32_t* r_dev = nullptr;   // new senders: read with the key ranges below
    *dirty = true;
    rc = intern_senders(q, d_batch, newidx, m, &nsid, &r_dev, s);
    if (rc) return rc;
    // 3. merged sequence: pool (sorted) then the new messages (arrival order)
    const uint32_t M = q->pool.n, T = M + m;
    DevBatch b{nb, d_batch->type, d_batch->height, d_batch->round, d_batch->valid_round, d_batch->value32,
               d_batch->from32, d_batch->sig65};
    MqSrc src{q->pool, b, newidx, nsid, M};
    int64_t* hk = (int64_t*)qbuf(q, MQ_HK, 8 * (size_t)T, &rc);
    int64_t* rk = (int64_t*)qbuf(q, MQ_RK, 8 * (size_t)T, &rc);
    uint32_t* sk = (uint32_t*)qbuf(q, MQ_SK, 4 * (size_t)T, &rc);
    uint32_t* p0 = (uint32_t*)qbuf(q, MQ_PERM0, 4 * (size_t)T, &rc);
    uint32_t* p1 = (uint32_t*)qbuf(q, MQ_PERM1, 4 * (size_t)T, &rc);
    if (rc) return rc;
    unsigned long long* red = (unsigned long long*)qbuf(q, MQ_RED, 5 * sizeof(uint64_t), &rc);
    if (rc) return rc;
    k_mq_keys<<<nblk(T), 256, 0, s>>>(src, T, hk, rk, sk, p0, red);
    // 4. stable LSD passes: round, height, sender (mq.go:120-128 order; the
    //    stability keeps arrival order among equal keys)
    //    (the three keys' ranges and the new senders in one host round trip)
    if ((rc = key_ranges_launch(q, T, rk, hk, sk, s, red))) return rc;
    int64_t rmn, rmx, hmn, hmx;
    uint32_t smx, r = 0;
    if ((rc = key_ranges_read(q, red, s, &rmn, &rmx, &hmn, &hmx, &smx, &r_dev, 1, &r))) return rc;
    q->nsend += r;
    hipcub::DoubleBuffer<uint32_t> perm(p0, p1);
    const int rb = bits_of((uint64_t)rmx - (uint64_t)rmn), hb = bits_of((uint64_t)hmx - (uint64_t)hmn),
              sb = bits_of(smx);
    if (rb + hb + sb <= 64) {
        // one radix sort over the packed key (usually ~25 bits: 3-4 digit
        // passes instead of three sorts' worth)
        if (rb + hb + sb > 0) {
            uint64_t* ka = (uint64_t*)qbuf(q, MQ_K64A, 8 * (size_t)T, &rc);
            uint64_t* kb = (uint64_t*)qbuf(q, MQ_K64B, 8 * (size_t)T, &rc);
            if (rc) return rc;
            k_mq_combine<<<nblk(T), 256, 0, s>>>(T, rk, hk, sk, rmn, hmn, rb, hb, ka);
            hipcub::DoubleBuffer<uint64_t> keys(ka, kb);
            size_t need = 0;
            QCHK(sort_pairs_bits(nullptr, need, keys, perm, T, rb + hb + sb, s), "sort size");
            void* tmp = qbuf(q, MQ_TMP, need, &rc);
            if (rc) return rc;
            QCHK(sort_pairs_bits(tmp, need, keys, perm, T, rb + hb + sb, s), "sort keys");
        }
    } else {
        if ((rc = sort_pass64(q, perm, rk, T, s, rmn, rmx))) return rc;
        if ((rc = sort_pass64(q, perm, hk, T, s, hmn, hmx))) return rc;
        if ((rc = sort_pass32(q, perm, sk, T, s, smx))) return rc;
    }
    // 5. per-sender capacity: keep the first max_cap of every sender run
    uint32_t* head = (uint32_t*)qbuf(q, MQ_HEAD, 4 * (size_t)T, &rc);
    uint8_t* keep = (uint8_t*)qbuf(q, MQ_KEEP, T, &rc);
    uint32_t* sel = (uint32_t*)qbuf(q, MQ_SEL, 4 * (size_t)T, &rc);
    if (rc) return rc;
    k_mq_heads<<<nblk(T), 256, 0, s>>>(T, perm.Current(), sk, head);
    {
        size_t need = 0;
        QCHK(hipcub::DeviceScan::InclusiveScan(nullptr, need, head, head, hipcub::Max(), T, s), "scan size");
        void* tmp = qbuf(q, MQ_TMP, need, &rc);
        if (rc) return rc;
        QCHK(hipcub::DeviceScan::InclusiveScan(tmp, need, head, head, hipcub::Max(), T, s), "scan heads");
    }
    k_mq_keep<<<nblk(T), 256, 0, s>>>(T, head, q->max_cap, keep);
    // the kept count stays on the device: compose, gather and the runs cover
    // T entries and stop at it; it comes back with the final synchronisation
    uint32_t* kept_dev = nullptr;
    rc = select_idx(q, keep, T, sel, nullptr, s, 3, false, &kept_dev);
    if (rc) return rc;
    // sel holds kept positions in sorted order -> element ids -> new pool
    uint32_t* ids = head;  // head is consumed by k_mq_keep; reuse its space
    const uint32_t ns = std::max(q->nsend, 1u);
    uint32_t* heads = (uint32_t*)qbuf(q, MQ_HEADS, 4 * (size_t)ns, &rc);
    uint32_t* sends = (uint32_t*)qbuf(q, MQ_SEND, 4 * (size_t)ns, &rc);
    if (rc) return rc;
    k_mq_compose<<<nblk(T), 256, 0, s>>>(T, perm.Current(), sel, ids, kept_dev, ns, heads, sends);
    rc = pool_reserve(q->ctx, q->spare, std::max(T, 1u));
    if (rc) return rc;
    k_mq_gather<<<nblk(T), 256, 0, s>>>(src, T, ids, q->spare, kept_dev);
    QCHK(hipGetLastError(), "mq insert kernels");
    std::swap(q->pool, q->spare);
    q->pool.n = T;   // an upper bound until the count arrives
    rc = mq_runs(q, s, kept_dev);
    if (rc) return rc;
    uint32_t kept = 0;
    const uint32_t* w[1] = {kept_dev};
    if ((rc = mq_reply(q, s, w, 1, &kept))) return rc;
    q->pool.n = kept;
    q->live = q->pool.n;
    return HD_OK;
}

// stream s (an insert's) ordered after everything queued on the context's
// stream so far
static int mq_order_after_ctx(hd_mq* q, hipStream_t s) {
    if (s == q->ctx->stream) return HD_OK;
    if (!q->order_ev) QCHK(hipEventCreateWithFlags(&q->order_ev, hipEventDisableTiming), "mq order event");
    QCHK(hipEventRecord(q->order_ev, q->ctx->stream), "mq order record");
    QCHK(hipStreamWaitEvent(s, q->order_ev, 0), "mq order wait");
    return HD_OK;
}

static int mq_refuse(hd_mq* q) {
    q->ctx->last_error = "message queue: an earlier insert failed part-way; the queue's state is lost";
    return HD_EDEVICE;
}

extern "C" {

int hd_mq_create(hd_ctx* ctx, uint32_t max_capacity, hd_mq** out) {
    if (!ctx || !out || max_capacity == 0) return HD_EINVAL;
    hd_mq* q = new (std::nothrow) hd_mq();
    if (!q) return HD_ENOMEM;
    q->ctx = ctx;
    q->max_cap = max_capacity;
    q->seed = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() * 0x9E3779B97F4A7C15ull ^
              (uint64_t)(uintptr_t)q;
    if (const char* e = getenv("HD_MQ_MAPPED")) q->mapped = atoi(e) != 0;
    *out = q;
    return HD_OK;
}

int hd_mq_destroy(hd_mq* q) {
    if (!q) return HD_EINVAL;
    (void)hipSetDevice(q->ctx->device);
    (void)hipStreamSynchronize(q->ctx->stream);
    if (q->pool.base) (void)hipFree(q->pool.base);
    if (q->spare.base) (void)hipFree(q->spare.base);
    if (q->keys) (void)hipFree(q->keys);
    if (q->slots) (void)hipFree(q->slots);
    for (auto& b : q->buf)
        if (b.p) (void)hipFree(b.p);
    if (q->hstage) (void)hipHostFree(q->hstage);
    if (q->mstage) (void)hipHostFree(q->mstage);
    if (q->rep) (void)hipHostFree(q->rep);
    if (q->order_ev) (void)hipEventDestroy(q->order_ev);
    delete q;
    return HD_OK;
}

int hd_mq_size(hd_mq* q, uint64_t* n) {
    if (!q || !n) return HD_EINVAL;
    *n = q->live;
    return HD_OK;
}

int hd_mq_senders(hd_mq* q, uint32_t* n) {
    if (!q || !n) return HD_EINVAL;
    *n = q->nsend;
    return HD_OK;
}

int hd_mq_insert_device(hd_mq* q, const hd_batch* d_batch, const uint8_t* d_insert, void* stream) {
    if (!q || !d_batch) return HD_EINVAL;
    if (q->failed) return mq_refuse(q);
    const uint32_t nb = d_batch->n;
    if (nb == 0) return HD_OK;  // empty device tensors may have NULL data pointers
    if (!d_batch->type || !d_batch->height || !d_batch->round || !d_batch->value32 || !d_batch->from32)
        return HD_EINVAL;
    (void)hipSetDevice(q->ctx->device);
    {
        const int rs = pf_sync(q);   // the queue on the device as consumed so far
        if (rs) return rs;
    }
    hipStream_t s = stream ? (hipStream_t)stream : q->ctx->stream;
    int rc = 0;
    uint8_t* flag = (uint8_t*)qbuf(q, MQ_FLAG, nb, &rc);
    if (rc) return rc;
    if ((rc = mq_order_after_ctx(q, s))) return rc;
    k_mq_flag_nz<<<nblk(nb), 256, 0, s>>>(nb, d_insert, flag);
    QCHK(hipGetLastError(), "k_mq_flag_nz");
    return mq_insert_flagged(q, d_batch, flag, s);
}

int hd_mq_insert_verified_device(hd_mq* q, const hd_batch* d_batch, const uint8_t* d_verdict, int64_t min_height,
                                 void* stream) {
    if (!q || !d_batch) return HD_EINVAL;
    if (q->failed) return mq_refuse(q);
    const uint32_t nb = d_batch->n;
    if (nb == 0) return HD_OK;
    if (!d_verdict) return HD_EINVAL;
    if (!d_batch->type || !d_batch->height || !d_batch->round || !d_batch->value32 || !d_batch->from32)
        return HD_EINVAL;
    (void)hipSetDevice(q->ctx->device);
    {
        const int rs = pf_sync(q);   // the queue on the device as consumed so far
        if (rs) return rs;
    }
    hipStream_t s = stream ? (hipStream_t)stream : q->ctx->stream;
    int rc = 0;
    uint8_t* flag = (uint8_t*)qbuf(q, MQ_FLAG, nb, &rc);
    if (rc) return rc;
    if ((rc = mq_order_after_ctx(q, s))) return rc;
    k_mq_ingress<<<nblk(nb), 256, 0, s>>>(nb, d_verdict, d_batch->height, min_height, flag);
    QCHK(hipGetLastError(), "k_mq_ingress");
    return mq_insert_flagged(q, d_batch, flag, s);
}

// the plan of a consume / drop (k_mq_plan) and its totals on the host
static int mq_plan(hd_mq* q, int64_t h, int strict, const uint8_t* allow, uint32_t totals[2], hipStream_t s) {
    int rc = 0;
    const uint32_t ns = q->nsend;
    uint32_t* newhead = (uint32_t*)qbuf(q, MQ_NEWHEAD, 4 * (size_t)ns, &rc);
    uint32_t* off = (uint32_t*)qbuf(q, MQ_OFF, 4 * (size_t)ns, &rc);
    uint32_t* tot = (uint32_t*)qbuf(q, MQ_TOT, 8, &rc);
    if (rc) return rc;
    if (q->hstage_cap < 64) {
        QCHK(hipHostMalloc(&q->hstage, 1u << 16, hipHostMallocDefault), "mq host stage");
        q->hstage_cap = 1u << 16;
    }
    k_mq_plan<<<1, 1024, 0, s>>>(ns, q->pool.h, (const uint32_t*)q->buf[MQ_HEADS].p,
                                 (const uint32_t*)q->buf[MQ_SEND].p, h, strict, allow, newhead, off, tot);
    QCHK(hipGetLastError(), "k_mq_plan");
    QCHK(hipMemcpyAsync(q->hstage, tot, 8, hipMemcpyDeviceToHost, s), "plan totals");
    QCHK(hipStreamSynchronize(s), "plan sync");
    memcpy(totals, q->hstage, 8);
    return HD_OK;
}

// the plan's new heads become the queue's
static int mq_commit(hd_mq* q, uint32_t removed, hipStream_t s) {
    if (!removed) return HD_OK;
    QCHK(hipMemcpyAsync(q->buf[MQ_HEADS].p, q->buf[MQ_NEWHEAD].p, 4 * (size_t)q->nsend, hipMemcpyDeviceToDevice, s),
         "commit heads");
    q->live -= removed;
    q->dead = true;
    return HD_OK;
}

#define HD_MQ_PF_ROWS 16384u     // window rows a prefetch may stage (160 B each)
#define HD_MQ_PF_WIN_MAX 64

// unpack `rows` staged rows (pointers) into the caller's SoA outputs
static void mq_unpack(const uint8_t* const* rows, uint32_t c, const hd_batch_out* out, int32_t* out_sender) {
    for (uint32_t k = 0; k < c; k++) {
        const uint8_t* row = rows[k];
        out->type[k] = row[153];
        memcpy(out->height + k, row, 8);
        memcpy(out->round + k, row + 8, 8);
        if (out->valid_round) memcpy(out->valid_round + k, row + 16, 8);
        memcpy(out->value32 + 32 * (size_t)k, row + 24, 32);
        memcpy(out->from32 + 32 * (size_t)k, row + 56, 32);
        if (out->sig65) memcpy(out->sig65 + 65 * (size_t)k, row + 88, 65);
        if (out_sender) memcpy(out_sender + k, row + 156, 4);
    }
    if (out->adv_class && c) memset(out->adv_class, 0, c);
}

// Commit the heads through pf_done on the device (the consumes served from
// the stage removed those messages on the host's count only) and forget the
// window.  Every operation that reads or changes the device queue calls it
// first.
static int pf_sync(hd_mq* q) {
    if (!q->pf) return HD_OK;
    q->pf = false;
    if (q->pf_done <= q->pf_dev) return HD_OK;
    hipStream_t s = q->ctx->stream;
    uint32_t tot[2];
    int rc = mq_plan(q, q->pf_done, 0, nullptr, tot, s);
    if (rc) return rc;
    if (tot[1]) {
        QCHK(hipMemcpyAsync(q->buf[MQ_HEADS].p, q->buf[MQ_NEWHEAD].p, 4 * (size_t)q->nsend, hipMemcpyDeviceToDevice,
                            s), "prefetch commit");
        q->dead = true;
    }
    QCHK(hipStreamSynchronize(s), "prefetch commit");
    return HD_OK;
}

// Index the window rows the last consume staged (np rows after the c
// delivered ones) by height, for the consumes of (h, h + win].
static void pf_index(hd_mq* q, int64_t h, int64_t hmax, const uint8_t* win, uint32_t np) {
    const uint32_t nh = (uint32_t)(hmax - h);
    q->pf_start.assign(nh + 1, 0u);
    q->pf_idx.resize(np);
    std::vector<uint32_t> hk(np);
    for (uint32_t k = 0; k < np; k++) {
        int64_t hv;
        memcpy(&hv, win + (size_t)HD_MQ_ROW * k, 8);
        hk[k] = (uint32_t)(hv - h - 1);   // in [0, nh): the kernel staged heights (h, hmax] only
        q->pf_start[hk[k] + 1]++;
    }
    for (uint32_t j = 0; j < nh; j++) q->pf_start[j + 1] += q->pf_start[j];
    std::vector<uint32_t> fill(q->pf_start.begin(), q->pf_start.end() - 1);
    for (uint32_t k = 0; k < np; k++) q->pf_idx[fill[hk[k]]++] = k;   // row order kept within a height
    q->pf_base = win;
    q->pf_dev = q->pf_done = h;
    q->pf_max = hmax;
    q->pf_adm_ver = q->ctx->adm_ver;
    q->pf = true;
}

// A consume of height h from the window (the caller checked pf, the admitted
// set and h <= pf_max): the rows of the heights (pf_done, h] in queue order.
static int pf_consume(hd_mq* q, int64_t h, const hd_batch_out* out, int32_t* out_sender, uint32_t cap,
                      uint32_t* n_out, uint32_t* n_removed) {
    *n_out = 0;
    if (n_removed) *n_removed = 0;
    if (h <= q->pf_done) return HD_OK;
    const uint32_t j0 = (uint32_t)(q->pf_done - q->pf_dev), j1 = (uint32_t)(h - q->pf_dev);
    // heights (pf_done, h] are buckets j0 .. j1 - 1 (bucket j = height pf_dev + 1 + j)
    std::vector<uint32_t> ids(q->pf_idx.begin() + q->pf_start[j0], q->pf_idx.begin() + q->pf_start[j1]);
    if (j1 - j0 > 1) std::sort(ids.begin(), ids.end());   // several heights: back to queue order
    std::vector<const uint8_t*> rows;
    rows.reserve(ids.size());
    for (uint32_t k : ids) {
        const uint8_t* row = q->pf_base + (size_t)HD_MQ_ROW * k;
        if (row[154]) rows.push_back(row);   // the sender is in procsAllowed
    }
    const uint32_t c = (uint32_t)rows.size(), nr = (uint32_t)ids.size();
    *n_out = c;
    if (c > cap) return HD_ECAP;   // nothing consumed
    if (n_removed) *n_removed = nr;
    mq_unpack(rows.data(), c, out, out_sender);
    q->live -= nr;
    q->pf_done = h;
    q->last_deliv = c;
    return HD_OK;
}

// Consume of a queue with at most 1024 senders and a capacity of at most
// HD_MQ_FUSED_ROWS: one kernel (k_mq_consume1), then a download of the
// header and of as many 160-byte rows as the previous consume delivered
// (twice that, at least 64), and a second copy only when this delivery is
// larger.  The rows are unpacked into the caller's SoA arrays on the host.
#define HD_MQ_FUSED_ROWS 65536u   // larger deliveries take the multi-block path
static int mq_consume1(hd_mq* q, int64_t h, const uint32_t* list, uint32_t na, int be, const hd_batch_out* out,
                       int32_t* out_sender, uint32_t cap, uint32_t* n_out, uint32_t* n_removed) {
    hipStream_t s = q->ctx->stream;
    int rc = 0;
    const uint32_t rows = std::max(cap, 1u);
    const size_t bytes = HD_MQ_HDR + (size_t)HD_MQ_ROW * rows;
    uint8_t* hs = nullptr;
    uint32_t c = 0, nr = 0;
    if (q->mapped) {
        // the kernel writes the header and rows straight into mapped host
        // memory and, last, the call's sequence number: no copy, no stream
        // synchronisation on the common path.  In the admitted-set mode the
        // launch also stages the next heights' window (prefetch).
        const bool pf = be != 0;
        // the window's end, clamped: a consume within pf_win of INT64_MAX
        // stages what is left up to INT64_MAX (no signed overflow)
        const int64_t hpf = !pf ? h : (h > INT64_MAX - q->pf_win ? INT64_MAX : h + q->pf_win);
        const size_t bytes_pf = bytes + (pf ? (size_t)HD_MQ_ROW * HD_MQ_PF_ROWS : 0);
        if (q->mstage_cap < bytes_pf) {
            if (q->mstage) (void)hipHostFree(q->mstage);
            q->mstage = nullptr;
            q->mstage_cap = 0;
            const size_t want = std::max(bytes_pf, (size_t)1 << 16);
            QCHK(hipHostMalloc(&q->mstage, want, hipHostMallocMapped | hipHostMallocCoherent), "mq mapped stage");
            void* dp = nullptr;
            QCHK(hipHostGetDevicePointer(&dp, q->mstage, 0), "mq mapped stage pointer");
            q->mstage_dev = (uint8_t*)dp;
            q->mstage_cap = want;
        }
        const uint32_t seq = ++q->seq ? q->seq : ++q->seq;   // never 0 (0 = no signal)
        uint32_t* meta = pf ? (uint32_t*)qbuf(q, MQ_WIN, 4 * (2 + 3 * 1024), &rc) : nullptr;
        if (rc) return rc;
        k_mq_consume1<<<1, 1024, 0, s>>>(q->nsend, q->pool, (uint32_t*)q->buf[MQ_HEADS].p,
                                         (const uint32_t*)q->buf[MQ_SEND].p, h, na, list, be, dict_of(q), rows, cap,
                                         q->mstage_dev, pf ? 0u : seq, hpf, pf ? HD_MQ_PF_ROWS : 0u, meta);
        if (pf) {
            k_mq_window_rows<<<64, 256, 0, s>>>(q->nsend, q->pool, meta, q->mstage_dev);
            k_mq_signal<<<1, 64, 0, s>>>(q->mstage_dev, seq);
        }
        QCHK(hipGetLastError(), "k_mq_consume1");
        hs = (uint8_t*)q->mstage;
        volatile uint32_t* word = (volatile uint32_t*)hs + 2;
        // spin for the sequence word; past ~0.2 s, wait for the stream (a
        // fault surfaces there) and read it once more
        const auto t0 = std::chrono::steady_clock::now();
        while (*word != seq) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                QCHK(hipStreamSynchronize(s), "consume sync");
                if (*word != seq) return hd_ctx_fail(q->ctx, hipErrorUnknown, "consume signal");
                break;
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        c = ((const uint32_t*)hs)[0];
        nr = ((const uint32_t*)hs)[1];
        *n_out = c;
        if (c > cap) return HD_ECAP;   // nothing committed
        const uint32_t np = ((const uint32_t*)hs)[3], win = ((const uint32_t*)hs)[4];
        if (win == 1) {
            pf_index(q, h, hpf, hs + HD_MQ_HDR + (size_t)HD_MQ_ROW * c, np);
            q->pf_win = std::min(2 * q->pf_win, HD_MQ_PF_WIN_MAX);
        } else if (win == 2) {
            q->pf_win = std::max(1, q->pf_win / 2);   // the window overflowed the stage: a narrower one next time
        }
    } else {
        uint8_t* dst = (uint8_t*)qbuf(q, MQ_STAGE, bytes, &rc);
        if (rc) return rc;
        if (q->hstage_cap < bytes) {
            if (q->hstage) (void)hipHostFree(q->hstage);
            q->hstage = nullptr;
            q->hstage_cap = 0;
            const size_t want = std::max(bytes, (size_t)1 << 16);
            QCHK(hipHostMalloc(&q->hstage, want, hipHostMallocDefault), "mq host stage");
            q->hstage_cap = want;
        }
        k_mq_consume1<<<1, 1024, 0, s>>>(q->nsend, q->pool, (uint32_t*)q->buf[MQ_HEADS].p,
                                         (const uint32_t*)q->buf[MQ_SEND].p, h, na, list, be, dict_of(q), rows, cap,
                                         dst, 0u, h, 0u, nullptr);
        QCHK(hipGetLastError(), "k_mq_consume1");
        const uint32_t guess = std::min(rows, std::max(64u, 2 * q->last_deliv));
        hs = (uint8_t*)q->hstage;
        QCHK(hipMemcpyAsync(hs, dst, HD_MQ_HDR + (size_t)HD_MQ_ROW * guess, hipMemcpyDeviceToHost, s),
             "consume download");
        QCHK(hipStreamSynchronize(s), "consume sync");
        c = ((const uint32_t*)hs)[0];
        nr = ((const uint32_t*)hs)[1];
        *n_out = c;
        if (c > cap) return HD_ECAP;   // nothing committed
        if (c > guess) {
            const size_t o = HD_MQ_HDR + (size_t)HD_MQ_ROW * guess;
            QCHK(hipMemcpyAsync(hs + o, dst + o, (size_t)HD_MQ_ROW * (c - guess), hipMemcpyDeviceToHost, s),
                 "consume download rest");
            QCHK(hipStreamSynchronize(s), "consume sync");
        }
    }
    q->last_deliv = c;
    if (n_removed) *n_removed = nr;
    if (nr) {
        q->live -= nr;
        q->dead = true;
    }
    std::vector<const uint8_t*> rp(c);
    for (uint32_t k = 0; k < c; k++) rp[k] = hs + HD_MQ_HDR + (size_t)HD_MQ_ROW * k;
    mq_unpack(rp.data(), c, out, out_sender);
    return HD_OK;
}

// Consume in one host round trip: allow flags -> plan -> the delivered rows
// gathered into a stage of `cap` rows (the caller's capacity) -> heads
// committed on the device if they fit -> ONE download of the plan totals and
// the stage (a small consume is latency-bound: a second sync costs more than
// the unused stage rows' bytes).  A stage larger than HD_MQ_STAGE_ROWS is
// sized by a planning round trip first.
#define HD_MQ_STAGE_ROWS 4096u
int hd_mq_consume(hd_mq* q, int64_t h, const uint8_t* allowed32, uint32_t n_allowed, const hd_batch_out* out,
                  int32_t* out_sender, uint32_t cap, uint32_t* n_out, uint32_t* n_removed) {
    if (!q || !out || !n_out) return HD_EINVAL;
    if (q->failed) return mq_refuse(q);
    if (!out->type || !out->height || !out->round || !out->value32 || !out->from32) return HD_EINVAL;
    if (allowed32 == nullptr && n_allowed != 0) return HD_EINVAL;
    *n_out = 0;
    if (n_removed) *n_removed = 0;
    if (q->pf) {   // a staged window: served by the host while it still holds
        if (!allowed32 && q->pf_adm_ver == q->ctx->adm_ver && h <= q->pf_max)
            return pf_consume(q, h, out, out_sender, cap, n_out, n_removed);
        (void)hipSetDevice(q->ctx->device);
        const int rs = pf_sync(q);
        if (rs) return rs;
    }
    if (q->live == 0) return HD_OK;
    (void)hipSetDevice(q->ctx->device);
    hipStream_t s = q->ctx->stream;
    int rc = 0;
    // procsAllowed: the allowed list (uploaded) or the ctx's admitted set
    const uint32_t* list = nullptr;
    uint32_t na = 0;
    int be = 0;
    if (allowed32) {
        na = n_allowed;
        if (na) {
            uint32_t* d = (uint32_t*)qbuf(q, MQ_LIST, 32 * (size_t)na, &rc);
            if (rc) return rc;
            QCHK(hipMemcpyAsync(d, allowed32, 32 * (size_t)na, hipMemcpyHostToDevice, s), "allowed upload");
            list = d;
        }
    } else {
        na = q->ctx->n_adm;   // the ctx's admitted set now (sorted, big-endian words)
        list = q->ctx->d_adm;
        be = 1;
    }
    const uint32_t ns = q->nsend;
    if (ns <= 1024 && cap <= HD_MQ_FUSED_ROWS) return mq_consume1(q, h, list, na, be, out, out_sender, cap, n_out,
                                                                   n_removed);
    uint8_t* allow = (uint8_t*)qbuf(q, MQ_ALLOW, q->nsend, &rc);
    if (rc) return rc;
    QCHK(hipMemsetAsync(allow, 0, q->nsend, s), "clear allow");
    if (na) k_mq_allow<<<nblk(na), 256, 0, s>>>(na, list, be, dict_of(q), allow);
    uint32_t* newhead = (uint32_t*)qbuf(q, MQ_NEWHEAD, 4 * (size_t)ns, &rc);
    uint32_t* off = (uint32_t*)qbuf(q, MQ_OFF, 4 * (size_t)ns, &rc);
    uint32_t* tot = (uint32_t*)qbuf(q, MQ_TOT, 64, &rc);
    if (rc) return rc;
    uint32_t* head = (uint32_t*)q->buf[MQ_HEADS].p;
    k_mq_plan<<<1, 1024, 0, s>>>(ns, q->pool.h, head, (const uint32_t*)q->buf[MQ_SEND].p, h, 0, allow, newhead, off,
                                 tot);
    QCHK(hipGetLastError(), "k_mq_plan");
    // stage rows: the caller's room, at most HD_MQ_STAGE_ROWS without knowing
    // the count (a larger delivery is planned first, then staged exactly)
    uint32_t rows = std::min(cap, HD_MQ_STAGE_ROWS);
    if (cap > HD_MQ_STAGE_ROWS) {
        uint32_t t[2];
        QCHK(hipMemcpyAsync(t, tot, 8, hipMemcpyDeviceToHost, s), "plan totals");
        QCHK(hipStreamSynchronize(s), "plan sync");
        rows = std::min(cap, t[0]);
    }
    const uint32_t r16 = (std::max(rows, 1u) + 15u) & ~15u;
    const size_t bytes = pool_bytes(r16);
    void* dst = qbuf(q, MQ_STAGE, bytes, &rc);
    if (rc) return rc;
    if (q->hstage_cap < bytes + 64) {
        if (q->hstage) (void)hipHostFree(q->hstage);
        q->hstage = nullptr;
        q->hstage_cap = 0;
        const size_t want = bytes + bytes / 2 + 64;
        QCHK(hipHostMalloc(&q->hstage, want, hipHostMallocDefault), "mq host stage");
        q->hstage_cap = want;
    }
    const Pool d = pool_view(dst, r16);
    if (rows) k_mq_take<<<ns, 256, 0, s>>>(q->pool, head, newhead, off, allow, rows, d);
    k_mq_commit<<<std::min(nblk(ns), 64u), 256, 0, s>>>(ns, newhead, tot, cap, head);
    QCHK(hipGetLastError(), "consume kernels");
    uint32_t* htot = (uint32_t*)q->hstage;                  // totals first, then the stage
    void* hrows = (char*)q->hstage + 64;
    QCHK(hipMemcpyAsync(htot, tot, 8, hipMemcpyDeviceToHost, s), "consume totals");
    if (rows) QCHK(hipMemcpyAsync(hrows, dst, bytes, hipMemcpyDeviceToHost, s), "consume download");
    QCHK(hipStreamSynchronize(s), "consume sync");
    const uint32_t c = htot[0], nr = htot[1];
    *n_out = c;
    if (c > cap) return HD_ECAP;   // nothing committed
    if (n_removed) *n_removed = nr;
    if (nr) {
        q->live -= nr;
        q->dead = true;
    }
    if (c) {
        const Pool hp = pool_view(hrows, r16);
        struct Cp { void* dst; const void* src; size_t sz; } cp[] = {
            {out->type, hp.type, (size_t)c},          {out->height, hp.h, 8 * (size_t)c},
            {out->round, hp.r, 8 * (size_t)c},        {out->valid_round, hp.vr, 8 * (size_t)c},
            {out->value32, hp.value, 32 * (size_t)c}, {out->from32, hp.from, 32 * (size_t)c},
            {out->sig65, hp.sig, 65 * (size_t)c},     {out_sender, hp.sender, 4 * (size_t)c},
        };
        for (auto& x : cp)
            if (x.dst) memcpy(x.dst, x.src, x.sz);
        if (out->adv_class) memset(out->adv_class, 0, c);
    }
    return HD_OK;
}

int hd_mq_consume_votes(hd_mq* q, struct hd_votes* v, int64_t h, const uint8_t* allowed32, uint32_t n_allowed,
                        const hd_batch_out* out, int32_t* out_sender, uint32_t cap, uint32_t* n_out,
                        uint32_t* n_removed, uint8_t* status, uint32_t* double_of, uint8_t* events,
                        uint32_t* n_inserted) {
    if (!v || !n_out) return HD_EINVAL;
    if (n_inserted) *n_inserted = 0;
    int rc = hd_mq_consume(q, h, allowed32, n_allowed, out, out_sender, cap, n_out, n_removed);
    if (rc || *n_out == 0) return rc;
    const hd_batch b{*n_out, out->type, out->height, out->round, out->valid_round, out->value32, out->from32,
                     out->sig65};
    return hd_votes_insert_batch(v, &b, nullptr, status, double_of, events, n_inserted);
}

int hd_mq_drop_below(hd_mq* q, int64_t h) {
    if (!q) return HD_EINVAL;
    if (q->failed) return mq_refuse(q);
    if (q->pf) {
        if (h - 1 <= q->pf_done) return HD_OK;   // nothing below h is left
        if (h - 1 <= q->pf_max) {                // the window's heights (pf_done, h - 1] leave undelivered
            const uint32_t j0 = (uint32_t)(q->pf_done - q->pf_dev), j1 = (uint32_t)(h - 1 - q->pf_dev);
            q->live -= q->pf_start[j1] - q->pf_start[j0];
            q->pf_done = h - 1;
            return HD_OK;
        }
        (void)hipSetDevice(q->ctx->device);
        const int rs = pf_sync(q);
        if (rs) return rs;
    }
    if (q->live == 0) return HD_OK;
    (void)hipSetDevice(q->ctx->device);
    hipStream_t s = q->ctx->stream;
    uint32_t tot[2];
    int rc = mq_plan(q, h, 1, nullptr, tot, s);
    if (rc) return rc;
    return mq_commit(q, tot[1], s);
}

}  // extern "C"
