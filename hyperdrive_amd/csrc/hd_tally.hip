// hd_tally.hip -- GPU tally of authenticated votes: the first-wins vote logs
// of process/process.go:823-892 and the counts the 2f+1 / f+1 rules read
// (process.go:486-494, 534, 574-582, 626-632, 658, 696-702, 751), for every
// (height, round) in a batch at once.
//
// Candidates are VALID Prevotes / Precommits.  Three group-bys:
//
//   G  (h, r)                 open-addressing hash table in HBM, one slot per
//                             round: distinct prevote and precommit signers,
//                             signers with both (probed once per wavefront:
//                             lanes of a wavefront usually share their round)
//   logs (h, r, type, From)   first-wins vote logs (process.go:834-847): for an
//                             admitted From a dense cell (round rank, type,
//                             admitted index) of an L2-resident word array,
//                             first-wins = atomicMin of the batch index; a From
//                             outside the admitted set takes the hashed table D
//   C  (G slot, type, value)  count of first-wins votes per value
//                             (process.go:574-579 and the other count loops)
//
// A hash slot's `claim` word holds the LOWEST batch index of its key: a new
// key claims an empty slot by CAS, an equal key with a lower index lowers it
// by atomicMin.  Keys are never copied -- a probe compares against the
// claimer's fields in the (immutable) batch, so there is no torn-key window.
// The distinct signers of a round over both types (TraceLogs[r] restricted to
// votes, process.go:744-754) are prevotes + precommits - signers with both.
// Counts are integer atomics, hence deterministic; outputs are ordered by the
// batch index of each group's first message (first-item bitmaps and their
// popcount prefixes, no sort).
// Non-winners compare their value with the winner's: identical -> dropped
// silently, different -> the double vote handed to Catcher.CatchDouble*
// (process.go:838-843, 875-880).
#include <hip/hip_runtime.h>

#include <chrono>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <vector>

#include "hd_internal.h"
#include "hd_verify_msg.h"

using namespace hd;

static const uint32_t kEmpty = 0xFFFFFFFFu;

struct TallyWork {
    DevBuf b[15];
    void* host = nullptr;   // pinned download stage (hipHostMalloc)
    size_t host_cap = 0;
    uint32_t* scalar = nullptr;   // pinned word (a partition's candidate count)
    // staged row capacities (the last call's counts + 1/4); atomic: an async
    // collect may raise them while another thread submits
    std::atomic<uint32_t> guess_hr{1024}, guess_cnt{1024};
    // the tables clean themselves (k_tally_emit): cleared only when their
    // allocation or capacity changes, or a call did not queue all its launches
    bool dirty = false;
    const void* tab_p = nullptr;
    uint32_t tab_k = 0;
};
// T_G: the hash tables and call counters; T_C: the dense log cells; T_D /
// T_SORTK / T_TMP: a partition's candidate compaction; T_GSLOT / T_DSLOT /
// T_CSLOT: per-item round slot, log reference and count slot; T_BITS: the
// first-item bitmaps and their prefixes; T_SEL: the output stage; T_NSEL: the
// overflow rows; T_DUP: a routed batch's classification when it is scattered
// on the device instead of staged; T_CHECK: HD_TALLY_CHECK's counters
enum TSlot { T_G, T_D, T_C, T_GSLOT, T_DSLOT, T_NSEL, T_SEL, T_SORTK, T_SORTV, T_TMP, T_DUP, T_ROUTE, T_CHECK,
             T_CSLOT, T_BITS };

// table layouts (structure of arrays inside one allocation, capacity cap)
struct GTab {   // (h, r)
    uint32_t* claim;
    uint32_t* nprev;
    uint32_t* nprec;
    uint32_t* nboth;
    uint32_t* gid;   // the round's number (creation order): its dense log cells
};
struct CTab {   // (G slot, type, value)
    uint32_t* claim;
    uint32_t* n;
};
struct TallyCtr {   // 64 B, zero between calls (k_tally_emit resets it)
    uint32_t n_rounds;   // rounds numbered so far (k_tally_rounds)
    uint32_t pad[15];
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

// verdict and bitmap both NULL: every Prevote / Precommit is a candidate (a
// batch of routed candidates, hd_unroute_device)
__device__ __forceinline__ bool candidate(const DevBatch& b, const uint8_t* verdict, const uint32_t* bitmap,
                                          uint32_t i, Part p) {
    const uint8_t t = b.type[i];
    if (t != T_PREVOTE && t != T_PRECOMMIT) return false;
    if (verdict && verdict[i] != V_VALID) return false;
    if (bitmap && !((bitmap[i >> 5] >> (i & 31)) & 1u)) return false;
    return p.nparts <= 1 || part_of(hash_hr(b.height[i], b.round[i]), p.nparts) == p.part;
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

// Items.  The whole-batch tally walks every message (item p = batch index
// p); a partition's tally first compacts its candidates into cand[] (in
// batch order, k_tally_flag + the ordered compaction below), so that every
// later pass and every index array is sized by the partition's candidates,
// not by the replicated batch (G ranks x the per-GPU batch).  Claim words
// hold item numbers, which order like batch indices.
__device__ __forceinline__ uint32_t msg_of(const uint32_t* cand, uint32_t p) { return cand ? cand[p] : p; }

// a partition's candidates: at[i] = i, others empty; dup of the others = 3
__global__ __launch_bounds__(256) void k_tally_flag(DevBatch b, const uint8_t* __restrict__ verdict,
                                                    const uint32_t* __restrict__ bitmap, Part p,
                                                    uint32_t* __restrict__ at, uint8_t* __restrict__ dup) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += gridDim.x * blockDim.x) {
        const bool c = candidate(b, verdict, bitmap, i, p);
        at[i] = c ? i : kEmpty;
        if (dup && !c) dup[i] = 3;
    }
}

// pass 1: every candidate -> its round (G slot).  Lanes of a wavefront
// usually share their round, so the first candidate lane probes for all lanes
// with its (h, r) (shfl64).  Without cand[] the pass also filters the
// candidates.  The lane that creates a round's slot numbers the round
// (gid, in creation order) and its wavefront clears the round's 2S dense log
// cells, so the cells need no clearing pass.  The loop is wavefront-uniform
// (every lane reaches the ballots).
__global__ void k_tally_rounds(DevBatch b, const uint32_t* __restrict__ cand, uint32_t m,
                               const uint8_t* __restrict__ verdict, const uint32_t* __restrict__ bitmap, Part p,
                               GTab G, uint32_t mask, uint32_t* __restrict__ gslot, uint8_t* __restrict__ dup,
                               TallyCtr* ctr, uint32_t* __restrict__ Dd, uint32_t per, uint32_t nd) {
    const uint32_t stride = gridDim.x * blockDim.x;
    const int lane = threadIdx.x & 63;
    for (uint32_t base = blockIdx.x * blockDim.x; base < m; base += stride) {
        const uint32_t q = base + threadIdx.x;
        bool c = q < m;
        const uint32_t i = c ? msg_of(cand, q) : 0u;
        if (c && !cand && !candidate(b, verdict, bitmap, i, p)) {
            if (dup) dup[i] = 3;
            gslot[q] = kEmpty;
            c = false;
        }
        const unsigned long long act = __ballot(c);
        if (!act) continue;
        const int lead = __ffsll((long long)act) - 1;
        const int64_t h = c ? b.height[i] : 0, r = c ? b.round[i] : 0;
        const int64_t hl = shfl64(h, lead), rl = shfl64(r, lead);   // every lane takes part in the shuffles
        const bool follower = c && lane != lead && hl == h && rl == r;
        uint32_t g = kEmpty, id = kEmpty;
        bool created = false;
        if (c && !follower) {
            g = probe(G.claim, mask, hash_hr(h, r), q,
                      [&](uint32_t o) {
                          const uint32_t io = msg_of(cand, o);
                          return b.height[io] == h && b.round[io] == r;
                      },
                      created);
            if (created) {
                id = atomicAdd(&ctr->n_rounds, 1u);
                G.gid[g] = id;
            }
        }
        const uint32_t gl = (uint32_t)__shfl((int)g, lead, 64);
        if (c) gslot[q] = follower ? gl : g;
        // the new rounds' dense cells, one round at a time by the whole wavefront
        unsigned long long cr = __ballot(created && id < nd);
        while (cr) {
            const int l = __ffsll((long long)cr) - 1;
            const uint32_t idl = (uint32_t)__shfl((int)id, l, 64);
            uint32_t* cells = Dd + (size_t)idl * per;
            for (uint32_t k = lane; k < per; k += 64) cells[k] = kEmpty;
            cr &= cr - 1;
        }
    }
}

// Dense vote logs.  A candidate's log key (h, r, type, From) is, for an
// admitted From, the cell (round number, type, admitted index) of an array of
// nd x 2 x S words -- a few MB, L2-resident -- and first-wins is one
// atomicMin of the item number into that cell: no hashing, no key compares
// against the batch.  A From outside the context's admitted set (possible
// when the caller's verdicts predate a set change), or a round numbered past
// the dense cells (a batch of very many rounds), takes the hashed table D
// instead; a signatory's prevote and precommit of a round always take the
// same path.  ref[q]: the cell index, or HD_REF_HASHED | the D slot.
#define HD_REF_HASHED 0x80000000u
__global__ void k_tally_logs(DevBatch b, const uint32_t* __restrict__ cand, uint32_t m,
                             const uint32_t* __restrict__ gslot, const uint32_t* __restrict__ gid,
                             AdmIndex ix, uint32_t S, uint32_t* __restrict__ Dd, uint32_t nd,
                             uint32_t* __restrict__ D, uint32_t mask, uint32_t* __restrict__ ref) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < m; q += stride) {
        const uint32_t g = gslot[q];
        if (g == kEmpty) continue;
        const uint32_t i = msg_of(cand, q);
        const uint8_t t = b.type[i];
        const uint8_t* from = b.from32 + 32 * (size_t)i;
        const uint32_t rid = gid[g];
        int32_t signer = -1;
        if (rid < nd) {
            uint32_t from_be[8];
            load_row32_be(from_be, b.from32, i);
            signer = adm_index_find(ix, from_be);
        }
        if (signer >= 0) {
            const uint32_t cell = (rid * 2u + (t == T_PRECOMMIT ? 1u : 0u)) * S + (uint32_t)signer;
            atomicMin(&Dd[cell], q);
            ref[q] = cell;
        } else {
            const int64_t h = b.height[i], r = b.round[i];
            bool created;
            const uint32_t d = probe(D, mask, hash_log(hash_hr(h, r), from, t), q,
                                     [&](uint32_t o) {
                                         const uint32_t io = msg_of(cand, o);
                                         return b.type[io] == t && b.height[io] == h && b.round[io] == r &&
                                                eq32(b.from32 + 32 * (size_t)io, from);
                                     },
                                     created);
            ref[q] = HD_REF_HASHED | d;
        }
    }
}

// the C table's key hash: (G slot, type, value)
__device__ __forceinline__ uint64_t hash_count(const uint8_t* value, uint32_t g, uint8_t t) {
    const uint64_t hv = *reinterpret_cast<const uint64_t*>(value) ^ *reinterpret_cast<const uint64_t*>(value + 8);
    return mix64(hv ^ ((uint64_t)g << 1 | (t & 1u)));
}

// Per-value counts of a wavefront's winners: the distinct (round, type,
// value) keys among the active lanes are handled one at a time -- the lowest
// lane holding a key (the lowest item, so first-wins of the claim word stays
// exact) probes C once and adds the number of lanes with that key in one
// atomic.  A batch's votes repeat few values per round, so this is a few
// probes and atomics per wavefront instead of one per lane on a handful of
// hot words.  Returns the C slot of this lane's key.
__device__ __forceinline__ uint32_t count_value(CTab C, uint32_t mask, const DevBatch& b, const uint32_t* cand,
                                                const uint32_t* gslot, uint32_t g, uint8_t t, uint32_t q,
                                                const uint8_t* value) {
    const uint4* vw = reinterpret_cast<const uint4*>(value);
    const uint4 v0 = vw[0], v1 = vw[1];
    const int lane = threadIdx.x & 63;
    unsigned long long pending = __ballot(true);
    uint32_t mine = 0;   // on a key's lowest lane: the number of lanes with the key
    int my_lead = lane;  // the lowest lane with this lane's key
    while (pending) {
        const int lead = __ffsll((long long)pending) - 1;
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
        const unsigned long long same = __ballot(diff == 0 && ((pending >> lane) & 1ull));
        if ((same >> lane) & 1ull) my_lead = lead;
        if (lane == lead) mine = (uint32_t)__popcll(same);
        pending &= ~same;
    }
    // the keys' lowest lanes probe C together (their keys differ), instead of
    // one after another inside the loop above
    uint32_t c = kEmpty;
    if (mine) {
        bool created;
        c = probe(C.claim, mask, hash_count(value, g, t), q,
                  [&](uint32_t o) {
                      const uint32_t io = msg_of(cand, o);
                      return gslot[o] == g && b.type[io] == t && eq32(b.value32 + 32 * (size_t)io, value);
                  },
                  created);
        atomicAdd(&C.n[c], mine);
    }
    return (uint32_t)__shfl((int)c, my_lead, 64);
}

// pass 3: each log entry's winner (the lowest item of its key) counts as a
// distinct signer of its type in the round and counts its value (C); a
// prevote winner whose signer also has a precommit log in the round counts
// in nboth.  The other candidates are classified against the winner's value.
// cslot[q]: a winner's C slot, kEmpty for the other candidates.
__global__ void k_tally_values(DevBatch b, const uint32_t* __restrict__ cand, uint32_t m,
                               const uint32_t* __restrict__ Dd, uint32_t S, const uint32_t* __restrict__ D,
                               GTab G, CTab C, uint32_t mask, const uint32_t* __restrict__ gslot,
                               const uint32_t* __restrict__ ref, uint32_t* __restrict__ cslot,
                               uint8_t* __restrict__ dup) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < m; q += stride) {
        const uint32_t g = gslot[q];
        if (g == kEmpty) continue;
        const uint32_t i = msg_of(cand, q);
        const uint32_t rf = ref[q];
        const bool hashed = (rf & HD_REF_HASHED) != 0;
        const uint32_t w = hashed ? D[rf & ~HD_REF_HASHED] : Dd[rf];
        const uint8_t* value = b.value32 + 32 * (size_t)i;
        if (w != q) {
            if (dup) dup[i] = eq32(b.value32 + 32 * (size_t)msg_of(cand, w), value) ? 1 : 2;
            cslot[q] = kEmpty;
            continue;
        }
        if (dup) dup[i] = 0;
        const uint8_t t = b.type[i];
        wave_add(G.nprev, g, t == T_PREVOTE);
        wave_add(G.nprec, g, t == T_PRECOMMIT);
        bool both = false;
        if (t == T_PREVOTE) {
            if (!hashed) {
                both = Dd[rf + S] != kEmpty;   // the same signer's precommit cell of the round
            } else {
                const int64_t h = b.height[i], r = b.round[i];
                const uint8_t* from = b.from32 + 32 * (size_t)i;
                const uint32_t o = find(D, mask, hash_log(hash_hr(h, r), from, T_PRECOMMIT), [&](uint32_t c) {
                    const uint32_t ic = msg_of(cand, c);
                    return b.type[ic] == T_PRECOMMIT && b.height[ic] == h && b.round[ic] == r &&
                           eq32(b.from32 + 32 * (size_t)ic, from);
                });
                both = o != kEmpty;
            }
        }
        wave_add(G.nboth, g, both);
        cslot[q] = count_value(C, mask, b, cand, gslot, g, t, q, value);
    }
}

// Output order: the groups of each table by their first item.  A group's
// first item is the one its slot's claim word holds; the per-item flags
// "first of its round" / "first of its (round, type, value)" are bitmaps
// Bg / Bc, one bit per item, and an item's output position is the number of
// flags before it.  Both passes below give each block IPB consecutive items
// (IPB / 32 bitmap words it alone writes; IPB = 256 .. 2048, the largest
// that still gives about four blocks per CU, tally_ipb()):
//   k_tally_firsts  the block's flags as whole words (two ballots per
//                   wavefront: no atomics, nothing to clear), their popcount
//                   prefix within the block, and the block's totals;
//   k_tally_emit    each block first sums the totals of the blocks before it
//                   (its offsets; the last block also writes the group counts
//                   into the stage header), then every first item writes its
//                   group's row at its position (rows past the staged
//                   capacity go to the overflow columns) and resets its table
//                   slots, so the tables are clean for the next call without
//                   a clearing pass.
// The offsets are summed by every emit block rather than scanned once by the
// last block of k_tally_firsts: that scan needed a ticket counter, and the
// device-scope release each block made before taking its ticket writes back
// the block's XCD L2 -- dirty with the verify kernels' rows when the tally
// runs beside them (39 us for 501 blocks of a 128k batch, against ~5 us
// for the sums, nb^2 / 2 L2-resident words).
#define HD_TALLY_IPB_MAX 2048u   // items per block (8 per thread)

template <uint32_t IPB>
__global__ __launch_bounds__(256) void k_tally_firsts(uint32_t m, const uint32_t* __restrict__ gslot,
                                                      const uint32_t* __restrict__ cslot, const uint32_t* G_claim,
                                                      const uint32_t* C_claim, uint32_t* __restrict__ Bg,
                                                      uint32_t* __restrict__ Bc, uint32_t* __restrict__ pre_g,
                                                      uint32_t* __restrict__ pre_c, uint32_t* __restrict__ blk) {
    constexpr uint32_t W = IPB / 32;   // words per block (<= 64: one wavefront scans them)
    __shared__ uint32_t wg[W], wc[W];
    const uint32_t nb = gridDim.x;
    const uint32_t lo = blockIdx.x * IPB;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t k = 0; k < IPB / 256; k++) {
        const uint32_t q = lo + k * 256 + threadIdx.x;
        bool fg = false, fc = false;
        if (q < m) {
            const uint32_t g = gslot[q];
            if (g != kEmpty) {
                fg = G_claim[g] == q;
                const uint32_t c = cslot[q];
                fc = c != kEmpty && C_claim[c] == q;
            }
        }
        const unsigned long long bg = __ballot(fg), bc = __ballot(fc);
        if (lane == 0) {
            const uint32_t w = k * 8 + wave * 2;
            wg[w] = (uint32_t)bg;
            wg[w + 1] = (uint32_t)(bg >> 32);
            wc[w] = (uint32_t)bc;
            wc[w + 1] = (uint32_t)(bc >> 32);
        }
    }
    __syncthreads();
    if (threadIdx.x < W) {   // one lane per word (wavefront 0)
        const uint32_t t = threadIdx.x, gw = wg[t], cw = wc[t];
        uint32_t ig = (uint32_t)__popc(gw), ic = (uint32_t)__popc(cw);
        for (int d = 1; d < 64; d <<= 1) {   // inclusive scan across the wavefront
            const uint32_t yg = (uint32_t)__shfl_up((int)ig, d, 64), yc = (uint32_t)__shfl_up((int)ic, d, 64);
            if ((int)t >= d) {
                ig += yg;
                ic += yc;
            }
        }
        const size_t wi = (size_t)blockIdx.x * W + t;
        Bg[wi] = gw;
        Bc[wi] = cw;
        pre_g[wi] = ig - (uint32_t)__popc(gw);
        pre_c[wi] = ic - (uint32_t)__popc(cw);
        if (t == W - 1) {
            blk[blockIdx.x] = ig;
            blk[nb + blockIdx.x] = ic;
        }
    }
}

// the output rows of one call, column arrays at capacities (H, Cg) in the
// stage and (m - H, m - Cg) in the overflow
struct TallyCols {
    int64_t *o_h, *o_r, *c_h, *c_r;
    uint32_t *o_prev, *o_prec, *o_any, *o_rep, *c_rep, *c_n;
    uint8_t* c_t;
};
HD_HOSTONLY TallyCols tally_cols(char* base, uint32_t h, uint32_t c) {
    TallyCols x;
    x.o_h = reinterpret_cast<int64_t*>(base);
    x.o_r = x.o_h + h;
    x.o_prev = reinterpret_cast<uint32_t*>(x.o_r + h);
    x.o_prec = x.o_prev + h;
    x.o_any = x.o_prec + h;
    x.o_rep = x.o_any + h;
    x.c_h = reinterpret_cast<int64_t*>(base + 32 * (size_t)h);
    x.c_r = x.c_h + c;
    x.c_rep = reinterpret_cast<uint32_t*>(x.c_r + c);
    x.c_n = x.c_rep + c;
    x.c_t = reinterpret_cast<uint8_t*>(x.c_n + c);
    return x;
}

template <uint32_t IPB>
__global__ __launch_bounds__(256) void k_tally_emit(DevBatch b, const uint32_t* __restrict__ cand, uint32_t m,
                                                    const uint32_t* __restrict__ gidx, const uint32_t* __restrict__ gslot,
                                                    const uint32_t* __restrict__ cslot, const uint32_t* __restrict__ ref,
                                                    GTab G, CTab C, uint32_t* __restrict__ D,
                                                    const uint32_t* __restrict__ Bg, const uint32_t* __restrict__ Bc,
                                                    const uint32_t* __restrict__ pre_g, const uint32_t* __restrict__ pre_c,
                                                    const uint32_t* __restrict__ blk, TallyCols st, uint32_t H,
                                                    uint32_t Cg, TallyCols ov, TallyCtr* ctr, uint32_t* stage_hdr) {
    const uint32_t nb = gridDim.x;
    // this block's offsets: the totals of the blocks before it
    __shared__ uint32_t part[2][4];
    uint32_t sg = 0, sc = 0;
    for (uint32_t k = threadIdx.x; k < blockIdx.x; k += 256) {
        sg += blk[k];
        sc += blk[nb + k];
    }
    for (int d = 32; d > 0; d >>= 1) {
        sg += (uint32_t)__shfl_xor((int)sg, d, 64);
        sc += (uint32_t)__shfl_xor((int)sc, d, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        part[0][threadIdx.x >> 6] = sg;
        part[1][threadIdx.x >> 6] = sc;
    }
    __syncthreads();
    const uint32_t og = part[0][0] + part[0][1] + part[0][2] + part[0][3];
    const uint32_t oc = part[1][0] + part[1][1] + part[1][2] + part[1][3];
    if (threadIdx.x == 0) {
        if (blockIdx.x == nb - 1) {
            stage_hdr[0] = og + blk[nb - 1];        // rounds (hr rows)
            stage_hdr[1] = oc + blk[2 * nb - 1];    // (round, type, value) groups
            stage_hdr[2] = 0;                       // an async ticket's completion word (k_tally_signal)
        }
        if (blockIdx.x == 0) ctr->n_rounds = 0;     // k_tally_rounds' numbering, for the next call
    }
    const uint32_t lo = blockIdx.x * IPB;
    for (uint32_t k = 0; k < IPB / 256; k++) {
        const uint32_t q = lo + k * 256 + threadIdx.x;
        if (q >= m) break;
        const uint32_t g = gslot[q];
        if (g == kEmpty) continue;
        const uint32_t i = msg_of(cand, q), w = q >> 5, below = (1u << (q & 31)) - 1u;
        const uint32_t gw = Bg[w], cw = Bc[w];
        if ((gw >> (q & 31)) & 1u) {   // the round's first candidate: its hr row
            const uint32_t pos = og + pre_g[w] + (uint32_t)__popc(gw & below);
            const TallyCols& x = pos < H ? st : ov;
            const uint32_t j = pos < H ? pos : pos - H;
            const uint32_t np = G.nprev[g], nc = G.nprec[g], nbo = G.nboth[g];
            x.o_h[j] = b.height[i];
            x.o_r[j] = b.round[i];
            x.o_prev[j] = np;
            x.o_prec[j] = nc;
            x.o_any[j] = np + nc - nbo;
            x.o_rep[j] = gidx ? gidx[i] : i;
            G.claim[g] = kEmpty;
            G.nprev[g] = G.nprec[g] = G.nboth[g] = 0;
        }
        if ((cw >> (q & 31)) & 1u) {   // the (round, type, value) group's first winner: its count row
            const uint32_t c = cslot[q];
            const uint32_t pos = oc + pre_c[w] + (uint32_t)__popc(cw & below);
            const TallyCols& x = pos < Cg ? st : ov;
            const uint32_t j = pos < Cg ? pos : pos - Cg;
            x.c_h[j] = b.height[i];
            x.c_r[j] = b.round[i];
            x.c_t[j] = b.type[i];
            x.c_rep[j] = gidx ? gidx[i] : i;
            x.c_n[j] = C.n[c];
            C.claim[c] = kEmpty;
            C.n[c] = 0;
        }
        const uint32_t rf = ref[q];
        if ((rf & HD_REF_HASHED) && D[rf & ~HD_REF_HASHED] == q) D[rf & ~HD_REF_HASHED] = kEmpty;   // the log's winner
    }
}

// An async tally's completion, after its download on the same stream: word 2
// of the caller's pinned stage (mapped) becomes 1.  hd_tally_collect polls it
// instead of synchronising an event: a thread blocked in hipEventSynchronize
// slowed the verify launches of the submitting thread 4x (c3_host_probe,
// HD_BENCH_ASYNC_TALLY=1: 0.18 ms per verify enqueue against 0.04).
__global__ void k_tally_signal(uint32_t* word) {
    if (threadIdx.x == 0) __hip_atomic_store(word, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// HD_TALLY_CHECK after k_tally_emit: the tables are clean again
__global__ void k_tally_check_clean(uint32_t cap, const uint32_t* __restrict__ tabs, TallyCtr* ctr, uint32_t* bad) {
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += gridDim.x * blockDim.x) {
        bool ok = true;
        for (int k = 0; k < 3; k++) ok &= tabs[(size_t)k * cap + s] == kEmpty;
        for (int k = 3; k < 7; k++) ok &= tabs[(size_t)k * cap + s] == 0u;
        if (!ok && atomicAdd(bad, 1u) == 0) printf("hd tally check: slot %u not clean after the emit\n", s);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && ctr->n_rounds) atomicAdd(bad, 1u);
}

// ------------------------------------------------- consistency check (debug)
// HD_TALLY_CHECK=1 in the environment: after k_tally_values, three kernels
// re-derive the tables' invariants and the host compares them (a violation is
// HD_EDEVICE with the counters in the context's last error, and the first
// offending slot printed by the device):
//   * every candidate's log cell holds an item of the same cell, no later than
//     itself (a stale or foreign cell would silently drop a winner);
//   * every non-empty dense cell / hashed D slot holds an item that maps to it;
//   * no two C (or D) slots hold the same key: the probe from the key of a
//     slot's claimer finds that slot first;
//   * every C claimer is a winner;
//   * winners == sum over G of (prevotes + precommits) == sum over C of n
//     == non-empty dense cells + D claims.
struct TallyCheck {
    uint32_t winners, cells, d_claims, sum_g, sum_c, stale, bad_cell, dup_key, bad_claim, pad[7];
};

__device__ __forceinline__ uint32_t cell_value(const uint32_t* Dd, const uint32_t* D, uint32_t rf) {
    return (rf & HD_REF_HASHED) ? D[rf & ~HD_REF_HASHED] : Dd[rf];
}

__global__ void k_tally_check_items(uint32_t m, const uint32_t* __restrict__ gslot, const uint32_t* __restrict__ ref,
                                    const uint32_t* __restrict__ Dd, const uint32_t* __restrict__ D,
                                    TallyCheck* chk) {
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < m; q += gridDim.x * blockDim.x) {
        if (gslot[q] == kEmpty) continue;
        const uint32_t rf = ref[q], w = cell_value(Dd, D, rf);
        if (w == q) {
            atomicAdd(&chk->winners, 1u);
        } else if (w == kEmpty || w > q || gslot[w] == kEmpty || ref[w] != rf) {
            if (atomicAdd(&chk->stale, 1u) == 0)
                printf("hd tally check: item %u ref %08x holds %u (ref %08x)\n", q, rf, w,
                       w < m ? ref[w] : 0xFFFFFFFFu);
        }
    }
}

__global__ void k_tally_check_cells(const uint32_t* __restrict__ Dd, const TallyCtr* ctr, uint32_t per, uint32_t nd,
                                    uint32_t m, const uint32_t* __restrict__ ref, TallyCheck* chk) {
    if (!Dd) return;
    const size_t cells = (size_t)min(ctr->n_rounds, nd) * per;   // the rounds numbered into dense cells
    for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < cells; c += (size_t)gridDim.x * blockDim.x) {
        const uint32_t w = Dd[c];
        if (w == kEmpty) continue;
        atomicAdd(&chk->cells, 1u);
        if (w >= m || ref[w] != (uint32_t)c)
            if (atomicAdd(&chk->bad_cell, 1u) == 0)
                printf("hd tally check: dense cell %lu holds item %u\n", (unsigned long)c, w);
    }
}

__global__ void k_tally_check_slots(DevBatch b, const uint32_t* __restrict__ cand, uint32_t m, uint32_t cap,
                                    GTab G, CTab C, const uint32_t* __restrict__ D, const uint32_t* __restrict__ Dd,
                                    const uint32_t* __restrict__ gslot, const uint32_t* __restrict__ ref,
                                    TallyCheck* chk) {
    const uint32_t mask = cap - 1;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += gridDim.x * blockDim.x) {
        if (G.claim[s] != kEmpty) atomicAdd(&chk->sum_g, G.nprev[s] + G.nprec[s]);
        const uint32_t c = C.claim[s];
        if (c != kEmpty) {
            atomicAdd(&chk->sum_c, C.n[s]);
            const uint32_t ic = msg_of(cand, c), g = gslot[c];
            const uint8_t t = b.type[ic];
            const uint8_t* value = b.value32 + 32 * (size_t)ic;
            if (c >= m || g == kEmpty || cell_value(Dd, D, ref[c]) != c)
                if (atomicAdd(&chk->bad_claim, 1u) == 0) printf("hd tally check: C slot %u claimer %u\n", s, c);
            const uint32_t f = find(C.claim, mask, hash_count(value, g, t), [&](uint32_t o) {
                const uint32_t io = msg_of(cand, o);
                return gslot[o] == g && b.type[io] == t && eq32(b.value32 + 32 * (size_t)io, value);
            });
            if (f != s)
                if (atomicAdd(&chk->dup_key, 1u) == 0)
                    printf("hd tally check: C slots %u and %u hold one key (claimers %u, %u)\n", f, s,
                           f == kEmpty ? kEmpty : C.claim[f], c);
        }
        const uint32_t d = D[s];
        if (d != kEmpty) {
            atomicAdd(&chk->d_claims, 1u);
            const uint32_t id = msg_of(cand, d);
            const uint8_t t = b.type[id];
            const int64_t h = b.height[id], r = b.round[id];
            const uint8_t* from = b.from32 + 32 * (size_t)id;
            const uint32_t f = find(D, mask, hash_log(hash_hr(h, r), from, t), [&](uint32_t o) {
                const uint32_t io = msg_of(cand, o);
                return b.type[io] == t && b.height[io] == h && b.round[io] == r &&
                       eq32(b.from32 + 32 * (size_t)io, from);
            });
            if (f != s)
                if (atomicAdd(&chk->dup_key, 1u) == 0) printf("hd tally check: D slots %u and %u hold one key\n", f, s);
        }
    }
}

// ordered compaction of at (n entries) in chunks of HD_CHUNK (a partition's
// candidates, in batch order): per-chunk counts, then each chunk writes from
// the sum of the counts before it (a block reads at most n / HD_CHUNK words)
#define HD_CHUNK 8192
__global__ __launch_bounds__(256) void k_tally_chunk_counts(uint32_t n, const uint32_t* __restrict__ at,
                                                            uint32_t* __restrict__ cnt) {
    typedef hipcub::BlockReduce<uint32_t, 256> Red;
    __shared__ typename Red::TempStorage ts;
    const uint32_t lo = blockIdx.x * HD_CHUNK, hi = min(n, lo + HD_CHUNK);
    uint32_t m = 0;
    for (uint32_t i = lo + threadIdx.x; i < hi; i += 256) m += at[i] != kEmpty ? 1u : 0u;
    const uint32_t t = Red(ts).Sum(m);
    if (threadIdx.x == 0) cnt[blockIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_tally_chunk_write(uint32_t n, const uint32_t* __restrict__ at,
                                                           const uint32_t* __restrict__ cnt,
                                                           uint32_t* __restrict__ order,
                                                           uint32_t* __restrict__ rank_of,
                                                           uint32_t* __restrict__ total) {
    typedef hipcub::BlockScan<uint32_t, 256> Scan;
    typedef hipcub::BlockReduce<uint32_t, 256> Red;
    __shared__ typename Scan::TempStorage ts;
    __shared__ typename Red::TempStorage rs;
    __shared__ uint32_t base;
    const uint32_t nch = (n + HD_CHUNK - 1) / HD_CHUNK;
    uint32_t bsum = 0;
    for (uint32_t k = threadIdx.x; k < blockIdx.x; k += 256) bsum += cnt[k];
    bsum = Red(rs).Sum(bsum);
    if (threadIdx.x == 0) {
        base = bsum;
        if (blockIdx.x == nch - 1) *total = bsum + cnt[blockIdx.x];
    }
    __syncthreads();
    constexpr uint32_t PER = HD_CHUNK / 256;   // contiguous entries per thread, in order
    const uint32_t lo = blockIdx.x * HD_CHUNK + threadIdx.x * PER;
    uint32_t mine = 0;
    for (uint32_t k = 0; k < PER; k++) mine += (lo + k < n && at[lo + k] != kEmpty) ? 1u : 0u;
    uint32_t off = 0;
    Scan(ts).ExclusiveSum(mine, off);
    uint32_t o = base + off;
    for (uint32_t k = 0; k < PER && mine; k++) {
        const uint32_t i = lo + k;
        if (i < n) {
            const uint32_t v = at[i];
            if (v != kEmpty) {
                order[o] = v;
                if (rank_of) rank_of[v] = o;
                o++;
            }
        }
    }
}

// ---------------------------------------------------------- routing (C4)
// The multi-GPU tally without a replicated batch: each device turns the
// candidates of ITS shard (VALID Prevotes / Precommits) into 64-byte route
// rows, grouped by the rank that owns the candidate's round
// (hd_tally_partition_of) and in index order inside a group; the groups
// cross xGMI (one grouped send/recv or all-to-all); the owner rebuilds a
// batch from the rows it received -- concatenated in source-rank order,
// which is global index order, since shards are contiguous index ranges --
// and tallies it (every row a candidate) with the reps mapped back to global
// indices.  First-wins is per (height, round, type, signer), so the owner of
// a round sees every candidate of its keys, in the order of the whole batch.
struct RouteRow {          // 64 B
    int64_t h, r;
    uint4 value[2];        // the 32 value bytes as stored
    uint32_t gidx;         // global batch index
    uint32_t signer_type;  // admitted (sorted) index << 8 | type
    uint32_t pad[2];
};
static_assert(sizeof(RouteRow) == 64, "route row");
#define HD_ROUTE_MAX_PARTS 64u

// Optional round filter of the route kernels: only candidates whose (h, r)
// is in a sorted list (lexicographic, signed) are routed -- the rounds that
// appear in more than one shard (hd_route_candidates_listed_device); every
// other round is tallied where it is.
struct RoundList {
    const int64_t* h;
    const int64_t* r;
    uint32_t n;
};
__device__ __forceinline__ bool round_listed(const RoundList& l, int64_t h, int64_t r) {
    if (!l.h) return true;
    uint32_t lo = 0, hi = l.n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const int64_t mh = l.h[mid], mr = l.r[mid];
        if (mh < h || (mh == h && mr < r)) lo = mid + 1;
        else hi = mid;
    }
    return lo < l.n && l.h[lo] == h && l.r[lo] == r;
}

// per block and owner: the number of candidates (o-major: cnt[o * nb + blk]);
// *outside counts candidates whose From is not in the context's admitted set
// (possible when the set changed since verification): a row carries the
// admitted index, not the From, so such a candidate cannot be routed
__global__ __launch_bounds__(256) void k_route_count(DevBatch b, const uint32_t* __restrict__ bitmap, uint32_t nparts,
                                                     AdmIndex ix, uint32_t n_adm, uint32_t* __restrict__ cnt,
                                                     uint32_t* __restrict__ outside, RoundList rl) {
    __shared__ uint32_t c[HD_ROUTE_MAX_PARTS];
    if (threadIdx.x < nparts) c[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < b.n && candidate(b, nullptr, bitmap, i, Part{0, 1}) && round_listed(rl, b.height[i], b.round[i])) {
        atomicAdd(&c[part_of(hash_hr(b.height[i], b.round[i]), nparts)], 1u);
        uint32_t from_be[8];
        load_row32_be(from_be, b.from32, i);
        const int32_t sg = n_adm ? adm_index_find(ix, from_be) : -1;
        if (sg < 0) atomicAdd(outside, 1u);
    }
    __syncthreads();
    if (threadIdx.x < nparts) cnt[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = c[threadIdx.x];
}

// the rows: block blk's candidates of owner o start at off[o * nb + blk]
// (the exclusive scan of k_route_count's counts), ranked inside the block by
// wavefront ballots, so each owner's rows keep the batch order
__global__ __launch_bounds__(256) void k_route_write(DevBatch b, const uint32_t* __restrict__ bitmap, uint32_t nparts,
                                                     uint32_t base, const uint32_t* __restrict__ off,
                                                     AdmIndex ix, uint32_t n_adm, RouteRow* __restrict__ rows,
                                                     RoundList rl) {
    __shared__ uint32_t wcnt[4][HD_ROUTE_MAX_PARTS];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const bool c = i < b.n && candidate(b, nullptr, bitmap, i, Part{0, 1}) && round_listed(rl, b.height[i], b.round[i]);
    const uint32_t o = c ? part_of(hash_hr(b.height[i], b.round[i]), nparts) : 0xFFFFFFFFu;
    uint32_t rank = 0;
    for (uint32_t k = 0; k < nparts; k++) {
        const unsigned long long bal = __ballot(o == k);
        if (o == k) rank = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wcnt[w][k] = (uint32_t)__popcll(bal);
    }
    __syncthreads();
    if (!c) return;
    uint32_t pos = off[(size_t)o * gridDim.x + blockIdx.x] + rank;
    for (uint32_t v = 0; v < w; v++) pos += wcnt[v][o];
    uint32_t from_be[8];
    load_row32_be(from_be, b.from32, i);
    const int32_t sg = n_adm ? adm_index_find(ix, from_be) : -1;
    RouteRow row;
    row.h = b.height[i];
    row.r = b.round[i];
    const uint4* vp = reinterpret_cast<const uint4*>(b.value32 + 32 * (size_t)i);
    row.value[0] = vp[0];
    row.value[1] = vp[1];
    row.gidx = base + i;
    // a VALID message's From is admitted (NOT_ADMITTED otherwise); a batch
    // with a candidate outside the current set was refused before this kernel
    row.signer_type = ((uint32_t)(sg >= 0 ? sg : 0xFFFFFF) << 8) | b.type[i];
    row.pad[0] = row.pad[1] = 0;
    rows[pos] = row;
}

// the owners' starts: starts[o] = off[o * nb], starts[nparts] = the total
__global__ void k_route_starts(const uint32_t* __restrict__ off, const uint32_t* __restrict__ cnt, uint32_t nparts,
                               uint32_t nb, uint32_t* __restrict__ starts) {
    const uint32_t o = threadIdx.x;
    if (o < nparts) starts[o] = off[(size_t)o * nb];
    if (o == 0) {
        const size_t last = (size_t)nparts * nb - 1;
        starts[nparts] = off[last] + cnt[last];
    }
}

// received rows -> a batch (From rebuilt from the admitted set) + gidx
__global__ __launch_bounds__(256) void k_unroute(const RouteRow* __restrict__ rows, uint32_t n,
                                                 const uint32_t* __restrict__ adm, uint32_t n_adm, hd_batch_out o,
                                                 uint32_t* __restrict__ gidx) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const RouteRow row = rows[j];
    const uint32_t sg = row.signer_type >> 8;
    o.type[j] = (uint8_t)(row.signer_type & 0xFFu);
    ((int64_t*)o.height)[j] = row.h;
    ((int64_t*)o.round)[j] = row.r;
    if (o.valid_round) ((int64_t*)o.valid_round)[j] = -1;
    uint4* vp = reinterpret_cast<uint4*>(o.value32 + 32 * (size_t)j);
    vp[0] = row.value[0];
    vp[1] = row.value[1];
    uint32_t f[8];
    HD_UNROLL for (int k = 0; k < 8; k++) f[k] = sg < n_adm ? adm[8 * (size_t)sg + k] : 0xFFFFFFFFu;
    store_row32_be(o.from32, j, f);
    gidx[j] = row.gidx;
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
    if (ctx->tally->host) (void)hipHostFree(ctx->tally->host);
    if (ctx->tally->scalar) (void)hipHostFree(ctx->tally->scalar);
    delete ctx->tally;
    ctx->tally = nullptr;
}

static inline uint32_t nblk(uint32_t n) { return (n + 255) / 256; }
// items per block of the order passes: the largest power of two in 256 ..
// HD_TALLY_IPB_MAX that leaves about four blocks per CU (a 128k-message batch
// at 2048 ran 63 blocks, latency-bound on a quarter of the chip)
static inline uint32_t tally_ipb(uint32_t m, uint32_t n_cu) {
    uint32_t ipb = HD_TALLY_IPB_MAX;
    while (ipb > 256u && (m + ipb - 1) / ipb < 4u * n_cu) ipb >>= 1;
    return ipb;
}

// dense log cells allowed (words): rounds numbered past nd = this / 2S take
// the hashed table (e.g. a batch of a million single-message rounds)
#define HD_TALLY_DENSE_MAX (64ull << 20)

// dup_global[gidx[j]] = dup[j] (a routed batch's classification at its
// global indices, in the owner's device memory: hd_multi)
__global__ __launch_bounds__(256) void k_dup_scatter(uint32_t n, const uint8_t* __restrict__ dup,
                                                     const uint32_t* __restrict__ gidx, uint8_t* __restrict__ dup_global) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) dup_global[gidx[j]] = dup[j];
}

// The first rows (at most capacities h, c of the column arrays at base) into
// out's arrays, starting at row (o_hr, o_cnt).
static void tally_unpack(const char* base, uint32_t h, uint32_t c, uint32_t n_hr, uint32_t n_cnt, hd_tally_out* out,
                         uint32_t o_hr = 0, uint32_t o_cnt = 0) {
    const TallyCols x = tally_cols(const_cast<char*>(base), h, c);
    auto put = [&](void* dst, size_t at, const void* src, size_t sz) {
        if (dst && sz) memcpy((char*)dst + at, src, sz);
    };
    put(out->hr_height, 8 * (size_t)o_hr, x.o_h, 8 * (size_t)n_hr);
    put(out->hr_round, 8 * (size_t)o_hr, x.o_r, 8 * (size_t)n_hr);
    put(out->hr_prevotes, 4 * (size_t)o_hr, x.o_prev, 4 * (size_t)n_hr);
    put(out->hr_precommits, 4 * (size_t)o_hr, x.o_prec, 4 * (size_t)n_hr);
    put(out->hr_any, 4 * (size_t)o_hr, x.o_any, 4 * (size_t)n_hr);
    put(out->hr_rep, 4 * (size_t)o_hr, x.o_rep, 4 * (size_t)n_hr);
    put(out->count_height, 8 * (size_t)o_cnt, x.c_h, 8 * (size_t)n_cnt);
    put(out->count_round, 8 * (size_t)o_cnt, x.c_r, 8 * (size_t)n_cnt);
    put(out->count_type, (size_t)o_cnt, x.c_t, (size_t)n_cnt);
    put(out->count_rep, 4 * (size_t)o_cnt, x.c_rep, 4 * (size_t)n_cnt);
    put(out->count_n, 4 * (size_t)o_cnt, x.c_n, 4 * (size_t)n_cnt);
}

// the stage layout: [n_hr, n_cnt | classification (n bytes, when staged) |
// per-round rows (32 B each, capacity h) | per-value rows (25 B each, capacity c)]
static size_t tally_rows_off(uint32_t n, bool dup) { return 64 + (((dup ? (size_t)n : 0) + 63) & ~(size_t)63); }
static size_t tally_stage_bytes(uint32_t n, bool dup, uint32_t h, uint32_t c) {
    return tally_rows_off(n, dup) + 32 * (size_t)h + 25 * (size_t)c + 64;
}

// HD_TALLY_CHECK: the invariants of the tables just built (k_tally_check_*),
// read back at once (a synchronisation: debug only)
static int tally_check(hd_ctx* ctx, const DevBatch& b, const uint32_t* cand, uint32_t m, uint32_t cap, GTab G,
                       CTab C, const uint32_t* D, const uint32_t* Dd, const TallyCtr* ctr, uint32_t per, uint32_t nd,
                       const uint32_t* gslot, const uint32_t* ref, hipStream_t s) {
    int rc = 0;
    TallyCheck* chk = (TallyCheck*)tbuf(ctx, T_CHECK, sizeof(TallyCheck), &rc);
    if (rc) return rc;
    TCHK(hipMemsetAsync(chk, 0, sizeof(TallyCheck), s), "tally check clear");
    const uint32_t grid = std::min<uint32_t>(nblk(std::max(m, cap)), (uint32_t)ctx->n_cu * 8u);
    k_tally_check_items<<<grid, 256, 0, s>>>(m, gslot, ref, Dd, D, chk);
    k_tally_check_cells<<<grid, 256, 0, s>>>(Dd, ctr, per, nd, m, ref, chk);
    k_tally_check_slots<<<grid, 256, 0, s>>>(b, cand, m, cap, G, C, D, Dd, gslot, ref, chk);
    TCHK(hipGetLastError(), "tally check kernels");
    TallyCheck h{};
    TCHK(hipMemcpyAsync(&h, chk, sizeof h, hipMemcpyDeviceToHost, s), "tally check download");
    TCHK(hipStreamSynchronize(s), "tally check sync");
    const bool ok = h.stale == 0 && h.bad_cell == 0 && h.dup_key == 0 && h.bad_claim == 0 && h.winners == h.sum_g &&
                    h.winners == h.sum_c && h.winners == h.cells + h.d_claims;
    if (ok) return HD_OK;
    char buf[320];
    snprintf(buf, sizeof buf,
             "tally check failed: winners %u, sum G %u, sum C %u, dense cells %u + D claims %u, stale %u, "
             "bad cells %u, duplicate keys %u, bad C claimers %u (m %u, cap %u)",
             h.winners, h.sum_g, h.sum_c, h.cells, h.d_claims, h.stale, h.bad_cell, h.dup_key, h.bad_claim, m, cap);
    ctx->last_error = buf;
    return HD_EDEVICE;
}

// HD_TALLY_CHECK after the emit: every table slot and the counters are clean
static int tally_check_clean(hd_ctx* ctx, uint32_t cap, const uint32_t* tabs, TallyCtr* ctr, hipStream_t s) {
    int rc = 0;
    uint32_t* bad = (uint32_t*)tbuf(ctx, T_CHECK, sizeof(TallyCheck), &rc);
    if (rc) return rc;
    TCHK(hipMemsetAsync(bad, 0, 4, s), "tally clean check clear");
    k_tally_check_clean<<<std::min<uint32_t>(nblk(cap), (uint32_t)ctx->n_cu * 8u), 256, 0, s>>>(cap, tabs, ctr, bad);
    uint32_t h = 0;
    TCHK(hipMemcpyAsync(&h, bad, 4, hipMemcpyDeviceToHost, s), "tally clean check download");
    TCHK(hipStreamSynchronize(s), "tally clean check sync");
    if (h == 0) return HD_OK;
    ctx->last_error = "tally check failed: " + std::to_string(h) + " table slots not clean after the emit";
    return HD_EDEVICE;
}

// gidx (optional): the batch's messages' global indices -- the rep outputs
// are mapped through it (a routed batch, hd_tally_routed_device); with
// dup_global the per-message classification is scattered there through gidx
// on the device instead of being downloaded (out->dup unused).  With `tk`
// (hd_tally_device_bitmap_async) nothing is waited for: the stage goes to the
// ticket's pinned buffer and hd_tally_collect unpacks it later.
//
// Launches per call: k_tally_rounds, k_tally_logs, k_tally_values,
// k_tally_firsts, k_tally_emit and one download (a partition adds its
// candidate compaction and one host read; a routed owner's scatter one
// kernel).  The hash tables and counters clean themselves (k_tally_emit), the
// dense cells are cleared by the round that takes them (k_tally_rounds), and
// the bitmaps are written whole: nothing is cleared per call unless the
// table capacity changed or an earlier call did not finish its launches.
// the device address of an async stage's completion word (word 2), or NULL
// when the stage is not mapped pinned memory (collect then waits on the event)
static uint32_t* ticket_signal(void* stage) {
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, stage, 0) != hipSuccess || !dp) {
        (void)hipGetLastError();
        return nullptr;
    }
    return reinterpret_cast<uint32_t*>(dp) + 2;
}

static int tally_device(hd_ctx* ctx, const hd_batch* hb, const uint8_t* d_verdict, const uint32_t* d_bitmap,
                        Part part, hd_tally_out* out, hipStream_t s, const uint32_t* gidx = nullptr,
                        uint8_t* dup_global = nullptr, hd_tally_ticket* tk = nullptr) {
    const uint32_t n = hb->n;
    if (!ctx->tally) ctx->tally = new TallyWork();
    DevBatch b{n, hb->type, hb->height, hb->round, hb->valid_round, hb->value32, hb->from32, hb->sig65};
    int rc = 0;
    // blocks per CU of the probe passes (HD_TALLY_BPC, default 16)
    static const uint32_t bpc = getenv("HD_TALLY_BPC") ? (uint32_t)std::max(1, atoi(getenv("HD_TALLY_BPC"))) : 16u;
    const bool check = [] {
        const char* e = getenv("HD_TALLY_CHECK");
        return e && atoi(e) != 0;
    }();
    // The output stage: [n_hr, n_cnt | per-message classification | per-round
    // rows (32 B each, capacity H) | per-value rows (25 B each, capacity Cg)],
    // downloaded with ONE copy after ONE host sync.  H and Cg are the previous
    // call's counts plus a margin; rows past them land in overflow columns on
    // the device, downloaded by a second round of copies when needed.
    TallyWork* tw = ctx->tally;
    // the classification is staged for download only when the caller reads it
    // (out->dup, or the ticket's dup); a routed owner's scatter (dup_global)
    // keeps it in device scratch of its own
    const bool stage_dup = tk ? tk->dup != 0 : out->dup != nullptr;
    const size_t dup_off = 64, rows_off = tally_rows_off(n, stage_dup);
    uint32_t H = tw->guess_hr, Cg = tw->guess_cnt;
    auto stage_bytes = [&](uint32_t h, uint32_t c) { return tally_stage_bytes(n, stage_dup, h, c); };
    if (tk) {
        if (part.nparts != 1 || gidx || dup_global) return HD_EINVAL;
        tk->n = n;
        tk->H = H;
        tk->Cg = Cg;
        tk->need = stage_bytes(H, Cg);
        if (!tk->stage || tk->stage_cap < tk->need) return HD_ECAP;
    }
    char* st = (char*)tbuf(ctx, T_SEL, stage_bytes(H, Cg), &rc);
    uint8_t* d_dup = stage_dup ? (uint8_t*)(st + dup_off) : nullptr;
    if (!stage_dup && dup_global) d_dup = (uint8_t*)tbuf(ctx, T_DUP, n, &rc);
    if (rc) return rc;
    // Items: the whole batch, or a partition's candidates compacted in batch
    // order (the rest of the tally then scales with the partition, not with
    // the replicated batch).
    uint32_t m = n;
    const uint32_t* cand = nullptr;
    if (part.nparts > 1) {
        uint32_t* at = (uint32_t*)tbuf(ctx, T_SORTK, 4 * (size_t)n, &rc);
        uint32_t* ccnt = (uint32_t*)tbuf(ctx, T_TMP, 4 * ((size_t)(n + HD_CHUNK - 1) / HD_CHUNK + 2), &rc);
        uint32_t* cl = (uint32_t*)tbuf(ctx, T_D, 4 * (size_t)n, &rc);
        if (rc) return rc;
        const uint32_t nch = (n + HD_CHUNK - 1) / HD_CHUNK;
        k_tally_flag<<<std::min<uint32_t>(nblk(n), (uint32_t)ctx->n_cu * 8u), 256, 0, s>>>(b, d_verdict, d_bitmap, part,
                                                                                            at, d_dup);
        k_tally_chunk_counts<<<nch, 256, 0, s>>>(n, at, ccnt);
        k_tally_chunk_write<<<nch, 256, 0, s>>>(n, at, ccnt, cl, nullptr, ccnt + nch);
        TCHK(hipGetLastError(), "tally candidate kernels");
        if (!tw->scalar) TCHK(hipHostMalloc((void**)&tw->scalar, 64, hipHostMallocDefault), "tally scalar");
        TCHK(hipMemcpyAsync(tw->scalar, ccnt + nch, 4, hipMemcpyDeviceToHost, s), "candidate count");
        TCHK(hipStreamSynchronize(s), "candidate count sync");
        m = tw->scalar[0];
        cand = cl;
    }
    if (m == 0) {   // nothing to tally here (dup: every message 3)
        out->n_hr = out->n_counts = 0;
        if (out->dup) memset(out->dup, 3, n);
        return HD_OK;
    }
    const uint32_t grid = std::min<uint32_t>(nblk(m), (uint32_t)ctx->n_cu * bpc);
    // the tables hold at most one key per item, load factor <= 1/2 so probes
    // terminate
    uint32_t cap = 1024;
    while (cap < 2 * m) cap <<= 1;
    const uint32_t mask = cap - 1;
    const uint32_t ipb = tally_ipb(m, (uint32_t)ctx->n_cu);
    const uint32_t nbo = (m + ipb - 1) / ipb;   // blocks of the order passes
    const size_t nw = (size_t)nbo * (ipb / 32);
    // one allocation for the tables: the claim words (G, C, D: empty), the
    // counters (G x 3, C: zero), the round numbers (gid); then the call
    // counters (TallyCtr)
    const size_t K = cap;
    char* tb = (char*)tbuf(ctx, T_G, 4 * 8 * K + sizeof(TallyCtr), &rc);
    uint32_t* gslot = (uint32_t*)tbuf(ctx, T_GSLOT, 4 * (size_t)m, &rc);
    uint32_t* ref = (uint32_t*)tbuf(ctx, T_DSLOT, 4 * (size_t)m, &rc);
    uint32_t* cslot = (uint32_t*)tbuf(ctx, T_CSLOT, 4 * (size_t)m, &rc);
    // Bg | Bc | pre_g | pre_c (nw words each) | block totals (2 nbo)
    uint32_t* bits = (uint32_t*)tbuf(ctx, T_BITS, 4 * (4 * nw + 2 * (size_t)nbo), &rc);
    // dense log cells (nd rounds x 2 x S) for admitted signatories, the hashed
    // D table for the rest: room for every item's round up to HD_TALLY_DENSE_MAX words
    const uint32_t S = ctx->n_adm;
    const size_t dcap = S > 0 ? std::min<size_t>(HD_TALLY_DENSE_MAX, (size_t)m * 2 * S) : 0;
    const uint32_t nd = S > 0 ? (uint32_t)(dcap / (2 * (size_t)S)) : 0u;
    uint32_t* Dd = dcap ? (uint32_t*)tbuf(ctx, T_C, 4 * dcap, &rc) : nullptr;
    if (rc) return rc;
    uint32_t* tabs = (uint32_t*)tb;
    GTab G{tabs, tabs + 3 * K, tabs + 4 * K, tabs + 5 * K, tabs + 7 * K};
    CTab C{tabs + K, tabs + 6 * K};
    uint32_t* d = tabs + 2 * K;
    TallyCtr* ctr = reinterpret_cast<TallyCtr*>(tb + 4 * 8 * K);
    if (tw->dirty || tw->tab_p != tb || tw->tab_k != cap) {   // first use, new capacity, or an unfinished call
        TCHK(hipMemsetAsync(tabs, 0xFF, 4 * 3 * K, s), "clear claims");
        TCHK(hipMemsetAsync(tabs + 3 * K, 0, 4 * 4 * K, s), "clear counters");
        TCHK(hipMemsetAsync(ctr, 0, sizeof(TallyCtr), s), "clear call counters");
        tw->tab_p = tb;
        tw->tab_k = cap;
    }
    tw->dirty = true;   // until every launch below is queued
    k_tally_rounds<<<grid, 256, 0, s>>>(b, cand, m, d_verdict, d_bitmap, part, G, mask, gslot, d_dup, ctr, Dd, 2 * S,
                                        nd);
    k_tally_logs<<<grid, 256, 0, s>>>(b, cand, m, gslot, G.gid, hd_adm_index(ctx), S, Dd, nd, d, mask, ref);
    k_tally_values<<<grid, 256, 0, s>>>(b, cand, m, Dd, S, d, G, C, mask, gslot, ref, cslot, d_dup);
    if (dup_global && gidx) k_dup_scatter<<<nblk(n), 256, 0, s>>>(n, d_dup, gidx, dup_global);
    TCHK(hipGetLastError(), "tally kernels");
    if (check) {
        rc = tally_check(ctx, b, cand, m, cap, G, C, d, Dd, ctr, 2 * S, nd, gslot, ref, s);
        if (rc) return rc;
    }
    uint32_t *Bg = bits, *Bc = bits + nw, *pre_g = bits + 2 * nw, *pre_c = bits + 3 * nw, *blk = bits + 4 * nw;
    // rows at capacity (H, Cg) in the stage, the rest in the overflow columns
    // (capacity m each: a batch has at most m groups of either kind)
    char* ovf = (char*)tbuf(ctx, T_NSEL, 57 * (size_t)m + 64, &rc);
    if (rc) return rc;
    const TallyCols sc = tally_cols(st + rows_off, H, Cg), oc = tally_cols(ovf, m, m);
    switch (ipb) {
#define HD_TALLY_ORDER(IPB)                                                                                         \
    case IPB:                                                                                                       \
        k_tally_firsts<IPB><<<nbo, 256, 0, s>>>(m, gslot, cslot, G.claim, C.claim, Bg, Bc, pre_g, pre_c, blk);       \
        k_tally_emit<IPB><<<nbo, 256, 0, s>>>(b, cand, m, gidx, gslot, cslot, ref, G, C, d, Bg, Bc, pre_g, pre_c, blk, \
                                              sc, H, Cg, oc, ctr, (uint32_t*)st);                                   \
        break;
        HD_TALLY_ORDER(256u)
        HD_TALLY_ORDER(512u)
        HD_TALLY_ORDER(1024u)
        HD_TALLY_ORDER(2048u)
#undef HD_TALLY_ORDER
    }
    TCHK(hipGetLastError(), "tally order kernels");
    tw->dirty = false;
    if (check) {
        rc = tally_check_clean(ctx, cap, tabs, ctr, s);
        if (rc) return rc;
    }
    const size_t total = stage_bytes(H, Cg);
    if (tk) {   // queued; hd_tally_collect waits for the signal (or tk->done), then reads the stage
        // the completion word restarts at 0 (the stage's previous ticket was collected)
        reinterpret_cast<volatile uint32_t*>(tk->stage)[2] = 0u;
        TCHK(hipMemcpyAsync(tk->stage, st, total, hipMemcpyDeviceToHost, s), "tally download");
        if (uint32_t* sig = ticket_signal(tk->stage)) k_tally_signal<<<1, 64, 0, s>>>(sig);
        if (!tk->done) TCHK(hipEventCreateWithFlags((hipEvent_t*)&tk->done, hipEventDisableTiming), "tally event");
        TCHK(hipEventRecord((hipEvent_t)tk->done, s), "tally event record");
        return hd_ctx_note_stream(ctx, s);
    }
    if (tw->host_cap < total) {
        if (tw->host) (void)hipHostFree(tw->host);
        tw->host = nullptr;
        tw->host_cap = 0;
        TCHK(hipHostMalloc(&tw->host, total + (total >> 2), hipHostMallocDefault), "tally host stage");
        tw->host_cap = total + (total >> 2);
    }
    TCHK(hipMemcpyAsync(tw->host, st, total, hipMemcpyDeviceToHost, s), "tally download");
    TCHK(hipStreamSynchronize(s), "tally sync");
    const uint32_t n_hr = reinterpret_cast<const uint32_t*>(tw->host)[0];
    const uint32_t n_cnt = reinterpret_cast<const uint32_t*>(tw->host)[1];
    out->n_hr = n_hr;
    out->n_counts = n_cnt;
    tw->guess_hr = std::max<uint32_t>(1024u, n_hr + n_hr / 4);
    tw->guess_cnt = std::max<uint32_t>(1024u, n_cnt + n_cnt / 4);
    if (n_hr > out->cap_hr || n_cnt > out->cap_counts) return HD_ECAP;
    if (out->dup) memcpy(out->dup, (const char*)tw->host + dup_off, (size_t)n);
    tally_unpack((const char*)tw->host + rows_off, H, Cg, std::min(n_hr, H), std::min(n_cnt, Cg), out);
    if (n_hr > H || n_cnt > Cg) {   // more groups than staged: the overflow columns, straight into out
        const uint32_t eh = n_hr > H ? n_hr - H : 0, ec = n_cnt > Cg ? n_cnt - Cg : 0;
        struct Piece {
            void* dst;
            const void* src;
            size_t sz;
        } pieces[] = {
            {out->hr_height ? out->hr_height + H : nullptr, oc.o_h, 8 * (size_t)eh},
            {out->hr_round ? out->hr_round + H : nullptr, oc.o_r, 8 * (size_t)eh},
            {out->hr_prevotes ? out->hr_prevotes + H : nullptr, oc.o_prev, 4 * (size_t)eh},
            {out->hr_precommits ? out->hr_precommits + H : nullptr, oc.o_prec, 4 * (size_t)eh},
            {out->hr_any ? out->hr_any + H : nullptr, oc.o_any, 4 * (size_t)eh},
            {out->hr_rep ? out->hr_rep + H : nullptr, oc.o_rep, 4 * (size_t)eh},
            {out->count_height ? out->count_height + Cg : nullptr, oc.c_h, 8 * (size_t)ec},
            {out->count_round ? out->count_round + Cg : nullptr, oc.c_r, 8 * (size_t)ec},
            {out->count_type ? out->count_type + Cg : nullptr, oc.c_t, (size_t)ec},
            {out->count_rep ? out->count_rep + Cg : nullptr, oc.c_rep, 4 * (size_t)ec},
            {out->count_n ? out->count_n + Cg : nullptr, oc.c_n, 4 * (size_t)ec},
        };
        for (const Piece& p : pieces)
            if (p.dst && p.sz) TCHK(hipMemcpyAsync(p.dst, p.src, p.sz, hipMemcpyDeviceToHost, s), "tally overflow");
        TCHK(hipStreamSynchronize(s), "tally overflow sync");
    }
    return HD_OK;
}

// hd_tally_routed_device with the classification scattered, on the device,
// to dup_global[global index] (n_global bytes the caller set to 3) instead of
// being downloaded (hd_multi.hip)
int hd_tally_routed_dup_device(hd_ctx* ctx, const hd_batch* dbatch, const uint32_t* d_gidx, hd_tally_out* out,
                               uint8_t* dup_global, hipStream_t s) {
    out->n_counts = out->n_hr = 0;
    if (dbatch->n == 0) return HD_OK;
    uint8_t* keep = out->dup;
    out->dup = nullptr;
    const int rc = tally_device(ctx, dbatch, nullptr, nullptr, Part{0, 1}, out, s, d_gidx, dup_global);
    out->dup = keep;
    return rc;
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

int hd_tally_device_bitmap_async(hd_ctx* ctx, const hd_batch* dbatch, const uint32_t* d_valid_bitmap,
                                 hd_tally_ticket* ticket, void* stream) {
    if (!ctx || !dbatch || !ticket) return HD_EINVAL;
    if (dbatch->n && !d_valid_bitmap) return HD_EINVAL;
    ticket->n = dbatch->n;
    ticket->H = ticket->Cg = 0;
    ticket->need = 0;
    if (dbatch->n == 0) return HD_OK;
    (void)hipSetDevice(ctx->device);
    hd_tally_out dummy{};
    return tally_device(ctx, dbatch, nullptr, d_valid_bitmap, Part{0, 1}, &dummy,
                        stream ? (hipStream_t)stream : ctx->stream, nullptr, nullptr, ticket);
}

int hd_tally_ticket_release(hd_tally_ticket* ticket) {
    if (!ticket) return HD_EINVAL;
    if (ticket->done) (void)hipEventDestroy((hipEvent_t)ticket->done);
    ticket->done = nullptr;
    return HD_OK;
}

size_t hd_tally_stage_bytes(hd_ctx* ctx, uint32_t n, int dup) {
    if (!ctx) return 0;
    const uint32_t h = ctx->tally ? ctx->tally->guess_hr.load() : 1024u, c = ctx->tally ? ctx->tally->guess_cnt.load() : 1024u;
    return tally_stage_bytes(n, dup != 0, h, c);
}

int hd_tally_collect(hd_ctx* ctx, const hd_tally_ticket* ticket, hd_tally_out* out) {
    if (!ctx || !ticket || !tally_out_ok(out)) return HD_EINVAL;
    out->n_counts = out->n_hr = 0;
    if (ticket->n == 0) return HD_OK;
    if (!ticket->stage || ticket->need == 0 || !ticket->done) return HD_EINVAL;
    (void)hipSetDevice(ctx->device);
    if (ticket_signal(ticket->stage)) {
        // poll the completion word without a HIP call per iteration; past
        // ~0.2 s, wait for the event (a fault surfaces there) and read it once more
        volatile const uint32_t* w = reinterpret_cast<volatile const uint32_t*>(ticket->stage) + 2;
        const auto t0 = std::chrono::steady_clock::now();
        while (*w != 1u) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                TCHK(hipEventSynchronize((hipEvent_t)ticket->done), "tally collect wait");
                if (*w != 1u) return hd_ctx_fail(ctx, hipErrorUnknown, "tally collect signal");
                break;
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    } else {
        TCHK(hipEventSynchronize((hipEvent_t)ticket->done), "tally collect wait");
    }
    const char* st = (const char*)ticket->stage;
    const uint32_t n_hr = reinterpret_cast<const uint32_t*>(st)[0];
    const uint32_t n_cnt = reinterpret_cast<const uint32_t*>(st)[1];
    out->n_hr = n_hr;
    out->n_counts = n_cnt;
    if (!ctx->tally) ctx->tally = new TallyWork();
    TallyWork* tw = ctx->tally;
    tw->guess_hr = std::max<uint32_t>(tw->guess_hr.load(), std::max<uint32_t>(1024u, n_hr + n_hr / 4));
    tw->guess_cnt = std::max<uint32_t>(tw->guess_cnt.load(), std::max<uint32_t>(1024u, n_cnt + n_cnt / 4));
    if (n_hr > out->cap_hr || n_cnt > out->cap_counts) return HD_ECAP;
    if (n_hr > ticket->H || n_cnt > ticket->Cg) return HD_EAGAIN;   // more groups than staged
    if (out->dup) {
        if (!ticket->dup) return HD_EINVAL;
        memcpy(out->dup, st + 64, (size_t)ticket->n);
    }
    tally_unpack(st + tally_rows_off(ticket->n, ticket->dup != 0), ticket->H, ticket->Cg, n_hr, n_cnt, out);
    return HD_OK;
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

static int route_candidates(hd_ctx* ctx, const hd_batch* dshard, const uint32_t* d_valid_bitmap,
                            uint32_t base_index, uint32_t nparts, RoundList rl, uint8_t* d_rows, uint32_t cap_rows,
                            uint32_t* counts, void* stream);

int hd_route_candidates_device(hd_ctx* ctx, const hd_batch* dshard, const uint32_t* d_valid_bitmap,
                               uint32_t base_index, uint32_t nparts, uint8_t* d_rows, uint32_t cap_rows,
                               uint32_t* counts, void* stream) {
    return route_candidates(ctx, dshard, d_valid_bitmap, base_index, nparts, RoundList{nullptr, nullptr, 0}, d_rows,
                            cap_rows, counts, stream);
}

int hd_route_candidates_listed_device(hd_ctx* ctx, const hd_batch* dshard, const uint32_t* d_valid_bitmap,
                                      uint32_t base_index, uint32_t nparts, const int64_t* d_round_h,
                                      const int64_t* d_round_r, uint32_t n_rounds, uint8_t* d_rows,
                                      uint32_t cap_rows, uint32_t* counts, void* stream) {
    if (!ctx || !counts || nparts == 0 || nparts > HD_ROUTE_MAX_PARTS) return HD_EINVAL;
    if (n_rounds == 0) {   // nothing is shared: nothing to route
        for (uint32_t o = 0; o < nparts; o++) counts[o] = 0;
        return HD_OK;
    }
    if (!d_round_h || !d_round_r) return HD_EINVAL;
    return route_candidates(ctx, dshard, d_valid_bitmap, base_index, nparts, RoundList{d_round_h, d_round_r, n_rounds},
                            d_rows, cap_rows, counts, stream);
}

}  // extern "C"

static int route_candidates(hd_ctx* ctx, const hd_batch* dshard, const uint32_t* d_valid_bitmap,
                            uint32_t base_index, uint32_t nparts, RoundList rl, uint8_t* d_rows, uint32_t cap_rows,
                            uint32_t* counts, void* stream) {
    if (!ctx || !dshard || !counts || nparts == 0 || nparts > HD_ROUTE_MAX_PARTS) return HD_EINVAL;
    for (uint32_t o = 0; o < nparts; o++) counts[o] = 0;
    const uint32_t n = dshard->n;
    if (n == 0) return HD_OK;
    if (!d_valid_bitmap || !d_rows || !dshard->type || !dshard->height || !dshard->round || !dshard->value32 ||
        !dshard->from32 || ((uintptr_t)d_rows & 15) || ((uintptr_t)dshard->value32 & 15))
        return HD_EINVAL;
    (void)hipSetDevice(ctx->device);
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    if (!ctx->tally) ctx->tally = new TallyWork();
    DevBatch b{n, dshard->type, dshard->height, dshard->round, nullptr, dshard->value32, dshard->from32, nullptr};
    const uint32_t nb = nblk(n);
    const size_t cells = (size_t)nparts * nb;
    int rc = 0;
    // starts[0 .. nparts] and, after them, the count of candidates outside the set
    uint32_t* cnt = (uint32_t*)tbuf(ctx, T_ROUTE, 4 * (2 * cells + nparts + 2) + 4096, &rc);
    if (rc) return rc;
    uint32_t* off = cnt + cells;
    uint32_t* starts = off + cells;
    void* tmp = (void*)(starts + nparts + 2);
    size_t tmp_bytes = 0;
    TCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt, off, (int)cells, s), "route scan size");
    // the scan's temporary storage after the counts (grown with them)
    cnt = (uint32_t*)tbuf(ctx, T_ROUTE, 4 * (2 * cells + nparts + 2) + 64 + tmp_bytes, &rc);
    if (rc) return rc;
    off = cnt + cells;
    starts = off + cells;
    tmp = (void*)(((uintptr_t)(starts + nparts + 2) + 63) & ~(uintptr_t)63);
    TCHK(hipMemsetAsync(starts + nparts + 1, 0, 4, s), "route outside count");
    k_route_count<<<nb, 256, 0, s>>>(b, d_valid_bitmap, nparts, hd_adm_index(ctx), ctx->n_adm, cnt,
                                     starts + nparts + 1, rl);
    TCHK(hipGetLastError(), "k_route_count");
    TCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, cnt, off, (int)cells, s), "route scan");
    k_route_starts<<<1, 64, 0, s>>>(off, cnt, nparts, nb, starts);
    std::vector<uint32_t> st(nparts + 2);
    TCHK(hipMemcpyAsync(st.data(), starts, 4 * (nparts + 2), hipMemcpyDeviceToHost, s), "route counts");
    TCHK(hipStreamSynchronize(s), "route counts");
    if (st[nparts + 1]) {
        // a VALID candidate whose From left the set since verification: its
        // row could not name it (the tally keys on the From), so refuse
        ctx->last_error = "hd_route_candidates_device: " + std::to_string(st[nparts + 1]) +
                          " candidates whose From is not in the current admitted set";
        return HD_EINVAL;
    }
    for (uint32_t o = 0; o < nparts; o++) counts[o] = st[o + 1] - st[o];
    if (st[nparts] > cap_rows) return HD_ECAP;
    k_route_write<<<nb, 256, 0, s>>>(b, d_valid_bitmap, nparts, base_index, off, hd_adm_index(ctx), ctx->n_adm,
                                     reinterpret_cast<RouteRow*>(d_rows), rl);
    TCHK(hipGetLastError(), "k_route_write");
    return hd_ctx_note_stream(ctx, s);
}

extern "C" {

int hd_unroute_device(hd_ctx* ctx, const uint8_t* d_rows, uint32_t n, const hd_batch_out* d_out, uint32_t* d_gidx,
                      void* stream) {
    if (!ctx || !d_out) return HD_EINVAL;
    if (n == 0) return HD_OK;
    if (!d_rows || !d_gidx || !d_out->type || !d_out->height || !d_out->round || !d_out->value32 || !d_out->from32 ||
        ((uintptr_t)d_rows & 15) || ((uintptr_t)d_out->value32 & 15) || ((uintptr_t)d_out->from32 & 15))
        return HD_EINVAL;
    (void)hipSetDevice(ctx->device);
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    k_unroute<<<nblk(n), 256, 0, s>>>(reinterpret_cast<const RouteRow*>(d_rows), n, ctx->d_adm, ctx->n_adm, *d_out,
                                      d_gidx);
    TCHK(hipGetLastError(), "k_unroute");
    return hd_ctx_note_stream(ctx, s);
}

int hd_tally_routed_device(hd_ctx* ctx, const hd_batch* dbatch, const uint32_t* d_gidx, hd_tally_out* out,
                           void* stream) {
    if (!ctx || !dbatch || !tally_out_ok(out)) return HD_EINVAL;
    out->n_counts = out->n_hr = 0;
    if (dbatch->n == 0) return HD_OK;
    if (!d_gidx) return HD_EINVAL;
    (void)hipSetDevice(ctx->device);
    return tally_device(ctx, dbatch, nullptr, nullptr, Part{0, 1}, out, stream ? (hipStream_t)stream : ctx->stream,
                        d_gidx);
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
