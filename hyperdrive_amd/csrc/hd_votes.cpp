// Incremental vote logs and count table of one height (include/hd_votes.h),
// SURVEY §8(f)1.  Host C++ only.
//
// Signatories seen at the height are interned to dense ids (one small, hot
// open-addressing table keyed by the 32-byte From).  Per round (process.go
// keys its logs by Round) and vote type: the logged vote of each signatory id
// (value slot, batch origin) in a dense array, the interned distinct values
// of that (round, type) with their vote counts, and the log length; per round
// the TraceLogs membership by id and its size.  Insert = one probe of the id
// table + one probe of the (round, type) value table; every query is O(1).
// The reference's equivalent state is process/state.go:44-57, the rules it
// serves process.go:486-491, 534, 574-579, 626-631, 658, 696-701, 751.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <new>
#include <random>
#include <unordered_map>
#include <vector>

#include "hd_votes.h"

namespace {

struct Key32 {
    uint64_t w[4];
    static Key32 load(const uint8_t* p) {
        Key32 k;
        memcpy(k.w, p, 32);
        return k;
    }
    bool operator==(const Key32& o) const {
        return ((w[0] ^ o.w[0]) | (w[1] ^ o.w[1]) | (w[2] ^ o.w[2]) | (w[3] ^ o.w[3])) == 0;
    }
};

// per-process random seed: values are sender-chosen bytes, so bucket placement
// must not be predictable from the key alone
uint64_t g_seed = [] {
    std::random_device rd;
    return (uint64_t(rd()) << 32) ^ rd() ^ 0x9E3779B97F4A7C15ull;
}();

inline uint64_t hash32(const Key32& k) {
    const unsigned __int128 a = (unsigned __int128)(k.w[0] ^ g_seed) * (k.w[1] ^ 0xA0761D6478BD642Full);
    const unsigned __int128 b = (unsigned __int128)(k.w[2] ^ 0xE7037ED1A0B428DBull) * (k.w[3] ^ g_seed ^ 0x8EBC6AF09C88C6E3ull);
    const uint64_t x = uint64_t(a) ^ uint64_t(a >> 64) ^ uint64_t(b) ^ uint64_t(b >> 64);
    return x ^ (x >> 29);
}

// open addressing, linear probing, load <= 1/2; V is trivially copyable
template <class V>
class Flat32 {
  public:
    size_t size() const { return n_; }

    V* find(const Key32& k) {
        if (n_ == 0) return nullptr;
        for (size_t i = hash32(k) & mask_;; i = (i + 1) & mask_) {
            if (!used_[i]) return nullptr;
            if (keys_[i] == k) return &vals_[i];
        }
    }
    const V* find(const Key32& k) const { return const_cast<Flat32*>(this)->find(k); }

    // returns the slot for k; *fresh = true when k was absent (slot value unset)
    V* insert(const Key32& k, bool* fresh) {
        if (2 * (n_ + 1) > keys_.size()) grow();
        size_t i = hash32(k) & mask_;
        for (; used_[i]; i = (i + 1) & mask_)
            if (keys_[i] == k) {
                *fresh = false;
                return &vals_[i];
            }
        used_[i] = 1;
        keys_[i] = k;
        ++n_;
        *fresh = true;
        return &vals_[i];
    }

    // empty, keeping the allocation
    void clear() {
        if (n_) memset(used_.data(), 0, used_.size());
        n_ = 0;
    }

  private:
    void grow() {
        const size_t cap = keys_.empty() ? 16 : 2 * keys_.size();
        std::vector<Key32> ok;
        std::vector<V> ov;
        std::vector<uint8_t> ou;
        ok.swap(keys_);
        ov.swap(vals_);
        ou.swap(used_);
        keys_.resize(cap);
        vals_.resize(cap);
        used_.assign(cap, 0);
        mask_ = cap - 1;
        for (size_t j = 0; j < ou.size(); ++j) {
            if (!ou[j]) continue;
            size_t i = hash32(ok[j]) & mask_;
            while (used_[i]) i = (i + 1) & mask_;
            used_[i] = 1;
            keys_[i] = ok[j];
            vals_[i] = ov[j];
        }
    }

    std::vector<Key32> keys_;
    std::vector<V> vals_;
    std::vector<uint8_t> used_;
    size_t n_ = 0, mask_ = 0;
};

struct Logged {
    uint32_t slot;    // 1 + index into TypeLog::values / counts; 0 = no vote
    uint32_t origin;  // batch index of the insert
    uint32_t epoch;   // insert call it came from
};

// grow-on-demand dense array indexed by signatory id (zero-filled)
template <class T>
inline T& at(std::vector<T>& a, uint32_t i) {
    if (i >= a.size()) a.resize(std::max<size_t>(size_t(i) + 1, 2 * a.size()));
    return a[i];
}

// PrevoteLogs[r] or PrecommitLogs[r] plus the per-value counts of that log
struct TypeLog {
    std::vector<Logged> by_signer;  // indexed by the height's signatory id
    uint32_t len = 0;               // len(PrevoteLogs[r])
    Flat32<uint32_t> slot_of_value;
    std::vector<Key32> values;
    std::vector<uint32_t> counts;

    void clear() {
        std::fill(by_signer.begin(), by_signer.end(), Logged{0, 0, 0});
        len = 0;
        slot_of_value.clear();
        values.clear();
        counts.clear();
    }
};

struct RoundLog {
    TypeLog t[2];                 // [0] Prevote, [1] Precommit
    std::vector<uint8_t> traced;  // TraceLogs[r], by signatory id
    uint32_t trace_len = 0;

    void clear() {
        t[0].clear();
        t[1].clear();
        std::fill(traced.begin(), traced.end(), 0);
        trace_len = 0;
    }
    // true when `id` is new to the trace
    bool trace(uint32_t id) {
        uint8_t& b = at(traced, id);
        const bool fresh = !b;
        trace_len += fresh;
        b = 1;
        return fresh;
    }
};

inline int type_ix(uint8_t type) {
    return type == HD_TYPE_PREVOTE ? 0 : type == HD_TYPE_PRECOMMIT ? 1 : -1;
}

}  // namespace

struct hd_votes {
    int64_t height = 0;
    uint32_t epoch = 0;
    uint32_t f = UINT32_MAX;     // quorum events off until hd_votes_set_f
    // signatories seen at this height -> dense id; the per-round logs are
    // arrays over these ids, so a vote costs one probe of this (small, hot)
    // table instead of probes of per-round tables keyed by 32-byte From
    Flat32<uint32_t> signatory_id;
    std::unordered_map<int64_t, RoundLog*> rounds;
    std::vector<std::unique_ptr<RoundLog>> pool;  // every RoundLog ever made
    size_t pool_used = 0;                          // pool[0, pool_used) are in `rounds`
    int64_t last_round = 0;
    RoundLog* last = nullptr;

    RoundLog* get(int64_t r) const {
        if (last && r == last_round) return last;
        auto it = rounds.find(r);
        return it == rounds.end() ? nullptr : it->second;
    }

    RoundLog* get_or_make(int64_t r) {
        if (last && r == last_round) return last;
        auto it = rounds.find(r);
        RoundLog* l;
        if (it != rounds.end()) {
            l = it->second;
        } else {
            if (pool_used == pool.size()) pool.emplace_back(new RoundLog());
            l = pool[pool_used++].get();
            rounds.emplace(r, l);
        }
        last_round = r;
        last = l;
        return l;
    }

    uint32_t id_of(const Key32& from) {
        bool fresh;
        uint32_t* id = signatory_id.insert(from, &fresh);
        if (fresh) *id = uint32_t(signatory_id.size() - 1);
        return *id;
    }
    // UINT32_MAX when `from` has not been seen at this height
    uint32_t find_id(const Key32& from) const {
        const uint32_t* id = signatory_id.find(from);
        return id ? *id : UINT32_MAX;
    }

    void reset(int64_t h) {
        for (size_t i = 0; i < pool_used; ++i) pool[i]->clear();
        pool_used = 0;
        rounds.clear();
        signatory_id.clear();
        last = nullptr;
        height = h;
    }

    // insertPrevote / insertPrecommit (process.go:823-855, 860-892)
    uint8_t insert(int ti, int64_t h, int64_t r, const Key32& value, const Key32& from, uint32_t origin,
                   const Logged** prior, uint8_t* ev) {
        *ev = 0;
        if (h != height) return HD_VOTE_WRONG_HEIGHT;
        RoundLog* l = get_or_make(r);
        TypeLog& t = l->t[ti];
        const uint32_t id = id_of(from);
        Logged& e = at(t.by_signer, id);
        if (e.slot) {
            *prior = &e;
            return t.values[e.slot - 1] == value ? HD_VOTE_DUPLICATE : HD_VOTE_DOUBLE;
        }
        bool vfresh;
        uint32_t* s = t.slot_of_value.insert(value, &vfresh);
        if (vfresh) {
            *s = uint32_t(t.values.size());
            t.values.push_back(value);
            t.counts.push_back(0);
        }
        t.counts[*s]++;
        t.len++;
        e = Logged{*s + 1, origin, epoch};
        const bool traced = l->trace(id);
        if (f != UINT32_MAX) {
            if (t.len == 2 * (uint64_t)f + 1) *ev |= ti == 0 ? HD_VOTE_EV_PREVOTE_2F1 : HD_VOTE_EV_PRECOMMIT_2F1;
            if (traced && l->trace_len == (uint64_t)f + 1) *ev |= HD_VOTE_EV_TRACE_F1;
        }
        return HD_VOTE_INSERTED;
    }

    const Logged* logged(int ti, int64_t r, const Key32& from) const {
        const RoundLog* l = get(r);
        const uint32_t id = find_id(from);
        if (!l || id == UINT32_MAX || id >= l->t[ti].by_signer.size()) return nullptr;
        const Logged& e = l->t[ti].by_signer[id];
        return e.slot ? &e : nullptr;
    }
};

#define HD_TRY_ALLOC(stmt)                 \
    try {                                  \
        stmt;                              \
    } catch (const std::bad_alloc&) {      \
        return HD_ENOMEM;                  \
    }

extern "C" {

int hd_votes_create(int64_t height, hd_votes** out) {
    if (!out) return HD_EINVAL;
    *out = nullptr;
    hd_votes* v = new (std::nothrow) hd_votes();
    if (!v) return HD_ENOMEM;
    v->height = height;
    *out = v;
    return HD_OK;
}

int hd_votes_set_f(hd_votes* v, uint32_t f) {
    if (!v) return HD_EINVAL;
    v->f = f;
    return HD_OK;
}

int hd_votes_destroy(hd_votes* v) {
    delete v;
    return HD_OK;
}

int hd_votes_reset(hd_votes* v, int64_t height) {
    if (!v) return HD_EINVAL;
    v->reset(height);
    return HD_OK;
}

int hd_votes_height(const hd_votes* v, int64_t* height) {
    if (!v || !height) return HD_EINVAL;
    *height = v->height;
    return HD_OK;
}

int hd_votes_insert(hd_votes* v, uint8_t type, int64_t height, int64_t round, const uint8_t* value32,
                    const uint8_t* from32, uint8_t* status, uint8_t* existing_value32, uint8_t* events) {
    const int ti = type_ix(type);
    if (!v || ti < 0 || !value32 || !from32 || !status) return HD_EINVAL;
    const Logged* prior = nullptr;
    uint8_t ev = 0;
    v->epoch++;
    HD_TRY_ALLOC(*status = v->insert(ti, height, round, Key32::load(value32), Key32::load(from32), UINT32_MAX,
                                     &prior, &ev));
    if (events) *events = ev;
    if (*status == HD_VOTE_DOUBLE && existing_value32)
        memcpy(existing_value32, v->get(round)->t[ti].values[prior->slot - 1].w, 32);
    return HD_OK;
}

int hd_votes_insert_batch(hd_votes* v, const hd_batch* b, const uint8_t* verdict, uint8_t* status,
                          uint32_t* double_of, uint8_t* events, uint32_t* n_inserted) {
    if (!v || !b) return HD_EINVAL;
    if (b->n && (!b->type || !b->height || !b->round || !b->value32 || !b->from32)) return HD_EINVAL;
    const uint32_t epoch = ++v->epoch;
    uint32_t ins = 0;
    for (uint32_t i = 0; i < b->n; ++i) {
        uint8_t st, ev = 0;
        uint32_t dof = UINT32_MAX;
        const int ti = type_ix(b->type[i]);
        if (verdict && verdict[i] != HD_VERDICT_VALID) {
            st = HD_VOTE_SKIPPED;
        } else if (ti < 0) {
            st = HD_VOTE_NOT_VOTE;
        } else {
            const Logged* prior = nullptr;
            HD_TRY_ALLOC(st = v->insert(ti, b->height[i], b->round[i], Key32::load(b->value32 + 32 * size_t(i)),
                                        Key32::load(b->from32 + 32 * size_t(i)), i, &prior, &ev));
            if (st == HD_VOTE_INSERTED) ins++;
            if (st == HD_VOTE_DOUBLE && prior->epoch == epoch) dof = prior->origin;
        }
        if (status) status[i] = st;
        if (double_of) double_of[i] = dof;
        if (events) events[i] = ev;
    }
    if (n_inserted) *n_inserted = ins;
    return HD_OK;
}

int hd_votes_trace_propose(hd_votes* v, int64_t round, const uint8_t* from32, uint8_t* events) {
    if (!v || !from32) return HD_EINVAL;
    RoundLog* l = nullptr;
    bool fresh = false;
    HD_TRY_ALLOC(l = v->get_or_make(round); fresh = l->trace(v->id_of(Key32::load(from32))));
    if (events) *events = (fresh && v->f != UINT32_MAX && l->trace_len == (uint64_t)v->f + 1) ? HD_VOTE_EV_TRACE_F1 : 0;
    return HD_OK;
}

int hd_votes_count(const hd_votes* v, uint8_t type, int64_t round, const uint8_t* value32, uint32_t* n) {
    const int ti = type_ix(type);
    if (!v || ti < 0 || !value32 || !n) return HD_EINVAL;
    *n = 0;
    const RoundLog* l = v->get(round);
    if (!l) return HD_OK;
    const uint32_t* s = l->t[ti].slot_of_value.find(Key32::load(value32));
    if (s) *n = l->t[ti].counts[*s];
    return HD_OK;
}

int hd_votes_len(const hd_votes* v, uint8_t type, int64_t round, uint32_t* n) {
    const int ti = type_ix(type);
    if (!v || ti < 0 || !n) return HD_EINVAL;
    const RoundLog* l = v->get(round);
    *n = l ? l->t[ti].len : 0;
    return HD_OK;
}

int hd_votes_trace_len(const hd_votes* v, int64_t round, uint32_t* n) {
    if (!v || !n) return HD_EINVAL;
    const RoundLog* l = v->get(round);
    *n = l ? l->trace_len : 0;
    return HD_OK;
}

int hd_votes_get(const hd_votes* v, uint8_t type, int64_t round, const uint8_t* from32, uint8_t* value32,
                 int* found) {
    const int ti = type_ix(type);
    if (!v || ti < 0 || !from32 || !found) return HD_EINVAL;
    *found = 0;
    const Logged* e = v->logged(ti, round, Key32::load(from32));
    if (!e) return HD_OK;
    *found = 1;
    if (value32) memcpy(value32, v->get(round)->t[ti].values[e->slot - 1].w, 32);
    return HD_OK;
}

}  // extern "C"
