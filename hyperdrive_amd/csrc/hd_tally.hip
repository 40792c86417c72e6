// hd_tally.hip -- GPU tally of authenticated votes: the first-wins vote logs
// of process/process.go:823-892 and the counts the 2f+1 / f+1 rules read
// (process.go:486-494, 534, 574-582, 626-632, 658, 696-702, 751), for every
// (height, round) in a batch at once.
//
// Pipeline (m = VALID Prevote/Precommit candidates, kept in batch order):
//   1. compact candidates                      (hipcub DeviceSelect)
//   2. stable LSD sort by (h, r, signer, type)  (3 hipcub radix passes; stable,
//      so inside a (h, r, signer, type) group the lowest batch index leads --
//      that element is the first-wins log entry)
//   3. k_mark: group heads -> winners, (h, r) segments, (h, r, signer) heads
//   4. per (h, r): distinct prevote / precommit signers and distinct signers
//      over both types -- wavefront-shuffle segmented reduction, one atomic
//      per segment per wavefront step (integer adds: order-independent, so the
//      result is deterministic)
//   5. winners sorted by (h, r, type, value bytes) (5 radix passes), run-length
//      groups -> count[(h, r, type, value)] by the same segmented reduction.
//   6. duplicates: a non-winner with the winner's value is an identical
//      duplicate (dropped silently); with another value it is the double vote
//      the reference hands to Catcher.CatchDoublePrevote/Precommit.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "hd_internal.h"
#include "hd_verify_msg.h"

using namespace hd;

struct TallyWork {
    DevBuf b[24];
};
enum TSlot {
    T_FLAG, T_CAND0, T_CAND1, T_K32A, T_K32B, T_K64A, T_K64B, T_NSEL, T_TMP, T_SIGNER, T_FHR, T_FHRS, T_FKEY,
    T_HRID, T_HEAD, T_WIN0, T_WIN1, T_HRMSG, T_GHEAD, T_GID, T_OUTHR, T_OUTCNT, T_DUP, T_VERD
};

static const uint64_t kSign = 0x8000000000000000ull;

// ---------------------------------------------------------------- kernels
__global__ void k_cand_flags(uint32_t n, const uint8_t* __restrict__ verdict, const uint8_t* __restrict__ type,
                             uint8_t* __restrict__ flag, uint8_t* __restrict__ dup) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t t = type[i];
    flag[i] = (verdict[i] == V_VALID && (t == T_PREVOTE || t == T_PRECOMMIT)) ? 1 : 0;
    if (dup) dup[i] = 3;
}

__global__ void k_cand_flags_bitmap(uint32_t n, const uint32_t* __restrict__ bitmap, const uint8_t* __restrict__ type,
                                    uint8_t* __restrict__ flag, uint8_t* __restrict__ dup) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t t = type[i];
    bool valid = (bitmap[i >> 5] >> (i & 31)) & 1u;
    flag[i] = (valid && (t == T_PREVOTE || t == T_PRECOMMIT)) ? 1 : 0;
    if (dup) dup[i] = 3;
}

// signer index (sorted admitted table) for candidates, when the verify pass
// did not provide one
__global__ void k_signer_lookup(uint32_t n, const uint8_t* __restrict__ flag, const uint8_t* __restrict__ from32,
                                const uint32_t* __restrict__ adm, uint32_t n_adm, int steps, int32_t* __restrict__ signer) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t s = -1;
    if (flag[i]) {
        uint32_t key[8];
        for (int w = 0; w < 8; w++) key[w] = load_be32(from32 + 32 * (size_t)i + 4 * w);
        s = admitted_find(adm, n_adm, steps, key);
    }
    signer[i] = s;
}

__global__ void k_key_signer_type(uint32_t m, const uint32_t* __restrict__ cand, const int32_t* __restrict__ signer,
                                  const uint8_t* __restrict__ type, uint32_t* __restrict__ key) {
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    uint32_t i = cand[k];
    key[k] = ((uint32_t)signer[i] << 1) | (uint32_t)(type[i] - T_PREVOTE);
}

__global__ void k_key_i64(uint32_t m, const uint32_t* __restrict__ idx, const int64_t* __restrict__ src,
                          uint64_t* __restrict__ key) {
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    key[k] = (uint64_t)src[idx[k]] ^ kSign;
}

// value word w (big-endian 8 bytes) of message idx[k]
__global__ void k_key_value(uint32_t m, const uint32_t* __restrict__ idx, const uint8_t* __restrict__ value32, int w,
                            uint64_t* __restrict__ key) {
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint8_t* p = value32 + 32 * (size_t)idx[k] + 8 * w;
    key[k] = ((uint64_t)load_be32(p) << 32) | load_be32(p + 4);
}

__global__ void k_key_hr_type(uint32_t m, const uint32_t* __restrict__ idx, const uint32_t* __restrict__ hr_msg,
                              const uint8_t* __restrict__ type, uint64_t* __restrict__ key) {
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    uint32_t i = idx[k];
    key[k] = ((uint64_t)hr_msg[i] << 1) | (uint64_t)(type[i] - T_PREVOTE);
}

// group heads over candidates sorted by (h, r, signer, type)
__global__ void k_mark(uint32_t m, const uint32_t* __restrict__ cand, const int64_t* __restrict__ h,
                       const int64_t* __restrict__ r, const int32_t* __restrict__ signer,
                       const uint8_t* __restrict__ type, uint32_t* __restrict__ f_hr, uint32_t* __restrict__ f_hrs,
                       uint32_t* __restrict__ f_key, uint32_t* __restrict__ head_pos) {
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    uint32_t i = cand[k];
    bool nhr = true, nhrs = true, nkey = true;
    if (k > 0) {
        uint32_t p = cand[k - 1];
        nhr = h[i] != h[p] || r[i] != r[p];
        nhrs = nhr || signer[i] != signer[p];
        nkey = nhrs || type[i] != type[p];
    }
    f_hr[k] = nhr;
    f_hrs[k] = nhrs;
    f_key[k] = nkey;
    head_pos[k] = nkey ? k : 0u;
}

// Wavefront-shuffle segmented sum: lanes hold (seg, val) with seg
// non-decreasing across the wave; each segment's partial sum is added to
// out[seg] by its last lane.  Inactive lanes carry seg = 0xFFFFFFFF.
__device__ __forceinline__ void wave_seg_add(uint32_t seg, uint32_t val, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    HD_UNROLL for (int off = 1; off < 64; off <<= 1) {
        uint32_t s2 = __shfl_up(seg, off, 64);
        uint32_t v2 = __shfl_up(val, off, 64);
        if (lane >= off && s2 == seg) val += v2;
    }
    uint32_t snext = __shfl_down(seg, 1, 64);
    bool last = (lane == 63) || (snext != seg);
    if (last && seg != 0xFFFFFFFFu && val) atomicAdd(&out[seg], val);
}

// per (h, r) segment: heads, distinct signers, distinct per type; duplicates
__global__ void k_hr_reduce(uint32_t m, const uint32_t* __restrict__ cand, const uint32_t* __restrict__ hr_id,
                            const uint32_t* __restrict__ f_hr, const uint32_t* __restrict__ f_hrs,
                            const uint32_t* __restrict__ f_key, const uint32_t* __restrict__ head,
                            const int64_t* __restrict__ h, const int64_t* __restrict__ r,
                            const uint8_t* __restrict__ type, const uint8_t* __restrict__ value32,
                            int64_t* __restrict__ hr_h, int64_t* __restrict__ hr_r, uint32_t* __restrict__ hr_prev,
                            uint32_t* __restrict__ hr_prec, uint32_t* __restrict__ hr_any,
                            uint32_t* __restrict__ hr_msg, uint8_t* __restrict__ dup) {
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    bool act = k < m;
    uint32_t seg = 0xFFFFFFFFu, any = 0, pv = 0, pc = 0;
    if (act) {
        uint32_t i = cand[k];
        seg = hr_id[k] - 1;  // inclusive scan -> 0-based
        hr_msg[i] = seg;
        if (f_hr[k]) { hr_h[seg] = h[i]; hr_r[seg] = r[i]; }
        any = f_hrs[k];
        if (f_key[k]) {
            pv = type[i] == T_PREVOTE;
            pc = type[i] == T_PRECOMMIT;
            if (dup) dup[i] = 0;
        } else if (dup) {
            uint32_t j = cand[head[k]];
            const uint4* a = reinterpret_cast<const uint4*>(value32 + 32 * (size_t)i);
            const uint4* b = reinterpret_cast<const uint4*>(value32 + 32 * (size_t)j);
            bool same = true;
            for (int w = 0; w < 32; w++) same = same && value32[32 * (size_t)i + w] == value32[32 * (size_t)j + w];
            (void)a;
            (void)b;
            dup[i] = same ? 1 : 2;
        }
    }
    wave_seg_add(seg, any, hr_any);
    wave_seg_add(seg, pv, hr_prev);
    wave_seg_add(seg, pc, hr_prec);
}

// winners sorted by (hr, type, value): group heads
__global__ void k_group_mark(uint32_t w, const uint32_t* __restrict__ win, const uint32_t* __restrict__ hr_msg,
                             const uint8_t* __restrict__ type, const uint8_t* __restrict__ value32,
                             uint32_t* __restrict__ ghead) {
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= w) return;
    bool head = true;
    if (k > 0) {
        uint32_t i = win[k], p = win[k - 1];
        head = hr_msg[i] != hr_msg[p] || type[i] != type[p];
        for (int b = 0; b < 32 && !head; b++) head = value32[32 * (size_t)i + b] != value32[32 * (size_t)p + b];
    }
    ghead[k] = head;
}

__global__ void k_group_reduce(uint32_t w, const uint32_t* __restrict__ win, const uint32_t* __restrict__ ghead,
                               const uint32_t* __restrict__ gid, const uint32_t* __restrict__ hr_msg,
                               const int64_t* __restrict__ hr_h, const int64_t* __restrict__ hr_r,
                               const uint8_t* __restrict__ type, int64_t* __restrict__ c_h, int64_t* __restrict__ c_r,
                               uint8_t* __restrict__ c_t, uint32_t* __restrict__ c_rep, uint32_t* __restrict__ c_n) {
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    bool act = k < w;
    uint32_t seg = 0xFFFFFFFFu;
    if (act) {
        uint32_t i = win[k];
        seg = gid[k] - 1;
        if (ghead[k]) {
            uint32_t hr = hr_msg[i];
            c_h[seg] = hr_h[hr];
            c_r[seg] = hr_r[hr];
            c_t[seg] = type[i];
            c_rep[seg] = i;
        }
    }
    wave_seg_add(seg, act ? 1u : 0u, c_n);
}

// ---------------------------------------------------------------- host side
#define TCHK(expr, what)                                     \
    do {                                                     \
        hipError_t _e = (expr);                              \
        if (_e != hipSuccess) return hd_ctx_fail(ctx, _e, what); \
    } while (0)

static void* tbuf(hd_ctx* ctx, int slot, size_t bytes, int* rc) {
    DevBuf& b = ctx->tally->b[slot];
    int r = hd_dev_grow(ctx, &b.p, &b.cap, bytes);
    if (r) { *rc = r; return nullptr; }
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

// Tally on device data; results copied to the caller's host hd_tally_out.
// d_signer: signer indices (any consistent per-signatory index) or NULL.
static int tally_device(hd_ctx* ctx, const hd_batch* db, const uint8_t* d_verdict, const uint32_t* d_bitmap,
                        const int32_t* d_signer, hd_tally_out* out, hipStream_t s) {
    const uint32_t n = db->n;
    if (!ctx->tally) ctx->tally = new TallyWork();
    int rc = 0;
    uint8_t* flag = (uint8_t*)tbuf(ctx, T_FLAG, n, &rc);
    uint8_t* d_dup = out->dup ? (uint8_t*)tbuf(ctx, T_DUP, n, &rc) : nullptr;
    if (rc) return rc;
    if (d_verdict) k_cand_flags<<<nblk(n), 256, 0, s>>>(n, d_verdict, db->type, flag, d_dup);
    else k_cand_flags_bitmap<<<nblk(n), 256, 0, s>>>(n, d_bitmap, db->type, flag, d_dup);
    int32_t* signer = const_cast<int32_t*>(d_signer);
    if (!signer) {
        signer = (int32_t*)tbuf(ctx, T_SIGNER, 4 * (size_t)n, &rc);
        if (rc) return rc;
        k_signer_lookup<<<nblk(n), 256, 0, s>>>(n, flag, db->from32, ctx->d_adm, ctx->n_adm, ctx->adm_steps, signer);
    }
    // 1. compact candidates
    uint32_t* cand0 = (uint32_t*)tbuf(ctx, T_CAND0, 4 * (size_t)n, &rc);
    uint32_t* cand1 = (uint32_t*)tbuf(ctx, T_CAND1, 4 * (size_t)n, &rc);
    uint32_t* nsel = (uint32_t*)tbuf(ctx, T_NSEL, 64, &rc);
    if (rc) return rc;
    size_t tmp_bytes = 0, need = 0;
    hipcub::CountingInputIterator<uint32_t> iota(0);
    TCHK(hipcub::DeviceSelect::Flagged(nullptr, need, iota, flag, cand0, nsel, n, s), "select size");
    tmp_bytes = std::max(tmp_bytes, need);
    // sort temp sizes
    {
        hipcub::DoubleBuffer<uint32_t> kk(nullptr, nullptr), vv(nullptr, nullptr);
        hipcub::DoubleBuffer<uint64_t> k64(nullptr, nullptr);
        TCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, need, kk, vv, n, 0, 32, s), "sort size");
        tmp_bytes = std::max(tmp_bytes, need);
        TCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, need, k64, vv, n, 0, 64, s), "sort size");
        tmp_bytes = std::max(tmp_bytes, need);
        TCHK(hipcub::DeviceScan::InclusiveSum(nullptr, need, (uint32_t*)nullptr, (uint32_t*)nullptr, n, s), "scan size");
        tmp_bytes = std::max(tmp_bytes, need);
        TCHK(hipcub::DeviceScan::InclusiveScan(nullptr, need, (uint32_t*)nullptr, (uint32_t*)nullptr, hipcub::Max(), n, s),
             "scan size");
        tmp_bytes = std::max(tmp_bytes, need);
    }
    void* tmp = tbuf(ctx, T_TMP, tmp_bytes, &rc);
    if (rc) return rc;
    TCHK(hipcub::DeviceSelect::Flagged(tmp, tmp_bytes, iota, flag, cand0, nsel, n, s), "select");
    uint32_t m = 0;
    TCHK(hipMemcpyAsync(&m, nsel, 4, hipMemcpyDeviceToHost, s), "nsel");
    TCHK(hipStreamSynchronize(s), "nsel sync");

    out->n_counts = 0;
    out->n_hr = 0;
    if (m == 0) {
        if (out->dup) {
            TCHK(hipMemcpyAsync(out->dup, d_dup, n, hipMemcpyDeviceToHost, s), "dup");
            TCHK(hipStreamSynchronize(s), "dup sync");
        }
        return HD_OK;
    }
    // 2. stable LSD sort by (h, r, signer, type)
    uint32_t* k32a = (uint32_t*)tbuf(ctx, T_K32A, 4 * (size_t)m, &rc);
    uint32_t* k32b = (uint32_t*)tbuf(ctx, T_K32B, 4 * (size_t)m, &rc);
    uint64_t* k64a = (uint64_t*)tbuf(ctx, T_K64A, 8 * (size_t)m, &rc);
    uint64_t* k64b = (uint64_t*)tbuf(ctx, T_K64B, 8 * (size_t)m, &rc);
    if (rc) return rc;
    hipcub::DoubleBuffer<uint32_t> vals(cand0, cand1);
    {
        int bits = 1;
        while ((1u << (bits - 1)) < std::max(ctx->n_adm, 1u)) bits++;
        k_key_signer_type<<<nblk(m), 256, 0, s>>>(m, vals.Current(), signer, db->type, k32a);
        hipcub::DoubleBuffer<uint32_t> keys(k32a, k32b);
        TCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, vals, m, 0, bits + 1, s), "sort signer");
        const int64_t* fields[2] = {db->round, db->height};
        for (int f = 0; f < 2; f++) {
            k_key_i64<<<nblk(m), 256, 0, s>>>(m, vals.Current(), fields[f], k64a);
            hipcub::DoubleBuffer<uint64_t> k64(k64a, k64b);
            TCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k64, vals, m, 0, 64, s), "sort h/r");
        }
    }
    uint32_t* cand = vals.Current();
    // 3. marks + scans
    uint32_t* f_hr = (uint32_t*)tbuf(ctx, T_FHR, 4 * (size_t)m, &rc);
    uint32_t* f_hrs = (uint32_t*)tbuf(ctx, T_FHRS, 4 * (size_t)m, &rc);
    uint32_t* f_key = (uint32_t*)tbuf(ctx, T_FKEY, 4 * (size_t)m, &rc);
    uint32_t* hr_id = (uint32_t*)tbuf(ctx, T_HRID, 4 * (size_t)m, &rc);
    uint32_t* head = (uint32_t*)tbuf(ctx, T_HEAD, 4 * (size_t)m, &rc);
    uint32_t* hr_msg = (uint32_t*)tbuf(ctx, T_HRMSG, 4 * (size_t)n, &rc);
    if (rc) return rc;
    k_mark<<<nblk(m), 256, 0, s>>>(m, cand, db->height, db->round, signer, db->type, f_hr, f_hrs, f_key, head);
    TCHK(hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, f_hr, hr_id, m, s), "scan hr");
    TCHK(hipcub::DeviceScan::InclusiveScan(tmp, tmp_bytes, head, head, hipcub::Max(), m, s), "scan head");
    uint32_t n_hr = 0;
    TCHK(hipMemcpyAsync(&n_hr, hr_id + (m - 1), 4, hipMemcpyDeviceToHost, s), "n_hr");
    // winners: compact f_key positions -> message indices
    uint32_t* win0 = (uint32_t*)tbuf(ctx, T_WIN0, 4 * (size_t)m, &rc);
    uint32_t* win1 = (uint32_t*)tbuf(ctx, T_WIN1, 4 * (size_t)m, &rc);
    if (rc) return rc;
    TCHK(hipcub::DeviceSelect::Flagged(tmp, tmp_bytes, cand, f_key, win0, nsel, m, s), "select winners");
    uint32_t w = 0;
    TCHK(hipMemcpyAsync(&w, nsel, 4, hipMemcpyDeviceToHost, s), "nwin");
    TCHK(hipStreamSynchronize(s), "sync");
    // 4. per (h, r)
    // layout of T_OUTHR: h[n_hr] r[n_hr] | prev any prec [n_hr] (u32)
    size_t hr_bytes = 16 * (size_t)n_hr + 12 * (size_t)n_hr;
    char* hrb = (char*)tbuf(ctx, T_OUTHR, hr_bytes, &rc);
    if (rc) return rc;
    int64_t* d_hr_h = (int64_t*)hrb;
    int64_t* d_hr_r = d_hr_h + n_hr;
    uint32_t* d_hr_prev = (uint32_t*)(d_hr_r + n_hr);
    uint32_t* d_hr_any = d_hr_prev + n_hr;
    uint32_t* d_hr_prec = d_hr_any + n_hr;
    TCHK(hipMemsetAsync(d_hr_prev, 0, 12 * (size_t)n_hr, s), "memset hr");
    k_hr_reduce<<<nblk(m), 256, 0, s>>>(m, cand, hr_id, f_hr, f_hrs, f_key, head, db->height, db->round, db->type,
                                       db->value32, d_hr_h, d_hr_r, d_hr_prev, d_hr_prec, d_hr_any, hr_msg, d_dup);
    // 5. winners by (hr, type, value)
    hipcub::DoubleBuffer<uint32_t> wv(win0, win1);
    for (int word = 3; word >= 0; word--) {
        k_key_value<<<nblk(w), 256, 0, s>>>(w, wv.Current(), db->value32, word, k64a);
        hipcub::DoubleBuffer<uint64_t> k64(k64a, k64b);
        TCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k64, wv, w, 0, 64, s), "sort value");
    }
    {
        k_key_hr_type<<<nblk(w), 256, 0, s>>>(w, wv.Current(), hr_msg, db->type, k64a);
        int bits = 2;
        while ((1ull << (bits - 1)) < (uint64_t)n_hr) bits++;
        hipcub::DoubleBuffer<uint64_t> k64(k64a, k64b);
        TCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k64, wv, w, 0, bits + 1, s), "sort hr/type");
    }
    uint32_t* win = wv.Current();
    uint32_t* ghead = (uint32_t*)tbuf(ctx, T_GHEAD, 4 * (size_t)w, &rc);
    uint32_t* gid = (uint32_t*)tbuf(ctx, T_GID, 4 * (size_t)w, &rc);
    if (rc) return rc;
    k_group_mark<<<nblk(w), 256, 0, s>>>(w, win, hr_msg, db->type, db->value32, ghead);
    TCHK(hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, ghead, gid, w, s), "scan groups");
    uint32_t n_cnt = 0;
    TCHK(hipMemcpyAsync(&n_cnt, gid + (w - 1), 4, hipMemcpyDeviceToHost, s), "n_cnt");
    TCHK(hipStreamSynchronize(s), "sync");
    size_t cb = (8 + 8 + 1 + 4 + 4) * (size_t)n_cnt + 64;
    char* cbuf = (char*)tbuf(ctx, T_OUTCNT, cb, &rc);
    if (rc) return rc;
    int64_t* c_h = (int64_t*)cbuf;
    int64_t* c_r = c_h + n_cnt;
    uint32_t* c_rep = (uint32_t*)(c_r + n_cnt);
    uint32_t* c_n = c_rep + n_cnt;
    uint8_t* c_t = (uint8_t*)(c_n + n_cnt);
    TCHK(hipMemsetAsync(c_n, 0, 4 * (size_t)n_cnt, s), "memset counts");
    k_group_reduce<<<nblk(w), 256, 0, s>>>(w, win, ghead, gid, hr_msg, d_hr_h, d_hr_r, db->type, c_h, c_r, c_t, c_rep,
                                           c_n);
    TCHK(hipGetLastError(), "tally kernels");
    out->n_hr = n_hr;
    out->n_counts = n_cnt;
    if (n_hr > out->cap_hr || n_cnt > out->cap_counts) {
        TCHK(hipStreamSynchronize(s), "sync");
        return HD_ECAP;
    }
    struct C { void* dst; const void* src; size_t sz; } cp[] = {
        {out->hr_height, d_hr_h, 8 * (size_t)n_hr},      {out->hr_round, d_hr_r, 8 * (size_t)n_hr},
        {out->hr_prevotes, d_hr_prev, 4 * (size_t)n_hr}, {out->hr_precommits, d_hr_prec, 4 * (size_t)n_hr},
        {out->hr_any, d_hr_any, 4 * (size_t)n_hr},       {out->count_height, c_h, 8 * (size_t)n_cnt},
        {out->count_round, c_r, 8 * (size_t)n_cnt},      {out->count_type, c_t, (size_t)n_cnt},
        {out->count_rep, c_rep, 4 * (size_t)n_cnt},      {out->count_n, c_n, 4 * (size_t)n_cnt},
        {out->dup, d_dup, (size_t)n},
    };
    for (auto& c : cp)
        if (c.dst && c.sz) TCHK(hipMemcpyAsync(c.dst, c.src, c.sz, hipMemcpyDeviceToHost, s), "tally download");
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
    return tally_device(ctx, &db, d_v, nullptr, nullptr, out, ctx->stream);
}

int hd_tally_device(hd_ctx* ctx, const hd_batch* dbatch, const uint8_t* d_verdict, const int32_t* d_signer,
                    hd_tally_out* out, void* stream) {
    if (!ctx || !dbatch || !d_verdict || !tally_out_ok(out)) return HD_EINVAL;
    out->n_counts = out->n_hr = 0;
    if (dbatch->n == 0) return HD_OK;
    (void)hipSetDevice(ctx->device);
    return tally_device(ctx, dbatch, d_verdict, nullptr, d_signer, out, stream ? (hipStream_t)stream : ctx->stream);
}

int hd_tally_device_bitmap(hd_ctx* ctx, const hd_batch* dbatch, const uint32_t* d_valid_bitmap, hd_tally_out* out,
                           void* stream) {
    if (!ctx || !dbatch || !d_valid_bitmap || !tally_out_ok(out)) return HD_EINVAL;
    out->n_counts = out->n_hr = 0;
    if (dbatch->n == 0) return HD_OK;
    (void)hipSetDevice(ctx->device);
    return tally_device(ctx, dbatch, nullptr, d_valid_bitmap, nullptr, out, stream ? (hipStream_t)stream : ctx->stream);
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
    // the verify pass left verdicts and caller-order signer indices on device
    return tally_device(ctx, &db, (const uint8_t*)ctx->bufs[BUF_VERDICT].p, nullptr,
                        (const int32_t*)ctx->bufs[BUF_SIGNER].p, tally, ctx->stream);
}

}  // extern "C"
