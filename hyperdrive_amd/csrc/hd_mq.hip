// hd_mq.hip -- bulk MessageQueue (include/hd_mq.h; mq/mq.go:19-143).
//
// The queue is one SoA pool of messages kept sorted by (sender, height,
// round, arrival).  A batch insert appends the batch's messages after the
// pool (so arrival order == position for equal keys), re-sorts with stable
// LSD radix passes over (round, height, sender) -- keys rebased to the batch's
// min and cut to their significant bits, so a typical insert costs a handful
// of 8-bit digit passes -- and keeps each sender's first max_capacity
// elements: exactly the result of inserting one message at a time with
// mq.go:133-142's truncation.  Consume(h) and DropMessagesBelowHeight(h) are
// order-preserving partitions (each sender's consumed messages are a prefix of
// its run, mq.go:38-41).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <new>

#include "../../include/hd_mq.h"
#include "hd_internal.h"

using namespace hd;

namespace {

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

// element e of the merged sequence: e < M -> pool[e]; else batch[newidx[e - M]]
struct MqSrc {
    Pool p;
    DevBatch b;
    const uint32_t* newidx;
    const int32_t* bsender;
    uint32_t M;
};

__device__ __forceinline__ void src_keys(const MqSrc& s, uint32_t e, int32_t& snd, int64_t& h, int64_t& r) {
    if (e < s.M) {
        snd = s.p.sender[e];
        h = s.p.h[e];
        r = s.p.r[e];
    } else {
        const uint32_t i = s.newidx[e - s.M];
        snd = s.bsender[i];
        h = s.b.height[i];
        r = s.b.round[i];
    }
}

__global__ void k_mq_flag_new(uint32_t n, const int32_t* __restrict__ sender, uint8_t* __restrict__ flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = sender[i] >= 0;
}

// Replica.Run ingress (replica.go:117-131): a verified message enters the
// queue iff VALID and filterHeight passes (height >= current, replica.go:247-249)
__global__ void k_mq_ingress(uint32_t n, const uint8_t* __restrict__ verdict, const int32_t* __restrict__ signer,
                             const int64_t* __restrict__ height, int64_t min_height, int32_t* __restrict__ snd) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) snd[i] = (verdict[i] == HD_VERDICT_VALID && height[i] >= min_height) ? signer[i] : -1;
}

__global__ void k_mq_keys(MqSrc s, uint32_t T, int64_t* __restrict__ hk, int64_t* __restrict__ rk,
                          uint32_t* __restrict__ sk, uint32_t* __restrict__ iota) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= T) return;
    int32_t snd;
    int64_t h, r;
    src_keys(s, e, snd, h, r);
    hk[e] = h;
    rk[e] = r;
    sk[e] = (uint32_t)snd;
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

// dst[k] := element sel[k] of the merged sequence
__global__ void k_mq_gather(MqSrc s, uint32_t n, const uint32_t* __restrict__ sel, Pool d) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
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
        for (int w = 0; w < 65; w++) d.sig[65 * (size_t)k + w] = s.p.sig[65 * (size_t)e + w];
    } else {
        const uint32_t i = s.newidx[e - s.M];
        d.sender[k] = s.bsender[i];
        d.type[k] = s.b.type[i];
        d.h[k] = s.b.height[i];
        d.r[k] = s.b.round[i];
        d.vr[k] = s.b.valid_round ? s.b.valid_round[i] : -1;
        for (int w = 0; w < 32; w++) {
            d.value[32 * (size_t)k + w] = s.b.value32[32 * (size_t)i + w];
            d.from[32 * (size_t)k + w] = s.b.from32[32 * (size_t)i + w];
        }
        for (int w = 0; w < 65; w++) d.sig[65 * (size_t)k + w] = s.b.sig65 ? s.b.sig65[65 * (size_t)i + w] : 0;
    }
}

__global__ void k_mq_compose(uint32_t n, const uint32_t* __restrict__ perm, const uint32_t* __restrict__ sel,
                             uint32_t* __restrict__ ids) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) ids[k] = perm[sel[k]];
}

// partition predicate over the pool: flag[e] = pool.h[e] <= h (consume) or
// pool.h[e] < h (drop); inv = the complement
__global__ void k_mq_pred(uint32_t n, const int64_t* __restrict__ ph, int64_t h, int strict, uint8_t* __restrict__ flag,
                          uint8_t* __restrict__ inv) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const bool f = strict ? ph[e] < h : ph[e] <= h;
    flag[e] = f;
    inv[e] = !f;
}

inline uint32_t nblk(uint32_t n) { return (n + 255) / 256; }

int bits_of(uint64_t range) {
    int b = 0;
    while (b < 64 && (range >> b)) b++;
    return b;
}

}  // namespace

enum MqSlot { MQ_FLAG, MQ_NEWIDX, MQ_NSEL, MQ_HK, MQ_RK, MQ_SK, MQ_PERM0, MQ_PERM1, MQ_K64A, MQ_K64B, MQ_K32A, MQ_K32B,
              MQ_HEAD, MQ_KEEP, MQ_SEL, MQ_RED, MQ_TMP, MQ_SND, MQ__N };

struct hd_mq {
    hd_ctx* ctx = nullptr;
    uint32_t max_cap = 1000;
    Pool pool, spare;
    DevBuf buf[MQ__N];
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

template <typename T>
static int dev_minmax(hd_mq* q, const T* d, uint32_t n, T* mn, T* mx, hipStream_t s) {
    int rc = 0;
    T* red = (T*)qbuf(q, MQ_RED, 2 * sizeof(T), &rc);
    if (rc) return rc;
    size_t need = 0, need2 = 0;
    QCHK(hipcub::DeviceReduce::Min(nullptr, need, d, red, n, s), "reduce size");
    QCHK(hipcub::DeviceReduce::Max(nullptr, need2, d, red + 1, n, s), "reduce size");
    void* tmp = qbuf(q, MQ_TMP, std::max(need, need2), &rc);
    if (rc) return rc;
    QCHK(hipcub::DeviceReduce::Min(tmp, need, d, red, n, s), "reduce min");
    QCHK(hipcub::DeviceReduce::Max(tmp, need2, d, red + 1, n, s), "reduce max");
    T host[2];
    QCHK(hipMemcpyAsync(host, red, 2 * sizeof(T), hipMemcpyDeviceToHost, s), "minmax");
    QCHK(hipStreamSynchronize(s), "minmax sync");
    *mn = host[0];
    *mx = host[1];
    return HD_OK;
}

// select-flagged over [0, n) -> out indices, returns count (synchronises)
static int select_idx(hd_mq* q, const uint8_t* flag, uint32_t n, uint32_t* out, uint32_t* count, hipStream_t s) {
    int rc = 0;
    uint32_t* nsel = (uint32_t*)qbuf(q, MQ_NSEL, 64, &rc);
    if (rc) return rc;
    hipcub::CountingInputIterator<uint32_t> iota(0);
    size_t need = 0;
    QCHK(hipcub::DeviceSelect::Flagged(nullptr, need, iota, flag, out, nsel, n, s), "select size");
    void* tmp = qbuf(q, MQ_TMP, need, &rc);
    if (rc) return rc;
    QCHK(hipcub::DeviceSelect::Flagged(tmp, need, iota, flag, out, nsel, n, s), "select");
    QCHK(hipMemcpyAsync(count, nsel, 4, hipMemcpyDeviceToHost, s), "select count");
    QCHK(hipStreamSynchronize(s), "select sync");
    return HD_OK;
}

// stable sort of perm (DoubleBuffer) by a 64-bit field rebased to its min
static int sort_pass64(hd_mq* q, hipcub::DoubleBuffer<uint32_t>& perm, const int64_t* field, uint32_t T, hipStream_t s) {
    int64_t mn = 0, mx = 0;
    int rc = dev_minmax(q, field, T, &mn, &mx, s);
    if (rc) return rc;
    const int bits = bits_of((uint64_t)mx - (uint64_t)mn);
    if (bits == 0) return HD_OK;
    uint64_t* ka = (uint64_t*)qbuf(q, MQ_K64A, 8 * (size_t)T, &rc);
    uint64_t* kb = (uint64_t*)qbuf(q, MQ_K64B, 8 * (size_t)T, &rc);
    if (rc) return rc;
    k_mq_rekey64<<<nblk(T), 256, 0, s>>>(T, perm.Current(), field, mn, ka);
    hipcub::DoubleBuffer<uint64_t> keys(ka, kb);
    size_t need = 0;
    QCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, need, keys, perm, T, 0, bits, s), "sort size");
    void* tmp = qbuf(q, MQ_TMP, need, &rc);
    if (rc) return rc;
    QCHK(hipcub::DeviceRadixSort::SortPairs(tmp, need, keys, perm, T, 0, bits, s), "sort 64");
    return HD_OK;
}

static int sort_pass32(hd_mq* q, hipcub::DoubleBuffer<uint32_t>& perm, const uint32_t* field, uint32_t T,
                       hipStream_t s) {
    uint32_t mn = 0, mx = 0;
    int rc = dev_minmax(q, field, T, &mn, &mx, s);
    if (rc) return rc;
    const int bits = bits_of(mx);
    if (bits == 0) return HD_OK;
    uint32_t* ka = (uint32_t*)qbuf(q, MQ_K32A, 4 * (size_t)T, &rc);
    uint32_t* kb = (uint32_t*)qbuf(q, MQ_K32B, 4 * (size_t)T, &rc);
    if (rc) return rc;
    k_mq_rekey32<<<nblk(T), 256, 0, s>>>(T, perm.Current(), field, ka);
    hipcub::DoubleBuffer<uint32_t> keys(ka, kb);
    size_t need = 0;
    QCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, need, keys, perm, T, 0, bits, s), "sort size");
    void* tmp = qbuf(q, MQ_TMP, need, &rc);
    if (rc) return rc;
    QCHK(hipcub::DeviceRadixSort::SortPairs(tmp, need, keys, perm, T, 0, bits, s), "sort 32");
    return HD_OK;
}

// keep the pool elements whose flag is set, in order
static int pool_filter(hd_mq* q, const uint8_t* keep, hipStream_t s) {
    int rc = 0;
    const uint32_t M = q->pool.n;
    uint32_t* sel = (uint32_t*)qbuf(q, MQ_SEL, 4 * (size_t)M, &rc);
    if (rc) return rc;
    uint32_t n = 0;
    rc = select_idx(q, keep, M, sel, &n, s);
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

extern "C" {

int hd_mq_create(hd_ctx* ctx, uint32_t max_capacity, hd_mq** out) {
    if (!ctx || !out || max_capacity == 0) return HD_EINVAL;
    hd_mq* q = new (std::nothrow) hd_mq();
    if (!q) return HD_ENOMEM;
    q->ctx = ctx;
    q->max_cap = max_capacity;
    *out = q;
    return HD_OK;
}

int hd_mq_destroy(hd_mq* q) {
    if (!q) return HD_EINVAL;
    (void)hipSetDevice(q->ctx->device);
    (void)hipStreamSynchronize(q->ctx->stream);
    if (q->pool.base) (void)hipFree(q->pool.base);
    if (q->spare.base) (void)hipFree(q->spare.base);
    for (auto& b : q->buf)
        if (b.p) (void)hipFree(b.p);
    delete q;
    return HD_OK;
}

int hd_mq_size(hd_mq* q, uint64_t* n) {
    if (!q || !n) return HD_EINVAL;
    *n = q->pool.n;
    return HD_OK;
}

int hd_mq_insert_device(hd_mq* q, const hd_batch* d_batch, const int32_t* d_sender, void* stream) {
    if (!q || !d_batch) return HD_EINVAL;
    const uint32_t nb = d_batch->n;
    if (nb == 0) return HD_OK;  // empty device tensors may have NULL data pointers
    if (!d_sender) return HD_EINVAL;
    if (!d_batch->type || !d_batch->height || !d_batch->round || !d_batch->value32 || !d_batch->from32)
        return HD_EINVAL;
    (void)hipSetDevice(q->ctx->device);
    hipStream_t s = stream ? (hipStream_t)stream : q->ctx->stream;
    int rc = 0;
    // 1. the batch's insertable messages, in batch order
    uint8_t* flag = (uint8_t*)qbuf(q, MQ_FLAG, nb, &rc);
    uint32_t* newidx = (uint32_t*)qbuf(q, MQ_NEWIDX, 4 * (size_t)nb, &rc);
    if (rc) return rc;
    k_mq_flag_new<<<nblk(nb), 256, 0, s>>>(nb, d_sender, flag);
    uint32_t m = 0;
    rc = select_idx(q, flag, nb, newidx, &m, s);
    if (rc || m == 0) return rc;
    // 2. merged sequence: pool (sorted) then the new messages (arrival order)
    const uint32_t M = q->pool.n, T = M + m;
    DevBatch b{nb, d_batch->type, d_batch->height, d_batch->round, d_batch->valid_round, d_batch->value32,
               d_batch->from32, d_batch->sig65};
    MqSrc src{q->pool, b, newidx, d_sender, M};
    int64_t* hk = (int64_t*)qbuf(q, MQ_HK, 8 * (size_t)T, &rc);
    int64_t* rk = (int64_t*)qbuf(q, MQ_RK, 8 * (size_t)T, &rc);
    uint32_t* sk = (uint32_t*)qbuf(q, MQ_SK, 4 * (size_t)T, &rc);
    uint32_t* p0 = (uint32_t*)qbuf(q, MQ_PERM0, 4 * (size_t)T, &rc);
    uint32_t* p1 = (uint32_t*)qbuf(q, MQ_PERM1, 4 * (size_t)T, &rc);
    if (rc) return rc;
    k_mq_keys<<<nblk(T), 256, 0, s>>>(src, T, hk, rk, sk, p0);
    // 3. stable LSD passes: round, height, sender (mq.go:120-128 order; the
    //    stability keeps arrival order among equal keys)
    hipcub::DoubleBuffer<uint32_t> perm(p0, p1);
    if ((rc = sort_pass64(q, perm, rk, T, s))) return rc;
    if ((rc = sort_pass64(q, perm, hk, T, s))) return rc;
    if ((rc = sort_pass32(q, perm, sk, T, s))) return rc;
    // 4. per-sender capacity: keep the first max_cap of every sender run
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
    uint32_t kept = 0;
    rc = select_idx(q, keep, T, sel, &kept, s);
    if (rc) return rc;
    // sel holds kept positions in sorted order -> element ids -> new pool
    uint32_t* ids = head;  // head is consumed by k_mq_keep; reuse its space
    k_mq_compose<<<nblk(kept), 256, 0, s>>>(kept, perm.Current(), sel, ids);
    rc = pool_reserve(q->ctx, q->spare, std::max(kept, 1u));
    if (rc) return rc;
    k_mq_gather<<<nblk(kept), 256, 0, s>>>(src, kept, ids, q->spare);
    QCHK(hipGetLastError(), "mq insert kernels");
    std::swap(q->pool, q->spare);
    q->pool.n = kept;
    QCHK(hipStreamSynchronize(s), "mq insert sync");
    return HD_OK;
}

int hd_mq_insert_verified_device(hd_mq* q, const hd_batch* d_batch, const uint8_t* d_verdict, const int32_t* d_signer,
                                 int64_t min_height, void* stream) {
    if (!q || !d_batch) return HD_EINVAL;
    const uint32_t nb = d_batch->n;
    if (nb == 0) return HD_OK;
    if (!d_verdict || !d_signer) return HD_EINVAL;
    if (!d_batch->height) return HD_EINVAL;
    (void)hipSetDevice(q->ctx->device);
    hipStream_t s = stream ? (hipStream_t)stream : q->ctx->stream;
    int rc = 0;
    int32_t* snd = (int32_t*)qbuf(q, MQ_SND, 4 * (size_t)nb, &rc);
    if (rc) return rc;
    k_mq_ingress<<<nblk(nb), 256, 0, s>>>(nb, d_verdict, d_signer, d_batch->height, min_height, snd);
    QCHK(hipGetLastError(), "k_mq_ingress");
    return hd_mq_insert_device(q, d_batch, snd, stream);
}

int hd_mq_consume(hd_mq* q, int64_t h, const hd_batch_out* out, int32_t* out_sender, uint32_t cap, uint32_t* n_out) {
    if (!q || !out || !n_out) return HD_EINVAL;
    if (!out->type || !out->height || !out->round || !out->value32 || !out->from32) return HD_EINVAL;
    *n_out = 0;
    const uint32_t M = q->pool.n;
    if (M == 0) return HD_OK;
    (void)hipSetDevice(q->ctx->device);
    hipStream_t s = q->ctx->stream;
    int rc = 0;
    uint8_t* flag = (uint8_t*)qbuf(q, MQ_FLAG, M, &rc);
    uint8_t* inv = (uint8_t*)qbuf(q, MQ_KEEP, M, &rc);
    uint32_t* sel = (uint32_t*)qbuf(q, MQ_SEL, 4 * (size_t)M, &rc);
    if (rc) return rc;
    k_mq_pred<<<nblk(M), 256, 0, s>>>(M, q->pool.h, h, 0, flag, inv);
    uint32_t c = 0;
    rc = select_idx(q, flag, M, sel, &c, s);
    if (rc) return rc;
    *n_out = c;
    if (c > cap) return HD_ECAP;
    if (c) {
        rc = pool_reserve(q->ctx, q->spare, c);
        if (rc) return rc;
        MqSrc src{q->pool, DevBatch{}, nullptr, nullptr, M};
        k_mq_gather<<<nblk(c), 256, 0, s>>>(src, c, sel, q->spare);
        const Pool& d = q->spare;
        struct Cp { void* dst; const void* src; size_t sz; } cp[] = {
            {out->type, d.type, (size_t)c},          {out->height, d.h, 8 * (size_t)c},
            {out->round, d.r, 8 * (size_t)c},        {out->valid_round, d.vr, 8 * (size_t)c},
            {out->value32, d.value, 32 * (size_t)c}, {out->from32, d.from, 32 * (size_t)c},
            {out->sig65, d.sig, 65 * (size_t)c},     {out_sender, d.sender, 4 * (size_t)c},
        };
        for (auto& x : cp)
            if (x.dst) QCHK(hipMemcpyAsync(x.dst, x.src, x.sz, hipMemcpyDeviceToHost, s), "consume download");
        if (out->adv_class) memset(out->adv_class, 0, c);
        QCHK(hipStreamSynchronize(s), "consume sync");
    }
    return pool_filter(q, inv, s);
}

int hd_mq_drop_below(hd_mq* q, int64_t h) {
    if (!q) return HD_EINVAL;
    const uint32_t M = q->pool.n;
    if (M == 0) return HD_OK;
    (void)hipSetDevice(q->ctx->device);
    hipStream_t s = q->ctx->stream;
    int rc = 0;
    uint8_t* flag = (uint8_t*)qbuf(q, MQ_FLAG, M, &rc);
    uint8_t* inv = (uint8_t*)qbuf(q, MQ_KEEP, M, &rc);
    if (rc) return rc;
    k_mq_pred<<<nblk(M), 256, 0, s>>>(M, q->pool.h, h, 1, flag, inv);
    return pool_filter(q, inv, s);
}

}  // extern "C"
