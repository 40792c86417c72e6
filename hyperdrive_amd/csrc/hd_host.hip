// hd_host.hip -- asynchronous host-buffer verification (include/hd_verify.h
// hd_verify_submit / hd_verify_wait / hd_host_alloc).
//
// The cgo caller hands over host messages (replica/replica.go:156-181);
// hd_verify_batch uploads, verifies and downloads in series, so its PCIe time
// adds to the kernels'.  Here a context keeps HD_HOST_SLOTS pipelines, each
// with its own stream, device buffers and pinned staging: a submit queues
// H2D copies -> hd_verify_batch_device -> D2H copies on its pipeline's stream
// and returns, so batch k+1's upload runs under batch k's kernels (and the
// two pipelines' verify calls overlap on the device, hd_fastverify.hip's
// scratch sets).  Inputs and outputs in pinned memory move by DMA straight
// from / to the caller's buffers; pageable ones pass through pinned staging,
// copied by host threads (one memcpy thread cannot keep up with PCIe).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/hd_verify.h"
#include "hd_internal.h"

namespace {

// device columns of a pipeline: the hd_batch fields, then the compact
// batch's index columns and dictionaries (hd_verify_submit_compact)
enum { HC_TYPE, HC_H, HC_R, HC_VR, HC_VALUE, HC_FROM, HC_SIG, HC_FIDX, HC_VIDX, HC_ESC, HC_VALS, HC_N };

struct HostSlot {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    uint64_t ticket = 0;     // in flight or awaiting delivery (0: idle)
    DevBuf col[HC_N], verdict, rec, bitmap;
    void* hin = nullptr;     // pinned input staging (pageable inputs)
    size_t hin_cap = 0;
    void* hout = nullptr;    // pinned output staging (pageable outputs)
    size_t hout_cap = 0;
    // delivery of staged outputs at completion: (dst, staged src, bytes)
    struct Copy { void* dst; const void* src; size_t n; };
    std::vector<Copy> deliver;
};

}  // namespace

struct HostPipe {
    HostSlot slot[HD_HOST_SLOTS];
    uint64_t next = 1;
};

namespace {

#define HCHK(expr, what)                                          \
    do {                                                          \
        hipError_t e_ = (expr);                                   \
        if (e_ != hipSuccess) return hd_ctx_fail(ctx, e_, what);  \
    } while (0)

// Outputs go to host memory by a kernel's stores over PCIe (the pinned
// buffer mapped into the device's address space), not by DMA: the DMA
// engine runs copies in the order they were queued, so a download queued
// behind batch k's kernels would hold back batch k+1's upload queued after
// it, and every batch's upload, kernels and download would run in series
// (rocprofv3 memory-copy trace, round 3).  With the downloads on the compute
// queue the engine carries only uploads, and batch k+1's upload runs under
// batch k's kernels.  HD_HOST_D2H=dma restores the copies for A/B.
struct HostOut {
    uint8_t* dst[3];
    const uint8_t* src[3];
    size_t n[3];
};
__global__ __launch_bounds__(256) void k_host_store(HostOut o) {
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    for (int k = 0; k < 3; k++) {
        if (!o.dst[k]) continue;
        const size_t n = o.n[k];
        // 16-byte words where both ends are 16-byte aligned, bytes otherwise
        if ((((uintptr_t)o.dst[k] | (uintptr_t)o.src[k]) & 15) == 0) {
            const size_t w = n / 16;
            const uint4* s4 = reinterpret_cast<const uint4*>(o.src[k]);
            uint4* d4 = reinterpret_cast<uint4*>(o.dst[k]);
            for (size_t i = t; i < w; i += stride) d4[i] = s4[i];
            for (size_t i = 16 * w + t; i < n; i += stride) o.dst[k][i] = o.src[k][i];
        } else {
            for (size_t i = t; i < n; i += stride) o.dst[k][i] = o.src[k][i];
        }
    }
}

// The compact batch's From and value columns, expanded on the device: row i
// of from32 is the caller's signatory from_idx[i] (the array last passed to
// hd_set_signatories, caller order) or escape row from_idx[i] - n_sig; row i
// of value32 is values row value_idx[i].  One lane per 16-byte half row, so
// a wavefront reads and writes whole 16-byte words.  Indices were range
// checked on the host.
__global__ __launch_bounds__(256) void k_compact_expand(uint32_t n, const uint16_t* __restrict__ from_idx,
                                                        const uint16_t* __restrict__ value_idx,
                                                        const uint4* __restrict__ sigs, uint32_t n_sig,
                                                        const uint4* __restrict__ esc,
                                                        const uint4* __restrict__ vals, uint4* __restrict__ from32,
                                                        uint4* __restrict__ value32) {
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= 2 * (size_t)n) return;
    const uint32_t i = (uint32_t)(t >> 1), h = (uint32_t)(t & 1);
    const uint32_t f = from_idx[i];
    from32[t] = f < n_sig ? sigs[2 * (size_t)f + h] : esc[2 * (size_t)(f - n_sig) + h];
    value32[t] = vals[2 * (size_t)value_idx[i] + h];
}

// largest element of a host index column (the range check before the upload)
uint32_t max_u16(const uint16_t* a, size_t n) {
    uint16_t m = 0;
    for (size_t i = 0; i < n; i++) m = a[i] > m ? a[i] : m;
    return m;
}

// the device address of pinned host memory (NULL if it is not mapped)
void* host_dev_ptr(void* p) {
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return d;
}

bool d2h_by_kernel() {
    static const bool k = !(getenv("HD_HOST_D2H") && strcmp(getenv("HD_HOST_D2H"), "dma") == 0);
    return k;
}

bool is_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();   // pageable memory is reported as an error on some runtimes
        return false;
    }
    return a.type == hipMemoryTypeHost || a.type == hipMemoryTypeManaged;
}

// memcpy with host threads for large copies
void par_copy(void* dst, const void* src, size_t n) {
    const size_t kMin = 4u << 20;
    unsigned t = std::min<unsigned>(8u, std::max(1u, std::thread::hardware_concurrency()));
    if (n < kMin || t <= 1) {
        memcpy(dst, src, n);
        return;
    }
    t = (unsigned)std::min<size_t>(t, n / kMin + 1);
    const size_t per = (n + t - 1) / t;
    std::vector<std::thread> th;
    for (unsigned k = 0; k < t; k++) {
        const size_t lo = k * per, hi = std::min(n, lo + per);
        if (lo >= hi) break;
        th.emplace_back([=] { memcpy((char*)dst + lo, (const char*)src + lo, hi - lo); });
    }
    for (auto& x : th) x.join();
}

int grow_pinned(hd_ctx* ctx, void** p, size_t* cap, size_t need) {
    if (need <= *cap) return HD_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t want = need + need / 4;
    HCHK(hipHostMalloc(p, want, hipHostMallocDefault), "pinned staging");
    *cap = want;
    return HD_OK;
}

// wait for the slot's ticket and deliver its staged outputs
int complete(hd_ctx* ctx, HostSlot& s) {
    if (!s.ticket) return HD_OK;
    HCHK(hipEventSynchronize(s.done), "host pipeline wait");
    for (const auto& c : s.deliver) par_copy(c.dst, c.src, c.n);
    s.deliver.clear();
    s.ticket = 0;
    return HD_OK;
}

// Each pipeline's stream gets a hardware queue of its own: a stream created
// with a CU mask (here every CU) is given a dedicated queue, while ordinary
// streams share the device's GPU_MAX_HW_QUEUES (4).  Two pipelines on one
// shared queue run in FIFO order, so one pipeline's output-store kernel
// (~0.7 ms of PCIe writes per 1M) held back the other's expansion and
// verification (rocprofv3 trace, round 4).  HD_HOST_CUMASK=0 uses ordinary
// streams (A/B).
bool host_cumask_streams() {
    static const bool on = !(getenv("HD_HOST_CUMASK") && strcmp(getenv("HD_HOST_CUMASK"), "0") == 0);
    return on;
}

int slot_init(hd_ctx* ctx, HostSlot& s) {
    if (s.stream) return HD_OK;
    bool made = false;
    if (host_cumask_streams()) {
        const int ncu = std::max(ctx->n_cu, 1);
        std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0xFFFFFFFFu);
        if (ncu % 32) mask.back() = (1u << (ncu % 32)) - 1u;
        made = hipExtStreamCreateWithCUMask(&s.stream, (uint32_t)mask.size(), mask.data()) == hipSuccess;
        if (!made) (void)hipGetLastError();
    }
    if (!made) HCHK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking), "host pipeline stream");
    HCHK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming), "host pipeline event");
    return HD_OK;
}

}  // namespace

void hd_host_release(hd_ctx* ctx) {
    HostPipe* p = ctx ? ctx->host : nullptr;
    if (!p) return;
    for (HostSlot& s : p->slot) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        for (DevBuf& b : s.col)
            if (b.p) (void)hipFree(b.p);
        for (DevBuf* b : {&s.verdict, &s.rec, &s.bitmap})
            if (b->p) (void)hipFree(b->p);
        if (s.hin) (void)hipHostFree(s.hin);
        if (s.hout) (void)hipHostFree(s.hout);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.stream) (void)hipStreamDestroy(s.stream);
    }
    delete p;
    ctx->host = nullptr;
}

namespace {

// One submit: the host columns `cols` (NULL src: absent) go to the slot's
// device columns (pinned ones by DMA, pageable ones through the staging);
// with `cb` the compact batch's From / value columns are expanded on the
// device first; then hd_verify_batch_device and the outputs.
struct Col { const void* src; size_t sz; };
struct CompactInfo { uint32_t n_sig, n_esc; };

int submit_impl(hd_ctx* ctx, uint32_t n, const Col (&cols)[HC_N], const CompactInfo* cb, uint8_t* verdict,
                uint8_t* recovered32, uint32_t* valid_bitmap, uint64_t* ticket) {
    (void)hipSetDevice(ctx->device);
    if (!ctx->host) ctx->host = new (std::nothrow) HostPipe();
    if (!ctx->host) return HD_ENOMEM;
    HostPipe* p = ctx->host;
    const uint64_t t = p->next++;
    HostSlot& s = p->slot[(t - 1) % HD_HOST_SLOTS];
    int rc = complete(ctx, s);
    if (rc) return rc;
    if ((rc = slot_init(ctx, s))) return rc;
    *ticket = t;
    if (n == 0) return HD_OK;
    size_t stage = 0;
    bool pinned[HC_N];
    for (int k = 0; k < HC_N; k++) {
        pinned[k] = cols[k].src && is_pinned(cols[k].src);
        if (cols[k].src && !pinned[k]) stage += (cols[k].sz + 255) & ~(size_t)255;
    }
    if (stage && (rc = grow_pinned(ctx, &s.hin, &s.hin_cap, stage))) return rc;
    const void* dst[HC_N];
    size_t off = 0;
    for (int k = 0; k < HC_N; k++) {
        dst[k] = nullptr;
        if (!cols[k].src) continue;
        if ((rc = hd_dev_grow(ctx, &s.col[k].p, &s.col[k].cap, cols[k].sz))) return rc;
        const void* src = cols[k].src;
        if (!pinned[k]) {
            void* st = (char*)s.hin + off;
            par_copy(st, src, cols[k].sz);
            off += (cols[k].sz + 255) & ~(size_t)255;
            src = st;
        }
        HCHK(hipMemcpyAsync(s.col[k].p, src, cols[k].sz, hipMemcpyHostToDevice, s.stream), "submit upload");
        dst[k] = s.col[k].p;
    }
    if (cb) {
        // From and value rows from the uploaded indices and dictionaries
        if ((rc = hd_dev_grow(ctx, &s.col[HC_FROM].p, &s.col[HC_FROM].cap, 32 * (size_t)n))) return rc;
        if ((rc = hd_dev_grow(ctx, &s.col[HC_VALUE].p, &s.col[HC_VALUE].cap, 32 * (size_t)n))) return rc;
        dst[HC_FROM] = s.col[HC_FROM].p;
        dst[HC_VALUE] = s.col[HC_VALUE].p;
        const uint32_t blocks = (uint32_t)((2 * (size_t)n + 255) / 256);
        k_compact_expand<<<blocks, 256, 0, s.stream>>>(
            n, (const uint16_t*)dst[HC_FIDX], (const uint16_t*)dst[HC_VIDX], (const uint4*)ctx->d_sig_caller,
            cb->n_sig, (const uint4*)dst[HC_ESC], (const uint4*)dst[HC_VALS], (uint4*)s.col[HC_FROM].p,
            (uint4*)s.col[HC_VALUE].p);
        HCHK(hipGetLastError(), "k_compact_expand");
    }
    hd_batch db{n,
                (const uint8_t*)dst[HC_TYPE],
                (const int64_t*)dst[HC_H],
                (const int64_t*)dst[HC_R],
                (const int64_t*)dst[HC_VR],
                (const uint8_t*)dst[HC_VALUE],
                (const uint8_t*)dst[HC_FROM],
                (const uint8_t*)dst[HC_SIG]};
    const size_t nwords = (n + 31) / 32;
    if ((rc = hd_dev_grow(ctx, &s.verdict.p, &s.verdict.cap, n))) return rc;
    if (recovered32 && (rc = hd_dev_grow(ctx, &s.rec.p, &s.rec.cap, 32 * (size_t)n))) return rc;
    if (valid_bitmap && (rc = hd_dev_grow(ctx, &s.bitmap.p, &s.bitmap.cap, 4 * nwords))) return rc;
    rc = hd_verify_batch_device(ctx, &db, (uint8_t*)s.verdict.p, recovered32 ? (uint8_t*)s.rec.p : nullptr, nullptr,
                                valid_bitmap ? (uint32_t*)s.bitmap.p : nullptr, s.stream);
    if (rc) return rc;
    // outputs: straight into pinned caller buffers, else into staging and
    // copied at completion
    struct Out { void* dst; const void* dev; size_t sz; };
    const Out outs[3] = {{verdict, s.verdict.p, n},
                         {recovered32, s.rec.p, 32 * (size_t)n},
                         {valid_bitmap, s.bitmap.p, 4 * nwords}};
    size_t ostage = 0;
    for (const Out& o : outs)
        if (o.dst && !is_pinned(o.dst)) ostage += (o.sz + 255) & ~(size_t)255;
    if (ostage && (rc = grow_pinned(ctx, &s.hout, &s.hout_cap, ostage))) return rc;
    off = 0;
    s.deliver.clear();
    HostOut ho{};
    int nk = 0;
    for (int k = 0; k < 3; k++) {
        const Out& o = outs[k];
        if (!o.dst) continue;
        void* dst = o.dst;
        if (!is_pinned(o.dst)) {   // into staging, delivered at completion
            dst = (char*)s.hout + off;
            off += (o.sz + 255) & ~(size_t)255;
            s.deliver.push_back({o.dst, dst, o.sz});
        }
        void* ddev = d2h_by_kernel() ? host_dev_ptr(dst) : nullptr;
        if (ddev) {
            ho.dst[k] = (uint8_t*)ddev;
            ho.src[k] = (const uint8_t*)o.dev;
            ho.n[k] = o.sz;
            nk++;
        } else {
            HCHK(hipMemcpyAsync(dst, o.dev, o.sz, hipMemcpyDeviceToHost, s.stream), "submit download");
        }
    }
    if (nk) {
        k_host_store<<<std::max(ctx->n_cu, 1) * 2, 256, 0, s.stream>>>(ho);
        HCHK(hipGetLastError(), "k_host_store");
    }
    HCHK(hipEventRecord(s.done, s.stream), "submit record");
    s.ticket = t;
    return HD_OK;
}

}  // namespace

extern "C" {

// A stream on a hardware queue of its own: a CU-mask stream with every CU set
// (ordinary streams share the device's GPU_MAX_HW_QUEUES queues round robin,
// and a cross-stream wait queued in a shared queue holds back every stream
// mapped to it).  Falls back to an ordinary non-blocking stream.
int hd_stream_create_dedicated(hd_ctx* ctx, void** stream) {
    if (!ctx || !stream) return HD_EINVAL;
    (void)hipSetDevice(ctx->device);
    hipStream_t st = nullptr;
    const int ncu = std::max(ctx->n_cu, 1);
    std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0xFFFFFFFFu);
    if (ncu % 32) mask.back() = (1u << (ncu % 32)) - 1u;
    if (hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
        (void)hipGetLastError();
        const hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
        if (e != hipSuccess) return hd_ctx_fail(ctx, e, "hd_stream_create_dedicated");
    }
    *stream = st;
    return HD_OK;
}

int hd_stream_destroy(hd_ctx* ctx, void* stream) {
    if (!ctx || !stream) return HD_EINVAL;
    (void)hipSetDevice(ctx->device);
    const hipError_t e = hipStreamDestroy((hipStream_t)stream);
    return e == hipSuccess ? HD_OK : hd_ctx_fail(ctx, e, "hd_stream_destroy");
}


int hd_verify_submit(hd_ctx* ctx, const hd_batch* batch, uint8_t* verdict, uint8_t* recovered32,
                     uint32_t* valid_bitmap, uint64_t* ticket) {
    if (!ctx || !batch || !verdict || !ticket) return HD_EINVAL;
    if (batch->n && (!batch->type || !batch->height || !batch->round || !batch->value32 || !batch->from32 ||
                     !batch->sig65))
        return HD_EINVAL;
    const uint32_t n = batch->n;
    const Col cols[HC_N] = {{batch->type, n},
                            {batch->height, 8 * (size_t)n},
                            {batch->round, 8 * (size_t)n},
                            {batch->valid_round, 8 * (size_t)n},
                            {batch->value32, 32 * (size_t)n},
                            {batch->from32, 32 * (size_t)n},
                            {batch->sig65, 65 * (size_t)n},
                            {nullptr, 0}, {nullptr, 0}, {nullptr, 0}, {nullptr, 0}};
    return submit_impl(ctx, n, cols, nullptr, verdict, recovered32, valid_bitmap, ticket);
}

int hd_verify_submit_compact(hd_ctx* ctx, const hd_batch_compact* batch, uint8_t* verdict, uint8_t* recovered32,
                             uint32_t* valid_bitmap, uint64_t* ticket) {
    if (!ctx || !batch || !verdict || !ticket) return HD_EINVAL;
    const uint32_t n = batch->n;
    if (n && (!batch->type || !batch->height || !batch->round || !batch->from_idx || !batch->value_idx ||
              !batch->sig65 || !batch->values32 || batch->n_values == 0))
        return HD_EINVAL;
    if ((batch->n_escape && !batch->escape32) || (size_t)ctx->n_sig_caller + batch->n_escape > 65536u ||
        batch->n_values > 65536u)
        return HD_EINVAL;
    if (n) {
        // every index names a row (the expansion reads no further)
        if (max_u16(batch->from_idx, n) >= ctx->n_sig_caller + batch->n_escape) return HD_EINVAL;
        if (max_u16(batch->value_idx, n) >= batch->n_values) return HD_EINVAL;
    }
    const CompactInfo ci{ctx->n_sig_caller, batch->n_escape};
    // (no escape rows: no upload -- a tiny copy would run as a blit kernel
    // queued behind another pipeline's kernels -- and the expansion, whose
    // indices were checked above, never reads the table)
    const Col cols[HC_N] = {{batch->type, n},
                            {batch->height, 8 * (size_t)n},
                            {batch->round, 8 * (size_t)n},
                            {batch->valid_round, 8 * (size_t)n},
                            {nullptr, 0},
                            {nullptr, 0},
                            {batch->sig65, 65 * (size_t)n},
                            {batch->from_idx, 2 * (size_t)n},
                            {batch->value_idx, 2 * (size_t)n},
                            {batch->n_escape ? (const void*)batch->escape32 : nullptr, 32 * (size_t)batch->n_escape},
                            {batch->values32, 32 * (size_t)batch->n_values}};
    return submit_impl(ctx, n, cols, &ci, verdict, recovered32, valid_bitmap, ticket);
}

int hd_verify_wait(hd_ctx* ctx, uint64_t ticket) {
    if (!ctx || ticket == 0) return HD_EINVAL;
    if (!ctx->host) return ticket == 0 ? HD_EINVAL : HD_OK;
    (void)hipSetDevice(ctx->device);
    for (HostSlot& s : ctx->host->slot)
        if (s.ticket == ticket) return complete(ctx, s);
    return ticket < ctx->host->next ? HD_OK : HD_EINVAL;
}

int hd_host_alloc(size_t bytes, void** out) {
    if (!out) return HD_EINVAL;
    *out = nullptr;
    if (hipHostMalloc(out, std::max<size_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) return HD_ENOMEM;
    return HD_OK;
}

int hd_host_free(void* p) {
    if (!p) return HD_OK;
    return hipHostFree(p) == hipSuccess ? HD_OK : HD_EINVAL;
}

}  // extern "C"
