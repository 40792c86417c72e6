// hd_multi.hip -- one batch verified and tallied on several GPUs of one node,
// behind the C ABI (include/hd_verify.h hd_multi_*).
//
// One context per device, one host thread per device while the devices work,
// and one RCCL communicator over the devices (ncclCommInitAll: the
// single-process, multi-device form a cgo caller -- one Go Replica -- needs).
// Per hd_multi_verify_batch:
//   1. device k uploads the batch metadata (type, height, round, valid round,
//      value, From: 81 B/message, replicated -- the tally needs every round's
//      messages) and the signatures of its shard only;
//   2. device k verifies its contiguous, 32-aligned shard (the known-key
//      check / full recovery of hd_verify_batch_device), writing its bitmap
//      words in place into a whole-batch bitmap;
//   3. one in-place ncclAllGather of those words over xGMI (the only
//      collective on the data path) gives every device the whole bitmap;
//   4. device k tallies only the rounds hd_tally_partition_of gives it
//      (hd_tally_device_bitmap_part); the host merges the small per-device
//      tables in first-batch-index order -- the single-device output.
// RCCL takes one rank per device; when a device is listed twice (e.g. two
// contexts on one GPU in a test) step 3 is done with device-to-device copies.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <numeric>
#include <set>
#include <thread>
#include <vector>

#include "../../include/hd_verify.h"
#include "hd_internal.h"

namespace {

struct Dev {
    hd_ctx* ctx = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;   // the ctx's stream
    DevBuf sig, verdict, rec, bitmap;
    uint32_t lo = 0, hi = 0;        // shard
    // this device's tally partition (host)
    std::vector<int64_t> ch, cr, hh, hr;
    std::vector<uint8_t> ct, dup;
    std::vector<uint32_t> crep, cn, hprev, hprec, hany, hrep;
    uint32_t n_counts = 0, n_hr = 0;
    int rc = HD_OK;
};

}  // namespace

struct hd_multi {
    std::vector<Dev> dev;
    std::vector<ncclComm_t> comm;   // empty: copy exchange
};

namespace {

int fail(Dev& d, hipError_t e, const char* what) { return hd_ctx_fail(d.ctx, e, what); }

#define MCHK(expr, what)                          \
    do {                                          \
        hipError_t e_ = (expr);                   \
        if (e_ != hipSuccess) return fail(d, e_, what); \
    } while (0)

// shard k of n over G devices: contiguous, a multiple of 32 messages except
// the last (the bitmap words of the shards never overlap)
void shard(uint32_t n, int G, int k, uint32_t* lo, uint32_t* hi, uint32_t* per) {
    uint32_t p = (uint32_t)(((uint64_t)n + G - 1) / G);
    p = (p + 31u) & ~31u;
    *per = p;
    *lo = std::min<uint64_t>(n, (uint64_t)k * p);
    *hi = std::min<uint64_t>(n, (uint64_t)*lo + p);
}

// steps 1-2 on device d
int verify_shard(Dev& d, const hd_batch* hb, uint32_t words_per_shard, int G, int k, bool want_rec, hd_batch* dfull) {
    (void)hipSetDevice(d.device);
    hd_batch meta = *hb;
    meta.sig65 = nullptr;
    int rc = hd_upload_batch(d.ctx, &meta, dfull);
    if (rc) return rc;
    const uint32_t m = d.hi - d.lo;
    const size_t words = (size_t)words_per_shard * G;
    if ((rc = hd_dev_grow(d.ctx, &d.bitmap.p, &d.bitmap.cap, 4 * words))) return rc;
    MCHK(hipMemsetAsync(d.bitmap.p, 0, 4 * words, d.stream), "clear bitmap");
    if (m == 0) return HD_OK;
    if ((rc = hd_dev_grow(d.ctx, &d.sig.p, &d.sig.cap, 65 * (size_t)m))) return rc;
    if ((rc = hd_dev_grow(d.ctx, &d.verdict.p, &d.verdict.cap, m))) return rc;
    if (want_rec && (rc = hd_dev_grow(d.ctx, &d.rec.p, &d.rec.cap, 32 * (size_t)m))) return rc;
    MCHK(hipMemcpyAsync(d.sig.p, hb->sig65 + 65 * (size_t)d.lo, 65 * (size_t)m, hipMemcpyHostToDevice, d.stream),
         "signature upload");
    const size_t lo = d.lo;
    hd_batch sh{m,
                dfull->type + lo,
                dfull->height + lo,
                dfull->round + lo,
                dfull->valid_round ? dfull->valid_round + lo : nullptr,
                dfull->value32 + 32 * lo,
                dfull->from32 + 32 * lo,
                (const uint8_t*)d.sig.p};
    uint32_t* bits = (uint32_t*)d.bitmap.p + (size_t)words_per_shard * k;
    rc = hd_verify_batch_device(d.ctx, &sh, (uint8_t*)d.verdict.p, want_rec ? (uint8_t*)d.rec.p : nullptr, nullptr,
                                bits, d.stream);
    if (rc) return rc;
    MCHK(hipStreamSynchronize(d.stream), "verify sync");
    return HD_OK;
}

// step 4 on device d: its partition of the rounds, into host vectors
int tally_part(Dev& d, const hd_batch* dfull, int G, int k) {
    (void)hipSetDevice(d.device);
    const uint32_t n = dfull->n;
    d.ch.resize(n); d.cr.resize(n); d.ct.resize(n); d.crep.resize(n); d.cn.resize(n);
    d.hh.resize(n); d.hr.resize(n); d.hprev.resize(n); d.hprec.resize(n); d.hany.resize(n); d.hrep.resize(n);
    d.dup.resize(n);
    hd_tally_out o{};
    o.cap_counts = n;
    o.count_height = d.ch.data(); o.count_round = d.cr.data(); o.count_type = d.ct.data();
    o.count_rep = d.crep.data(); o.count_n = d.cn.data();
    o.cap_hr = n;
    o.hr_height = d.hh.data(); o.hr_round = d.hr.data(); o.hr_prevotes = d.hprev.data();
    o.hr_precommits = d.hprec.data(); o.hr_any = d.hany.data(); o.hr_rep = d.hrep.data();
    o.dup = d.dup.data();
    const int rc = hd_tally_device_bitmap_part(d.ctx, dfull, (const uint32_t*)d.bitmap.p, (uint32_t)k, (uint32_t)G, &o,
                                               d.stream);
    d.n_counts = o.n_counts;
    d.n_hr = o.n_hr;
    return rc;
}

template <typename F>
int on_all_devices(hd_multi* m, F f) {
    const int G = (int)m->dev.size();
    std::vector<std::thread> th;
    for (int k = 0; k < G; k++) th.emplace_back([&, k] { m->dev[k].rc = f(m->dev[k], k); });
    for (auto& t : th) t.join();
    for (auto& d : m->dev)
        if (d.rc) return d.rc;
    return HD_OK;
}

// the merged tally into the caller's arrays (HD_ECAP when they are too small)
int merge_tally(hd_multi* m, uint32_t n, hd_tally_out* out) {
    struct Ref { uint32_t rep; int dev; uint32_t row; };
    std::vector<Ref> cr, hr;
    for (int k = 0; k < (int)m->dev.size(); k++) {
        const Dev& d = m->dev[k];
        for (uint32_t j = 0; j < d.n_counts; j++) cr.push_back({d.crep[j], k, j});
        for (uint32_t j = 0; j < d.n_hr; j++) hr.push_back({d.hrep[j], k, j});
    }
    auto by_rep = [](const Ref& a, const Ref& b) { return a.rep < b.rep; };
    std::sort(cr.begin(), cr.end(), by_rep);
    std::sort(hr.begin(), hr.end(), by_rep);
    out->n_counts = (uint32_t)cr.size();
    out->n_hr = (uint32_t)hr.size();
    if (out->n_counts > out->cap_counts || out->n_hr > out->cap_hr) return HD_ECAP;
    for (size_t j = 0; j < cr.size(); j++) {
        const Dev& d = m->dev[cr[j].dev];
        const uint32_t r = cr[j].row;
        out->count_height[j] = d.ch[r];
        out->count_round[j] = d.cr[r];
        out->count_type[j] = d.ct[r];
        out->count_rep[j] = d.crep[r];
        out->count_n[j] = d.cn[r];
    }
    for (size_t j = 0; j < hr.size(); j++) {
        const Dev& d = m->dev[hr[j].dev];
        const uint32_t r = hr[j].row;
        out->hr_height[j] = d.hh[r];
        out->hr_round[j] = d.hr[r];
        out->hr_prevotes[j] = d.hprev[r];
        out->hr_precommits[j] = d.hprec[r];
        out->hr_any[j] = d.hany[r];
        if (out->hr_rep) out->hr_rep[j] = d.hrep[r];
    }
    if (out->dup) {
        // a partition that does not own a message's round reports 3
        memset(out->dup, 3, n);
        for (const Dev& d : m->dev)
            for (uint32_t i = 0; i < n; i++) out->dup[i] = std::min(out->dup[i], d.dup[i]);
    }
    return HD_OK;
}

}  // namespace

extern "C" {

int hd_multi_create(int ngpus, const int* devices, hd_multi** out) {
    if (ngpus <= 0 || !out) return HD_EINVAL;
    *out = nullptr;
    int have = 0;
    if (hipGetDeviceCount(&have) != hipSuccess || have <= 0) return HD_EDEVICE;
    std::vector<int> list(ngpus);
    for (int k = 0; k < ngpus; k++) {
        list[k] = devices ? devices[k] : k;
        if (list[k] < 0 || list[k] >= have) return HD_EINVAL;
    }
    hd_multi* m = new (std::nothrow) hd_multi();
    if (!m) return HD_ENOMEM;
    m->dev.resize(ngpus);
    for (int k = 0; k < ngpus; k++) {
        Dev& d = m->dev[k];
        d.device = list[k];
        const int rc = hd_ctx_create(list[k], &d.ctx);
        if (rc) {
            hd_multi_destroy(m);
            return rc;
        }
        d.stream = d.ctx->stream;
    }
    if (std::set<int>(list.begin(), list.end()).size() == list.size()) {
        m->comm.resize(ngpus);
        if (ncclCommInitAll(m->comm.data(), ngpus, list.data()) != ncclSuccess) {
            m->comm.clear();
            hd_multi_destroy(m);
            return HD_EDEVICE;
        }
    }
    *out = m;
    return HD_OK;
}

int hd_multi_destroy(hd_multi* m) {
    if (!m) return HD_EINVAL;
    for (ncclComm_t c : m->comm) (void)ncclCommDestroy(c);
    for (Dev& d : m->dev) {
        if (!d.ctx) continue;
        (void)hipSetDevice(d.device);
        (void)hipStreamSynchronize(d.stream);
        for (DevBuf* b : {&d.sig, &d.verdict, &d.rec, &d.bitmap})
            if (b->p) (void)hipFree(b->p);
        hd_ctx_destroy(d.ctx);
    }
    delete m;
    return HD_OK;
}

int hd_multi_size(hd_multi* m, int* ngpus, int* uses_rccl) {
    if (!m) return HD_EINVAL;
    if (ngpus) *ngpus = (int)m->dev.size();
    if (uses_rccl) *uses_rccl = m->comm.empty() ? 0 : 1;
    return HD_OK;
}

hd_ctx* hd_multi_ctx(hd_multi* m, int k) {
    if (!m || k < 0 || k >= (int)m->dev.size()) return nullptr;
    return m->dev[k].ctx;
}

int hd_multi_set_signatories(hd_multi* m, const uint8_t* sigs32, uint32_t n) {
    if (!m) return HD_EINVAL;
    return on_all_devices(m, [&](Dev& d, int) { return hd_set_signatories(d.ctx, sigs32, n); });
}

int hd_multi_set_pubkey_format(hd_multi* m, int format) {
    if (!m) return HD_EINVAL;
    for (Dev& d : m->dev) {
        const int rc = hd_ctx_set_pubkey_format(d.ctx, format);
        if (rc) return rc;
    }
    return HD_OK;
}

int hd_multi_verify_batch(hd_multi* m, const hd_batch* batch, uint8_t* verdict, uint8_t* recovered32,
                          uint32_t* valid_bitmap, hd_tally_out* tally) {
    if (!m || !batch || !verdict) return HD_EINVAL;
    const uint32_t n = batch->n;
    if (tally) tally->n_counts = tally->n_hr = 0;
    if (n == 0) return HD_OK;
    if (!batch->type || !batch->height || !batch->round || !batch->value32 || !batch->from32 || !batch->sig65)
        return HD_EINVAL;
    if (tally && (!tally->count_height || !tally->count_round || !tally->count_type || !tally->count_rep ||
                  !tally->count_n || !tally->hr_height || !tally->hr_round || !tally->hr_prevotes ||
                  !tally->hr_precommits || !tally->hr_any))
        return HD_EINVAL;
    const int G = (int)m->dev.size();
    uint32_t per = 0;
    for (int k = 0; k < G; k++) shard(n, G, k, &m->dev[k].lo, &m->dev[k].hi, &per);
    const uint32_t wps = per / 32;   // bitmap words per shard
    std::vector<hd_batch> dfull(G);
    // 1-2: upload and verify every shard, one host thread per device
    int rc = on_all_devices(m, [&](Dev& d, int k) {
        return verify_shard(d, batch, wps, G, k, recovered32 != nullptr, &dfull[k]);
    });
    if (rc) return rc;
    // 3: every device gets the whole bitmap
    if (G > 1) {
        if (!m->comm.empty()) {
            if (ncclGroupStart() != ncclSuccess) return HD_EDEVICE;
            for (int k = 0; k < G; k++) {
                Dev& d = m->dev[k];
                uint32_t* bm = (uint32_t*)d.bitmap.p;
                if (ncclAllGather(bm + (size_t)wps * k, bm, wps, ncclUint32, m->comm[k], d.stream) != ncclSuccess) {
                    (void)ncclGroupEnd();
                    return HD_EDEVICE;
                }
            }
            if (ncclGroupEnd() != ncclSuccess) return HD_EDEVICE;
        } else {
            for (int k = 0; k < G; k++)
                for (int j = 0; j < G; j++) {
                    if (j == k) continue;
                    Dev& d = m->dev[k];
                    const size_t off = (size_t)wps * j;
                    MCHK(hipMemcpyPeerAsync((uint32_t*)d.bitmap.p + off, d.device,
                                            (const uint32_t*)m->dev[j].bitmap.p + off, m->dev[j].device, 4 * (size_t)wps,
                                            d.stream),
                         "bitmap exchange");
                }
        }
        for (Dev& d : m->dev) {
            (void)hipSetDevice(d.device);
            MCHK(hipStreamSynchronize(d.stream), "bitmap exchange sync");
        }
    }
    // outputs of the shards
    for (int k = 0; k < G; k++) {
        Dev& d = m->dev[k];
        const uint32_t len = d.hi - d.lo;
        if (!len) continue;
        (void)hipSetDevice(d.device);
        MCHK(hipMemcpy(verdict + d.lo, d.verdict.p, len, hipMemcpyDeviceToHost), "verdict download");
        if (recovered32)
            MCHK(hipMemcpy(recovered32 + 32 * (size_t)d.lo, d.rec.p, 32 * (size_t)len, hipMemcpyDeviceToHost),
                 "recovered download");
    }
    if (valid_bitmap) {
        Dev& d = m->dev[0];
        (void)hipSetDevice(d.device);
        MCHK(hipMemcpy(valid_bitmap, d.bitmap.p, 4 * (size_t)((n + 31) / 32), hipMemcpyDeviceToHost),
             "bitmap download");
    }
    if (!tally) return HD_OK;
    // 4: each device its rounds; merged on the host
    rc = on_all_devices(m, [&](Dev& d, int k) { return tally_part(d, &dfull[k], G, k); });
    if (rc) return rc;
    return merge_tally(m, n, tally);
}

}  // extern "C"
