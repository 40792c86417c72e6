// hd_multi.hip -- one batch verified and tallied on several GPUs of one node,
// behind the C ABI (include/hd_verify.h hd_multi_*).
//
// One context per device, one host thread per device while the devices work,
// and one RCCL communicator over the devices (ncclCommInitAll: the
// single-process, multi-device form a cgo caller -- one Go Replica -- needs).
// Per hd_multi_verify_batch:
//   1. device k uploads its contiguous, 32-aligned shard only (every column:
//      146 B per message, 1/G of the batch per device over PCIe);
//   2. device k verifies it (the known-key check / full recovery of
//      hd_verify_batch_device): verdicts, signatories, its bitmap words;
//   3. with a tally: device k routes its shard's candidates (VALID Prevotes /
//      Precommits) to the owners of their rounds (hd_route_candidates_device,
//      64-byte rows); one grouped ncclSend / ncclRecv moves every group over
//      xGMI (the only collective on the data path); device o rebuilds a batch
//      from what it received, in global index order, and tallies it
//      (hd_unroute_device + hd_tally_routed_device);
//   4. the host merges the owners' disjoint tables in first-batch-index order
//      -- the single-device output -- and scatters their per-row dup
//      classification to the global indices (3 for non-candidates).
// RCCL takes one rank per device; when a device is listed twice (e.g. two
// contexts on one GPU in a test) step 3 moves the groups with device copies.
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
    DevBuf verdict, rec, bitmap;
    DevBuf rows, recv, gidx, rb[5];  // route rows out / in, global indices, the rebuilt batch (type h r value from)
    uint32_t lo = 0, hi = 0;        // shard
    std::vector<uint32_t> counts;   // route rows per owner
    uint32_t m = 0;                 // rows received
    // this device's tally of the rounds it owns (host)
    std::vector<int64_t> ch, cr, hh, hr;
    std::vector<uint8_t> ct, dup;
    std::vector<uint32_t> crep, cn, hprev, hprec, hany, hrep, gidx_h;
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

// steps 1-2 on device d: its shard only
int verify_shard(Dev& d, const hd_batch* hb, bool want_rec, hd_batch* dshard) {
    (void)hipSetDevice(d.device);
    const uint32_t m = d.hi - d.lo;
    dshard->n = 0;
    if (m == 0) return HD_OK;
    const size_t lo = d.lo;
    hd_batch sh{m,
                hb->type + lo,
                hb->height + lo,
                hb->round + lo,
                hb->valid_round ? hb->valid_round + lo : nullptr,
                hb->value32 + 32 * lo,
                hb->from32 + 32 * lo,
                hb->sig65 + 65 * lo};
    int rc = hd_upload_batch(d.ctx, &sh, dshard);
    if (rc) return rc;
    if ((rc = hd_dev_grow(d.ctx, &d.bitmap.p, &d.bitmap.cap, 4 * (size_t)((m + 31) / 32)))) return rc;
    if ((rc = hd_dev_grow(d.ctx, &d.verdict.p, &d.verdict.cap, m))) return rc;
    if (want_rec && (rc = hd_dev_grow(d.ctx, &d.rec.p, &d.rec.cap, 32 * (size_t)m))) return rc;
    rc = hd_verify_batch_device(d.ctx, dshard, (uint8_t*)d.verdict.p, want_rec ? (uint8_t*)d.rec.p : nullptr, nullptr,
                                (uint32_t*)d.bitmap.p, d.stream);
    if (rc) return rc;
    MCHK(hipStreamSynchronize(d.stream), "verify sync");
    return HD_OK;
}

// step 3a on device d: its candidates as route rows, grouped by owner
int route_shard(Dev& d, const hd_batch* dshard, int G) {
    (void)hipSetDevice(d.device);
    d.counts.assign(G, 0);
    const uint32_t m = d.hi - d.lo;
    if (m == 0) return HD_OK;
    int rc = hd_dev_grow(d.ctx, &d.rows.p, &d.rows.cap, (size_t)HD_ROUTE_ROW_BYTES * m);
    if (rc) return rc;
    return hd_route_candidates_device(d.ctx, dshard, (const uint32_t*)d.bitmap.p, d.lo, (uint32_t)G,
                                      (uint8_t*)d.rows.p, m, d.counts.data(), d.stream);
}

// step 3c on device d: the received rows -> a batch -> the tally of its
// rounds (host vectors sized by what it received)
int tally_owned(Dev& d, bool want_dup) {
    (void)hipSetDevice(d.device);
    const uint32_t m = d.m;
    d.n_counts = d.n_hr = 0;
    if (m == 0) return HD_OK;
    const size_t sz[5] = {m, 8 * (size_t)m, 8 * (size_t)m, 32 * (size_t)m, 32 * (size_t)m};
    for (int k = 0; k < 5; k++) {
        const int rc = hd_dev_grow(d.ctx, &d.rb[k].p, &d.rb[k].cap, sz[k]);
        if (rc) return rc;
    }
    int rc = hd_dev_grow(d.ctx, &d.gidx.p, &d.gidx.cap, 4 * (size_t)m);
    if (rc) return rc;
    hd_batch_out o{(uint8_t*)d.rb[0].p, (int64_t*)d.rb[1].p, (int64_t*)d.rb[2].p, nullptr, (uint8_t*)d.rb[3].p,
                   (uint8_t*)d.rb[4].p, nullptr, nullptr};
    rc = hd_unroute_device(d.ctx, (const uint8_t*)d.recv.p, m, &o, (uint32_t*)d.gidx.p, d.stream);
    if (rc) return rc;
    hd_batch b{m, o.type, o.height, o.round, nullptr, o.value32, o.from32, nullptr};
    d.ch.resize(m); d.cr.resize(m); d.ct.resize(m); d.crep.resize(m); d.cn.resize(m);
    d.hh.resize(m); d.hr.resize(m); d.hprev.resize(m); d.hprec.resize(m); d.hany.resize(m); d.hrep.resize(m);
    d.dup.resize(want_dup ? m : 0);
    hd_tally_out t{};
    t.cap_counts = m;
    t.count_height = d.ch.data(); t.count_round = d.cr.data(); t.count_type = d.ct.data();
    t.count_rep = d.crep.data(); t.count_n = d.cn.data();
    t.cap_hr = m;
    t.hr_height = d.hh.data(); t.hr_round = d.hr.data(); t.hr_prevotes = d.hprev.data();
    t.hr_precommits = d.hprec.data(); t.hr_any = d.hany.data(); t.hr_rep = d.hrep.data();
    t.dup = want_dup ? d.dup.data() : nullptr;
    rc = hd_tally_routed_device(d.ctx, &b, (const uint32_t*)d.gidx.p, &t, d.stream);
    d.n_counts = t.n_counts;
    d.n_hr = t.n_hr;
    if (rc || !want_dup) return rc;
    d.gidx_h.resize(m);
    MCHK(hipMemcpyAsync(d.gidx_h.data(), d.gidx.p, 4 * (size_t)m, hipMemcpyDeviceToHost, d.stream), "gidx download");
    MCHK(hipStreamSynchronize(d.stream), "gidx download");
    return HD_OK;
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
        // non-candidates 3; each owner's rows at their global indices
        memset(out->dup, 3, n);
        for (const Dev& d : m->dev)
            for (size_t j = 0; j < d.dup.size(); j++) out->dup[d.gidx_h[j]] = d.dup[j];
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
        for (DevBuf* b : {&d.verdict, &d.rec, &d.bitmap, &d.rows, &d.recv, &d.gidx})
            if (b->p) (void)hipFree(b->p);
        for (DevBuf& b : d.rb)
            if (b.p) (void)hipFree(b.p);
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
    std::vector<hd_batch> dshard(G);
    // 1-2: every shard uploaded to and verified on its device
    int rc = on_all_devices(m, [&](Dev& d, int k) { return verify_shard(d, batch, recovered32 != nullptr, &dshard[k]); });
    if (rc) return rc;
    // outputs of the shards (the bitmap words of a shard are its own: shards
    // are whole words except the last)
    for (int k = 0; k < G; k++) {
        Dev& d = m->dev[k];
        const uint32_t len = d.hi - d.lo;
        if (!len) continue;
        (void)hipSetDevice(d.device);
        MCHK(hipMemcpyAsync(verdict + d.lo, d.verdict.p, len, hipMemcpyDeviceToHost, d.stream), "verdict download");
        if (recovered32)
            MCHK(hipMemcpyAsync(recovered32 + 32 * (size_t)d.lo, d.rec.p, 32 * (size_t)len, hipMemcpyDeviceToHost,
                                d.stream),
                 "recovered download");
        if (valid_bitmap)
            MCHK(hipMemcpyAsync(valid_bitmap + d.lo / 32, d.bitmap.p, 4 * (size_t)((len + 31) / 32),
                                hipMemcpyDeviceToHost, d.stream),
                 "bitmap download");
    }
    for (Dev& d : m->dev) {
        (void)hipSetDevice(d.device);
        MCHK(hipStreamSynchronize(d.stream), "output download");
    }
    if (!tally) return HD_OK;
    // 3a: candidates -> route rows grouped by owner
    rc = on_all_devices(m, [&](Dev& d, int k) { return route_shard(d, &dshard[k], G); });
    if (rc) return rc;
    // 3b: the groups to their owners, source-rank order (= global index order)
    std::vector<std::vector<size_t>> soff(G, std::vector<size_t>(G + 1, 0)), roff(G, std::vector<size_t>(G + 1, 0));
    for (int k = 0; k < G; k++)
        for (int o = 0; o < G; o++) {
            soff[k][o + 1] = soff[k][o] + m->dev[k].counts[o];
            roff[o][k + 1] = roff[o][k] + m->dev[k].counts[o];
        }
    const size_t RB = HD_ROUTE_ROW_BYTES;
    for (int o = 0; o < G; o++) {
        Dev& d = m->dev[o];
        d.m = (uint32_t)roff[o][G];
        (void)hipSetDevice(d.device);
        if ((rc = hd_dev_grow(d.ctx, &d.recv.p, &d.recv.cap, RB * std::max<size_t>(d.m, 1)))) return rc;
    }
    if (!m->comm.empty()) {
        if (ncclGroupStart() != ncclSuccess) return HD_EDEVICE;
        for (int k = 0; k < G; k++) {
            Dev& d = m->dev[k];
            for (int o = 0; o < G; o++) {
                const size_t c = m->dev[k].counts[o];   // k -> o
                const size_t r = m->dev[o].counts[k];   // o -> k
                if (c && ncclSend((const char*)d.rows.p + RB * soff[k][o], RB * c, ncclUint8, o, m->comm[k], d.stream) !=
                             ncclSuccess) {
                    (void)ncclGroupEnd();
                    return HD_EDEVICE;
                }
                if (r && ncclRecv((char*)d.recv.p + RB * roff[k][o], RB * r, ncclUint8, o, m->comm[k], d.stream) !=
                             ncclSuccess) {
                    (void)ncclGroupEnd();
                    return HD_EDEVICE;
                }
            }
        }
        if (ncclGroupEnd() != ncclSuccess) return HD_EDEVICE;
    } else {
        for (int k = 0; k < G; k++)
            for (int o = 0; o < G; o++) {
                const size_t c = m->dev[k].counts[o];
                if (!c) continue;
                Dev& d = m->dev[o];
                (void)hipSetDevice(d.device);
                MCHK(hipMemcpyPeerAsync((char*)d.recv.p + RB * roff[o][k], d.device,
                                        (const char*)m->dev[k].rows.p + RB * soff[k][o], m->dev[k].device, RB * c,
                                        d.stream),
                     "route exchange");
            }
    }
    for (Dev& d : m->dev) {
        (void)hipSetDevice(d.device);
        MCHK(hipStreamSynchronize(d.stream), "route exchange sync");
    }
    // 3c-4: each owner tallies its rounds; merged on the host
    rc = on_all_devices(m, [&](Dev& d, int) { return tally_owned(d, tally->dup != nullptr); });
    if (rc) return rc;
    return merge_tally(m, n, tally);
}

}  // extern "C"
