// hd_multi.hip -- one batch verified and tallied on several GPUs of one node,
// behind the C ABI (include/hd_verify.h hd_multi_*).
//
// One context per device, one host thread per device while the devices work,
// and one RCCL communicator over the devices (ncclCommInitAll: the
// single-process, multi-device form a cgo caller -- one Go Replica -- needs).
// Per hd_multi_verify_batch, everything of a device on its context's stream:
//   1. device k uploads its contiguous, 32-aligned shard only (every column:
//      146 B per message, 1/G of the batch per device over PCIe), verifies it
//      (the known-key check / full recovery of hd_verify_batch_device) and
//      queues the download of its verdicts, signatories and bitmap words --
//      no host wait;
//   2. with a tally: device k routes its shard's candidates (VALID Prevotes /
//      Precommits) to the owners of their rounds (hd_route_candidates_device,
//      64-byte rows; its one host read is the group sizes); one grouped
//      ncclSend / ncclRecv moves every group over xGMI (the only collective
//      on the data path);
//   3. device o rebuilds a batch from what it received, in global index order,
//      tallies it (hd_unroute_device + the routed tally) and scatters the
//      per-row duplicate classification to the global indices of an n-byte
//      array of its own, on the device (3 = not a candidate / not owned);
//   4. the classifications merge by minimum on the devices (ncclReduce with
//      ncclMin into device 0: an owner reports 0/1/2 for its rows and 3 for
//      the rest), one download; the owners' small tables -- each already in
//      first-batch-index order -- merge on the host by a k-way merge (no sort).
// RCCL takes one rank per device; when a device is listed twice (e.g. two
// contexts on one GPU in a test) steps 2 and 4 use device copies ordered by
// events.
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
    hipEvent_t routed = nullptr;    // after this device's route rows (copy exchange)
    hipEvent_t owned = nullptr;     // after this device's dup classification (copy exchange)
    DevBuf verdict, rec, bitmap;
    DevBuf rows, recv, gidx, rb[5];  // route rows out / in, global indices, the rebuilt batch (type h r value from)
    DevBuf dupg, dupx;              // classification at global indices (n); device 0: the other owners' (copy exchange)
    uint32_t lo = 0, hi = 0;        // shard
    std::vector<uint32_t> counts;   // route rows per owner
    uint32_t m = 0;                 // rows received
    // this device's tally of the rounds it owns (host; grown, never shrunk)
    std::vector<int64_t> ch, cr, hh, hr;
    std::vector<uint8_t> ct;
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

// step 1 on device d: its shard only, outputs queued for download into the
// caller's arrays (no host wait)
int verify_shard(Dev& d, const hd_batch* hb, uint8_t* verdict, uint8_t* recovered32, uint32_t* valid_bitmap,
                 hd_batch* dshard) {
    const bool want_rec = recovered32 != nullptr;
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
    // the bitmap words of a shard are its own: shards are whole words except the last
    MCHK(hipMemcpyAsync(verdict + d.lo, d.verdict.p, m, hipMemcpyDeviceToHost, d.stream), "verdict download");
    if (recovered32)
        MCHK(hipMemcpyAsync(recovered32 + 32 * lo, d.rec.p, 32 * (size_t)m, hipMemcpyDeviceToHost, d.stream),
             "recovered download");
    if (valid_bitmap)
        MCHK(hipMemcpyAsync(valid_bitmap + d.lo / 32, d.bitmap.p, 4 * (size_t)((m + 31) / 32), hipMemcpyDeviceToHost,
                            d.stream),
             "bitmap download");
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
    rc = hd_route_candidates_device(d.ctx, dshard, (const uint32_t*)d.bitmap.p, d.lo, (uint32_t)G,
                                    (uint8_t*)d.rows.p, m, d.counts.data(), d.stream);
    if (rc) return rc;
    // (the rows are written by a kernel still in flight: a copy exchange on
    // another stream waits for this event)
    MCHK(hipEventRecord(d.routed, d.stream), "route event");
    return HD_OK;
}

// step 3c on device d: the received rows -> a batch -> the tally of its
// rounds (host vectors sized by what it received)
int tally_owned(Dev& d, uint32_t n, bool want_dup) {
    (void)hipSetDevice(d.device);
    const uint32_t m = d.m;
    d.n_counts = d.n_hr = 0;
    if (want_dup) {
        int rc = hd_dev_grow(d.ctx, &d.dupg.p, &d.dupg.cap, n);
        if (rc) return rc;
        MCHK(hipMemsetAsync(d.dupg.p, 3, n, d.stream), "dup clear");
    }
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
    if (d.ch.size() < m) {   // host rows: grown, never shrunk (no per-call reallocation)
        const size_t c = m + m / 4;
        d.ch.resize(c); d.cr.resize(c); d.ct.resize(c); d.crep.resize(c); d.cn.resize(c);
        d.hh.resize(c); d.hr.resize(c); d.hprev.resize(c); d.hprec.resize(c); d.hany.resize(c); d.hrep.resize(c);
    }
    hd_tally_out t{};
    t.cap_counts = m;
    t.count_height = d.ch.data(); t.count_round = d.cr.data(); t.count_type = d.ct.data();
    t.count_rep = d.crep.data(); t.count_n = d.cn.data();
    t.cap_hr = m;
    t.hr_height = d.hh.data(); t.hr_round = d.hr.data(); t.hr_prevotes = d.hprev.data();
    t.hr_precommits = d.hprec.data(); t.hr_any = d.hany.data(); t.hr_rep = d.hrep.data();
    // the classification stays on the device, scattered to global indices
    rc = want_dup ? hd_tally_routed_dup_device(d.ctx, &b, (const uint32_t*)d.gidx.p, &t, (uint8_t*)d.dupg.p, d.stream)
                  : hd_tally_routed_device(d.ctx, &b, (const uint32_t*)d.gidx.p, &t, d.stream);
    d.n_counts = t.n_counts;
    d.n_hr = t.n_hr;
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

// The merged tally into the caller's arrays (HD_ECAP when they are too
// small).  Each owner's rows are in first-batch-index order already (the
// routed tally emits them by rep) and the owners' rep sets are disjoint, so a
// k-way merge by rep gives the single-device order without sorting.
int merge_tally(hd_multi* m, hd_tally_out* out) {
    const int G = (int)m->dev.size();
    uint32_t nc = 0, nh = 0;
    for (const Dev& d : m->dev) {
        nc += d.n_counts;
        nh += d.n_hr;
    }
    out->n_counts = nc;
    out->n_hr = nh;
    if (nc > out->cap_counts || nh > out->cap_hr) return HD_ECAP;
    std::vector<uint32_t> pos(G);
    std::fill(pos.begin(), pos.end(), 0u);
    for (uint32_t j = 0; j < nc; j++) {
        int best = -1;
        for (int k = 0; k < G; k++)
            if (pos[k] < m->dev[k].n_counts && (best < 0 || m->dev[k].crep[pos[k]] < m->dev[best].crep[pos[best]]))
                best = k;
        const Dev& d = m->dev[best];
        const uint32_t r = pos[best]++;
        out->count_height[j] = d.ch[r];
        out->count_round[j] = d.cr[r];
        out->count_type[j] = d.ct[r];
        out->count_rep[j] = d.crep[r];
        out->count_n[j] = d.cn[r];
    }
    std::fill(pos.begin(), pos.end(), 0u);
    for (uint32_t j = 0; j < nh; j++) {
        int best = -1;
        for (int k = 0; k < G; k++)
            if (pos[k] < m->dev[k].n_hr && (best < 0 || m->dev[k].hrep[pos[k]] < m->dev[best].hrep[pos[best]])) best = k;
        const Dev& d = m->dev[best];
        const uint32_t r = pos[best]++;
        out->hr_height[j] = d.hh[r];
        out->hr_round[j] = d.hr[r];
        out->hr_prevotes[j] = d.hprev[r];
        out->hr_precommits[j] = d.hprec[r];
        out->hr_any[j] = d.hany[r];
        if (out->hr_rep) out->hr_rep[j] = d.hrep[r];
    }
    return HD_OK;
}

// k_dup_min: a[i] = min(a[i], b[i]) (the copy exchange's merge on device 0)
__global__ __launch_bounds__(256) void k_dup_min(uint32_t n, uint8_t* __restrict__ a, const uint8_t* __restrict__ b) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = b[i] < a[i] ? b[i] : a[i];
}

// Step 4's classification: every owner's n-byte array merged by minimum into
// device 0's, then one download into `dup`.
int merge_dup(hd_multi* m, uint32_t n, uint8_t* dup) {
    Dev& d = m->dev[0];
    const int G = (int)m->dev.size();
    if (!m->comm.empty()) {
        if (ncclGroupStart() != ncclSuccess) return HD_EDEVICE;
        for (int k = 0; k < G; k++) {
            Dev& e = m->dev[k];
            if (ncclReduce(e.dupg.p, e.dupg.p, n, ncclUint8, ncclMin, 0, m->comm[k], e.stream) != ncclSuccess) {
                (void)ncclGroupEnd();
                return HD_EDEVICE;
            }
        }
        if (ncclGroupEnd() != ncclSuccess) return HD_EDEVICE;
    } else {
        (void)hipSetDevice(d.device);
        int rc = hd_dev_grow(d.ctx, &d.dupx.p, &d.dupx.cap, n);
        if (rc) return rc;
        for (int k = 1; k < G; k++) {
            Dev& e = m->dev[k];
            MCHK(hipStreamWaitEvent(d.stream, e.owned, 0), "dup order");
            MCHK(hipMemcpyPeerAsync(d.dupx.p, d.device, e.dupg.p, e.device, n, d.stream), "dup gather");
            k_dup_min<<<(n + 255) / 256, 256, 0, d.stream>>>(n, (uint8_t*)d.dupg.p, (const uint8_t*)d.dupx.p);
            MCHK(hipGetLastError(), "k_dup_min");
        }
    }
    (void)hipSetDevice(d.device);
    MCHK(hipMemcpyAsync(dup, d.dupg.p, n, hipMemcpyDeviceToHost, d.stream), "dup download");
    MCHK(hipStreamSynchronize(d.stream), "dup download");
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
        (void)hipSetDevice(d.device);
        if (hipEventCreateWithFlags(&d.routed, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&d.owned, hipEventDisableTiming) != hipSuccess) {
            hd_multi_destroy(m);
            return HD_EDEVICE;
        }
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
    // every device's stream first: a device's buffers receive copies queued
    // on the other devices' streams (the copy exchange), so none is freed
    // before all of them have drained
    for (Dev& d : m->dev) {
        if (!d.ctx) continue;
        (void)hipSetDevice(d.device);
        (void)hipStreamSynchronize(d.stream);
    }
    for (ncclComm_t c : m->comm) (void)ncclCommDestroy(c);
    for (Dev& d : m->dev) {
        if (!d.ctx) continue;
        (void)hipSetDevice(d.device);
        for (DevBuf* b : {&d.verdict, &d.rec, &d.bitmap, &d.rows, &d.recv, &d.gidx, &d.dupg, &d.dupx})
            if (b->p) (void)hipFree(b->p);
        if (d.routed) (void)hipEventDestroy(d.routed);
        if (d.owned) (void)hipEventDestroy(d.owned);
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

}  // extern "C"

namespace {

int multi_verify(hd_multi* m, const hd_batch* batch, uint8_t* verdict, uint8_t* recovered32, uint32_t* valid_bitmap,
                 hd_tally_out* tally) {
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
    // 1: every shard uploaded to, verified on and downloaded from its device,
    // queued on the device's stream
    int rc = on_all_devices(m, [&](Dev& d, int k) {
        return verify_shard(d, batch, verdict, recovered32, valid_bitmap, &dshard[k]);
    });
    if (rc) return rc;
    if (!tally) {
        for (Dev& d : m->dev) {
            (void)hipSetDevice(d.device);
            MCHK(hipStreamSynchronize(d.stream), "output download");
        }
        return HD_OK;
    }
    // 2: candidates -> route rows grouped by owner (each device's one host
    // read: its group sizes, after its verification)
    rc = on_all_devices(m, [&](Dev& d, int k) { return route_shard(d, &dshard[k], G); });
    if (rc) return rc;
    // the groups to their owners, source-rank order (= global index order)
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
        // copies on the owner's stream, after the source's route kernel
        for (int k = 0; k < G; k++)
            for (int o = 0; o < G; o++) {
                const size_t c = m->dev[k].counts[o];
                if (!c) continue;
                Dev& d = m->dev[o];
                (void)hipSetDevice(d.device);
                MCHK(hipStreamWaitEvent(d.stream, m->dev[k].routed, 0), "route order");
                MCHK(hipMemcpyPeerAsync((char*)d.recv.p + RB * roff[o][k], d.device,
                                        (const char*)m->dev[k].rows.p + RB * soff[k][o], m->dev[k].device, RB * c,
                                        d.stream),
                     "route exchange");
            }
    }
    // 3: each owner tallies its rounds (its one host read: its table), the
    // classification scattered to global indices on the device
    const bool want_dup = tally->dup != nullptr;
    rc = on_all_devices(m, [&](Dev& d, int) {
        const int r = tally_owned(d, n, want_dup);
        if (r || !want_dup) return r;
        MCHK(hipEventRecord(d.owned, d.stream), "owner event");
        return HD_OK;
    });
    if (rc) return rc;
    // 4: classifications merged by minimum on the devices; tables on the host
    if (want_dup && (rc = merge_dup(m, n, tally->dup))) return rc;
    rc = merge_tally(m, tally);
    if (rc) return rc;
    for (Dev& d : m->dev) {   // the shards' output downloads
        (void)hipSetDevice(d.device);
        MCHK(hipStreamSynchronize(d.stream), "output download");
    }
    return HD_OK;
}

}  // namespace

extern "C" {

int hd_multi_verify_batch(hd_multi* m, const hd_batch* batch, uint8_t* verdict, uint8_t* recovered32,
                          uint32_t* valid_bitmap, hd_tally_out* tally) {
    if (!m || !batch || !verdict) return HD_EINVAL;
    const int rc = multi_verify(m, batch, verdict, recovered32, valid_bitmap, tally);
    if (rc) {
        // step 1 queues the output downloads into the caller's arrays without
        // waiting, and a later step may fail (a device error, HD_ECAP from the
        // merge): drain every device before handing the arrays back
        for (Dev& d : m->dev) {
            (void)hipSetDevice(d.device);
            (void)hipStreamSynchronize(d.stream);
        }
    }
    return rc;
}

}  // extern "C"
