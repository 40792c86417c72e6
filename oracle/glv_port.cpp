// glv_port.cpp -- CPU BASELINE ONLY (bench.py's cpu_baseline leg; tests).
// Not the oracle and not a product path: the repository's own recovery
// (hyperdrive_amd/csrc/hd_verify_msg.h -> hd_group.h: GLV split, 12-bit
// windows over precomputed affine tables of G and lambda G, Booth-windowed
// 4-scalar ladder, divstep inversions) compiled for the host, run over a
// batch on host threads.  This is the libsecp256k1 shape of the reference's
// CPU path (the reference recovers through go-ethereum's cgo libsecp256k1:
// /root/reference/process/message_test.go:152), so it is
// a fairer CPU rate than the naive 4x64-limb restatement (hd_oracle.c).
// Semantics are verify_msg's: digest -> recover -> signatory -> Equal(From)
// -> admitted (process/message.go:53-78, 165-186, 263-284; mq/mq.go:49-51).
#include <algorithm>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../hyperdrive_amd/csrc/hd_verify_msg.h"

using namespace hd;

namespace {
const ge* glv_tables() {
    static std::vector<ge> tab;
    static std::once_flag once;
    std::call_once(once, [] {
        tab.resize(2 * HD_GLV_GTAB_N);
        build_gtab_glv(tab.data());
    });
    return tab.data();
}
}  // namespace

extern "C" {
// verdict / rec32 / signer per message, as hd_verify_batch; adm32 any order
// (sorted here, duplicates dropped: signer = the first caller index)
int glv_verify(uint32_t n, const uint8_t* type, const int64_t* h, const int64_t* r, const int64_t* vr,
               const uint8_t* value32, const uint8_t* from32, const uint8_t* sig65, const uint8_t* adm32,
               uint32_t n_adm, int compressed, uint8_t* verdict, uint8_t* rec32, int32_t* signer, int threads) {
    const ge* gt = glv_tables();
    std::vector<uint32_t> order(n_adm);
    for (uint32_t i = 0; i < n_adm; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return memcmp(adm32 + 32 * (size_t)a, adm32 + 32 * (size_t)b, 32) < 0;
    });
    std::vector<uint32_t> aw;
    std::vector<int32_t> perm;
    for (uint32_t k = 0; k < n_adm; k++) {
        const uint8_t* s = adm32 + 32 * (size_t)order[k];
        if (!perm.empty() && memcmp(s, adm32 + 32 * (size_t)perm.back(), 32) == 0) continue;
        for (int w = 0; w < 8; w++) aw.push_back(load_be32(s + 4 * w));
        perm.push_back((int32_t)order[k]);
    }
    const uint32_t m = (uint32_t)perm.size();
    int steps = 0;
    while ((1u << steps) < m) steps++;
    threads = std::max(1, threads);
    auto work = [&](uint32_t lo, uint32_t hi) {
        for (uint32_t i = lo; i < hi; i++) {
            MsgIn msg;
            msg.type = type[i];
            msg.h = h[i];
            msg.r = r[i];
            msg.vr = vr ? vr[i] : -1;
            for (int w = 0; w < 8; w++) {
                msg.value_be[w] = load_be32(value32 + 32 * (size_t)i + 4 * w);
                msg.from_be[w] = load_be32(from32 + 32 * (size_t)i + 4 * w);
                msg.r_be[w] = load_be32(sig65 + 65 * (size_t)i + 4 * w);
                msg.s_be[w] = load_be32(sig65 + 65 * (size_t)i + 32 + 4 * w);
            }
            msg.v = sig65[65 * (size_t)i + 64];
            uint32_t rec[8];
            int32_t s;
            verdict[i] = verify_msg(msg, gt, aw.data(), m, steps, compressed, rec, s);
            if (signer) signer[i] = s >= 0 ? perm[s] : -1;
            if (rec32)
                for (int w = 0; w < 8; w++) store_be32(rec32 + 32 * (size_t)i + 4 * w, rec[w]);
        }
    };
    std::vector<std::thread> th;
    const uint32_t per = (n + (uint32_t)threads - 1) / (uint32_t)threads;
    for (int t = 0; t < threads; t++) {
        const uint32_t lo = std::min(n, (uint32_t)t * per), hi = std::min(n, lo + per);
        if (lo < hi) th.emplace_back(work, lo, hi);
    }
    for (auto& x : th) x.join();
    return 0;
}
}
