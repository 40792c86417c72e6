// hd_internal.h -- host-side context shared by the .hip translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <utility>
#include <vector>

#include "../../include/hd_verify.h"
#include "hd_fixedbase.h"
#include "hd_verify_msg.h"

struct DevBatch {
    uint32_t n;
    const uint8_t* type;
    const int64_t* height;
    const int64_t* round;
    const int64_t* valid_round;
    const uint8_t* value32;
    const uint8_t* from32;
    const uint8_t* sig65;
};

enum BufSlot {
    BUF_TYPE, BUF_HEIGHT, BUF_ROUND, BUF_VROUND, BUF_VALUE, BUF_FROM, BUF_SIG,
    BUF_VERDICT, BUF_REC, BUF_SIGNER, BUF_BITMAP, BUF_DUP, BUF__COUNT
};

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

struct TallyWork;  // hd_tally.hip
struct HostPipe;   // hd_host.hip: hd_verify_submit pipelines
struct FbWork;     // hd_fastverify.hip: known-key tables and fast-path scratch

struct hd_ctx {
    int device = 0;
    int n_cu = 256;
    int verify_waves = 3;   // register budget of k_verify (waves per SIMD)
    int var[HD_VAR__COUNT] = {3, 0, 1, 0, -1, 0, 2, 0, 0, 0, 16, 1, 0, 0, 0};   // hd_ctx_set_variant (var[0] mirrors verify_waves)
    hipStream_t stream = nullptr;
    int pkfmt = HD_PUBKEY_COMPRESSED;   // id.NewSignatory's pubkey encoding (hd_ctx_set_pubkey_format)
    hd::ge* d_gtab = nullptr;
    uint32_t* d_adm = nullptr;      // sorted admitted signatories, 8 BE words each
    int32_t* d_adm_perm = nullptr;  // sorted index -> caller's index
    size_t cap_adm = 0, cap_adm_perm = 0;
    uint32_t n_adm = 0;
    uint32_t adm_ver = 0;           // bumped by every hd_set_signatories (hd_mq's prefetch checks it)
    // the hd_set_signatories array as given (caller order, duplicates kept):
    // the From rows of the compact host batch (hd_verify_submit_compact)
    uint8_t* d_sig_caller = nullptr;
    size_t cap_sig_caller = 0;
    uint32_t n_sig_caller = 0;
    int adm_steps = 0;
    // hashed index of d_adm (hd_verify_msg.h AdmIndex): adm_ix_mask + 1 slots
    uint32_t* d_adm_ix = nullptr;
    size_t cap_adm_ix = 0;
    uint32_t adm_ix_mask = 0;
    DevBuf bufs[BUF__COUNT];
    TallyWork* tally = nullptr;
    FbWork* fb = nullptr;
    bool fastpath = true;   // known-key fast path (HD_VERIFY_FASTPATH=0 disables)
    hipEvent_t ev_slow = nullptr;   // after the last full-recovery-only verify call (fast path off)
    HostPipe* host = nullptr;
    // caller streams that ran work reading this context's scratch or tables
    // (route, unroute, async tallies, the generator), each with an event
    // recorded after its last such work: hd_ctx_destroy waits for these
    // instead of for the whole device
    std::vector<std::pair<hipStream_t, hipEvent_t>> caller_ev;
    std::string last_error;
};

// Record (after work just queued on s) that s uses this context; a no-op for
// the context's own stream, which destroy synchronises anyway.
int hd_ctx_note_stream(hd_ctx* ctx, hipStream_t s);

// Wait (host) for every kernel this context queued: its own stream and the
// verify calls on caller streams.  Replaces device-wide synchronisation, so a
// set change does not stall other contexts or streams of the device.
int hd_ctx_quiesce(hd_ctx* ctx);
int hd_fb_quiesce(hd_ctx* ctx);   // the known-key path's calls (hd_fastverify.hip)

int hd_ctx_fail(hd_ctx* ctx, hipError_t e, const char* what);
int hd_dev_grow(hd_ctx* ctx, void** p, size_t* cap, size_t need);
// the admitted table's hashed index (valid lookups need ctx->n_adm > 0)
inline hd::AdmIndex hd_adm_index(const hd_ctx* ctx) { return hd::AdmIndex{ctx->d_adm, ctx->d_adm_ix, ctx->adm_ix_mask}; }
int hd_upload_batch(hd_ctx* ctx, const hd_batch* hb, hd_batch* db);
int hd_verify_uploaded(hd_ctx* ctx, const hd_batch* db, uint8_t* verdict, uint8_t* recovered32, uint32_t* valid_bitmap);
void hd_tally_release(hd_ctx* ctx);
// hd_tally_routed_device with the per-row classification scattered on the
// device to dup_global[global index] (hd_multi's owners; hd_tally.hip)
int hd_tally_routed_dup_device(hd_ctx* ctx, const hd_batch* dbatch, const uint32_t* d_gidx, hd_tally_out* out,
                               uint8_t* dup_global, hipStream_t s);
void hd_host_release(hd_ctx* ctx);

// known-key fast path (hd_fastverify.hip)
int hd_fb_init(hd_ctx* ctx);                    // tables of G (slot 0); at context creation
void hd_fb_release(hd_ctx* ctx);
const hd::gp* hd_fb_gtab(const hd_ctx* ctx);    // the shared fixed-base G table (NULL: none)
int hd_fb_map_signatories(hd_ctx* ctx, const uint8_t* sorted_sigs32, uint32_t m);  // after hd_set_signatories
int hd_fb_clear_keys(hd_ctx* ctx);               // pubkey format changed: learned keys no longer apply
// fast kernel + slow recovery of the rest + learning; the whole verify of a device batch
// (auth: hd_authenticate_batch_device -- a failed known-key check is final, NOT_AUTHENTIC)
int hd_fb_verify(hd_ctx* ctx, const DevBatch& b, const uint8_t* d_digest, uint8_t* d_verdict, uint8_t* d_rec32,
                 int32_t* d_signer, uint32_t* d_bitmap, hipStream_t s, bool auth = false);

// slow-path control for k_verify (hd_verify.hip): an index list and key learning
struct SlowCtl {
    const uint32_t* list;   // message indices to verify, or NULL for all
    const uint32_t* count;  // device count of list
    const int32_t* adm_slot;  // admitted sorted index -> table slot (-1 none), NULL: no learning
    uint32_t* fb_state;
    hd::ge* fb_pub;
    uint32_t* bitmap_or;      // list mode: set the valid bit of each VALID message (the rest already written)
    uint32_t* est_out;        // list mode: the list length is stored here (host-mapped; sizes later grids)
    int prio;                 // wave issue priority (s_setprio 0..3; HD_VAR_WAVE_PRIO) of the list mode
    // foreign keys (HD_VAR_FOREIGN_KEYS): a NOT_ADMITTED recovery publishes
    // its key into one of the fcap reserved slots fbase .. (fdict: hd_fixedbase.h)
    uint32_t* fdict;
    uint32_t* fnext;
    uint32_t fbase, fcap;
    uint32_t* fpend;          // host-mapped: the claim count, so the host builds the new tables
    // slot eviction (hd_fastverify.hip fb_evict): a From the dictionary holds
    // without a slot keeps its key in fkey[bucket] and counts its recoveries
    // in fbhit[bucket]; fmiss (host-mapped) is set on every such recovery
    uint32_t* fbhit;
    hd::ge* fkey;
    uint32_t* fmiss;
};
int hd_launch_slow(hd_ctx* ctx, const DevBatch& b, const uint8_t* d_digest, uint8_t* d_verdict, uint8_t* d_rec32,
                   int32_t* d_signer, uint32_t* d_bitmap, const SlowCtl& ctl, uint32_t blocks, hipStream_t s);
