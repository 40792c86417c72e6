// hd_internal.h -- host-side context shared by the .hip translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/hd_verify.h"
#include "hd_group.h"

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

struct hd_ctx {
    int device = 0;
    int n_cu = 256;
    int verify_waves = 3;   // register budget of k_verify (waves per SIMD)
    hipStream_t stream = nullptr;
    bool compressed = true;
    hd::ge* d_gtab = nullptr;
    uint32_t* d_adm = nullptr;      // sorted admitted signatories, 8 BE words each
    int32_t* d_adm_perm = nullptr;  // sorted index -> caller's index
    size_t cap_adm = 0, cap_adm_perm = 0;
    uint32_t n_adm = 0;
    int adm_steps = 0;
    DevBuf bufs[BUF__COUNT];
    TallyWork* tally = nullptr;
    std::string last_error;
};

int hd_ctx_fail(hd_ctx* ctx, hipError_t e, const char* what);
int hd_dev_grow(hd_ctx* ctx, void** p, size_t* cap, size_t need);
int hd_upload_batch(hd_ctx* ctx, const hd_batch* hb, hd_batch* db);
int hd_verify_uploaded(hd_ctx* ctx, const hd_batch* db, uint8_t* verdict, uint8_t* recovered32, uint32_t* valid_bitmap);
void hd_tally_release(hd_ctx* ctx);
