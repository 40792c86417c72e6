// hd_genk.hip -- kernels + C ABI of the seeded synthetic workload
// (input construction for benchmarks and tests; see hd_gen.h).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/hd_verify.h"
#include "hd_gen.h"
#include "hd_internal.h"

using namespace hd;

struct BeWords {  // 32-byte strings addressed as big-endian words
    const uint8_t* p;
    __device__ __forceinline__ uint32_t operator[](size_t k) const { return load_be32(p + 4 * k); }
};

__global__ __launch_bounds__(256) void k_keys(uint32_t S, int pkfmt, const ge* __restrict__ gtab,
                                              uint8_t* sigs32, uint8_t* foreign32) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= S + HD_NONADMITTED_KEYS) return;
    uint32_t idx = j < S ? j : HD_NONADMITTED_BASE + (j - S);
    sc sk;
    signer_sk(sk, idx);
    uint32_t o[8];
    pubkey_signatory(o, sk, pkfmt, gtab);
    uint8_t* dst = j < S ? sigs32 + 32 * (size_t)j : foreign32 + 32 * (size_t)(j - S);
    for (int w = 0; w < 8; w++) store_be32(dst + 4 * w, o[w]);
}

__global__ __launch_bounds__(256) void k_gen(uint32_t kind, uint64_t start, uint32_t n, uint32_t S, uint32_t adv_pct,
                                             const ge* __restrict__ gtab_g, const uint8_t* __restrict__ sigs32,
                                             const uint8_t* __restrict__ foreign32, hd_batch_out out) {
    __shared__ ge s_gtab[HD_GTAB_N];
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(gtab_g);
        uint32_t* dst = reinterpret_cast<uint32_t*>(s_gtab);
        for (int k = threadIdx.x; k < (int)(HD_GTAB_N * sizeof(ge) / 4); k += blockDim.x) dst[k] = src[k];
    }
    __syncthreads();
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        BeWords sw{sigs32}, fw{foreign32};
        int cls = gen_message(kind, start + k, S, adv_pct, (const ge*)s_gtab, sw, fw, out.type[k], out.height[k],
                              out.round[k], out.valid_round[k], out.value32 + 32 * (size_t)k,
                              out.from32 + 32 * (size_t)k, out.sig65 + 65 * (size_t)k);
        if (out.adv_class) out.adv_class[k] = (int8_t)cls;
    }
}

extern "C" {

int hd_gen_keys(hd_ctx* ctx, uint32_t S, uint8_t* signatories32, uint8_t* foreign32) {
    if (!ctx || !signatories32 || !foreign32) return HD_EINVAL;
    (void)hipSetDevice(ctx->device);
    uint8_t* d = nullptr;
    size_t bytes = 32 * (size_t)(S + HD_NONADMITTED_KEYS);
    hipError_t e = hipMalloc(&d, bytes);
    if (e != hipSuccess) return hd_ctx_fail(ctx, e, "gen_keys alloc");
    uint32_t total = S + HD_NONADMITTED_KEYS;
    k_keys<<<(total + 255) / 256, 256, 0, ctx->stream>>>(S, ctx->pkfmt, ctx->d_gtab, d, d + 32 * (size_t)S);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(signatories32, d, 32 * (size_t)S, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(foreign32, d + 32 * (size_t)S, 32 * HD_NONADMITTED_KEYS, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return hd_ctx_fail(ctx, e, "gen_keys");
    return HD_OK;
}

int hd_gen_batch_device(hd_ctx* ctx, uint32_t kind, uint64_t start, uint32_t n, uint32_t S, uint32_t adv_pct,
                        const uint8_t* d_signatories32, const uint8_t* d_foreign32, const hd_batch_out* d_out,
                        void* stream) {
    if (!ctx || !d_out || !d_signatories32 || !d_foreign32 || S == 0 || kind > 1 || adv_pct > 100) return HD_EINVAL;
    if (!d_out->type || !d_out->height || !d_out->round || !d_out->valid_round || !d_out->value32 ||
        !d_out->from32 || !d_out->sig65)
        return HD_EINVAL;
    if (n == 0) return HD_OK;
    (void)hipSetDevice(ctx->device);
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    uint32_t blocks = std::min((n + 255) / 256, (uint32_t)std::max(ctx->n_cu, 1) * 8u);
    k_gen<<<blocks, 256, 0, s>>>(kind, start, n, S, adv_pct, ctx->d_gtab, d_signatories32, d_foreign32, *d_out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hd_ctx_fail(ctx, e, "k_gen launch");
    return hd_ctx_note_stream(ctx, s);   // k_gen reads the context's G table
}

}  // extern "C"
