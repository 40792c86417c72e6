// hd_codec.hip -- batch surge codec of Propose / Prevote / Precommit records
// (include/hd_codec.h; process/message.go:102-149, 208-247, 306-345).
//
// HBM-bound byte shuffling: a record is 80 / 88 bytes (+65 signature bytes),
// an odd stride, so a workgroup moves its 128 (decode) / 256 (encode) records between HBM and LDS
// with aligned 16-byte vector accesses and the lanes (de)serialise their own
// record in LDS.  Field arrays on the SoA side are written / read with
// per-lane-contiguous stores and loads.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/hd_codec.h"
#include "hd_internal.h"

using namespace hd;

#define HD_CODEC_BLOCK 256
#define HD_CODEC_MAXREC (88 + 65)

// 4 bytes at any byte offset of an LDS buffer: two aligned dword reads and a
// byte-align (the record stride is odd, so lanes sit at every alignment)
__device__ __forceinline__ uint32_t lds_word(const uint8_t* base, uint32_t off) {
    const uint32_t a = off & ~3u, sh = off & 3u;
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(base + a);
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(base + a + 4);
    return sh ? __builtin_amdgcn_alignbyte(w1, w0, sh) : w0;
}
__device__ __forceinline__ uint64_t lds_be64(const uint8_t* base, uint32_t off) {
    return ((uint64_t)__builtin_bswap32(lds_word(base, off)) << 32) | __builtin_bswap32(lds_word(base, off + 4));
}
__device__ __forceinline__ void st_be64(uint8_t* p, uint64_t v) {
    HD_UNROLL for (int k = 7; k >= 0; k--) {
        p[k] = (uint8_t)v;
        v >>= 8;
    }
}

// decode: 128 records per workgroup (20 KB of LDS -> 8 workgroups per CU)
#define HD_DEC_BLOCK 128
template <bool PROPOSE, bool SIG>
__global__ __launch_bounds__(HD_DEC_BLOCK) void k_unmarshal(const uint8_t* __restrict__ buf, uint64_t len, uint32_t n,
                                                            uint8_t type, hd_batch_out out,
                                                            uint8_t* __restrict__ status) {
    constexpr uint32_t S = (PROPOSE ? 88u : 80u) + (SIG ? 65u : 0u);
    __shared__ uint4 lds[(HD_DEC_BLOCK * HD_CODEC_MAXREC + 48) / 16];
    const uint32_t rec0 = blockIdx.x * HD_DEC_BLOCK;
    const uint32_t nrec = min((uint32_t)HD_DEC_BLOCK, n - rec0);
    const uint64_t byte0 = (uint64_t)rec0 * S;
    const uint64_t want = byte0 + (uint64_t)nrec * S;
    const uint64_t byte1 = want < len ? want : len;  // bytes that exist
    const uint64_t a0 = byte0 & ~15ull;
    // HBM -> LDS, 16 bytes per lane per step (the last partial word bytewise)
    for (uint64_t w = threadIdx.x; byte1 > a0 && a0 + 16 * w < byte1; w += HD_DEC_BLOCK) {
        const uint64_t addr = a0 + 16 * w;
        if (addr + 16 <= len) {
            lds[w] = *reinterpret_cast<const uint4*>(buf + addr);
        } else {
            uint8_t* d = reinterpret_cast<uint8_t*>(&lds[w]);
            for (int k = 0; k < 16; k++) d[k] = addr + k < len ? buf[addr + k] : 0;
        }
    }
    __syncthreads();
    const uint32_t t = threadIdx.x;
    if (SIG && out.sig65) {
        // The block's signatures form one contiguous 65 * nrec byte range of
        // sig65 starting at s0 = 65 * rec0, a multiple of 16 (rec0 is a
        // multiple of 128).  Each lane builds whole 16-byte output words from
        // LDS dwords: an output dword lies inside one signature, or straddles
        // two (the last 1..3 bytes of one and the first of the next) and is
        // merged from two reads.  Only a partial last word goes bytewise.
        const uint64_t s0 = 65ull * rec0;
        const uint32_t sbytes = 65u * nrec;
        const uint8_t* Lb = reinterpret_cast<const uint8_t*>(lds);
        const uint32_t base = (uint32_t)(byte0 - a0) + (S - 65u);   // LDS offset of signature 0
        auto sig_ok = [&](uint32_t r) { return byte0 + (uint64_t)(r + 1) * S <= len; };
        auto out_dword = [&](uint32_t rel) -> uint32_t {   // bytes [rel, rel + 4) of the signature stream
            const uint32_t r = rel / 65u, kb = rel - 65u * r;
            const uint32_t src = base + r * S + kb;
            const uint32_t lo = sig_ok(r) ? lds_word(Lb, src) : 0u;
            if (kb <= 61u) return lo;
            const uint32_t nlo = 65u - kb;   // 1..3 bytes of signature r, the rest from r + 1
            const uint32_t m = (1u << (8u * nlo)) - 1u;
            const uint32_t hi = (r + 1 < nrec && sig_ok(r + 1)) ? lds_word(Lb, base + (r + 1) * S - nlo) : 0u;
            return (lo & m) | (hi & ~m);
        };
        for (uint32_t w = t; 16 * w < sbytes; w += HD_DEC_BLOCK) {
            const uint32_t rel = 16 * w;
            const uint4 v = make_uint4(out_dword(rel), rel + 4 < sbytes ? out_dword(rel + 4) : 0u,
                                       rel + 8 < sbytes ? out_dword(rel + 8) : 0u,
                                       rel + 12 < sbytes ? out_dword(rel + 12) : 0u);
            uint8_t* dst = out.sig65 + s0 + rel;
            if (rel + 16 <= sbytes) {
                *reinterpret_cast<uint4*>(dst) = v;
            } else {
                const uint8_t* b = reinterpret_cast<const uint8_t*>(&v);
                for (uint32_t k = 0; rel + k < sbytes; k++) dst[k] = b[k];
            }
        }
    }
    if (t >= nrec) return;
    const uint32_t i = rec0 + t;
    const uint64_t rs = byte0 + (uint64_t)t * S;
    const bool ok = rs + S <= len;
    const uint8_t* Lb = reinterpret_cast<const uint8_t*>(lds);
    const uint32_t L0 = (uint32_t)(rs - a0);
    status[i] = ok ? 0 : 1;
    out.type[i] = type;
    uint32_t off = L0;
    out.height[i] = ok ? (int64_t)lds_be64(Lb, off) : 0;
    off += 8;
    out.round[i] = ok ? (int64_t)lds_be64(Lb, off) : 0;
    off += 8;
    if (PROPOSE) {
        out.valid_round[i] = ok ? (int64_t)lds_be64(Lb, off) : 0;
        off += 8;
    } else if (out.valid_round) {
        out.valid_round[i] = -1;
    }
    // value, from: 32 bytes each -> two 16-byte stores per field
    HD_UNROLL for (int f = 0; f < 2; f++) {
        uint32_t w[8];
        HD_UNROLL for (int k = 0; k < 8; k++) w[k] = ok ? lds_word(Lb, off + 4 * k) : 0u;
        uint4* dst = reinterpret_cast<uint4*>((f == 0 ? out.value32 : out.from32) + 32 * (size_t)i);
        dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
        dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
        off += 32;
    }
}

template <bool PROPOSE, bool SIG>
__global__ __launch_bounds__(HD_CODEC_BLOCK) void k_marshal(hd_batch in, uint32_t n, uint8_t* __restrict__ buf) {
    constexpr uint32_t S = (PROPOSE ? 88u : 80u) + (SIG ? 65u : 0u);
    __shared__ uint4 lds[(HD_CODEC_BLOCK * HD_CODEC_MAXREC + 32) / 16];
    const uint32_t rec0 = blockIdx.x * HD_CODEC_BLOCK;
    const uint32_t nrec = min((uint32_t)HD_CODEC_BLOCK, n - rec0);
    const uint64_t byte0 = (uint64_t)rec0 * S;
    const uint64_t byte1 = byte0 + (uint64_t)nrec * S;
    const uint64_t a0 = byte0 & ~15ull;
    uint8_t* Lb = reinterpret_cast<uint8_t*>(lds);
    const uint32_t t = threadIdx.x;
    if (t < nrec) {
        const uint32_t i = rec0 + t;
        uint8_t* L = Lb + (byte0 - a0) + (uint64_t)t * S;
        uint32_t off = 0;
        st_be64(L + off, (uint64_t)in.height[i]);
        off += 8;
        st_be64(L + off, (uint64_t)in.round[i]);
        off += 8;
        if (PROPOSE) {
            st_be64(L + off, (uint64_t)(in.valid_round ? in.valid_round[i] : -1));
            off += 8;
        }
        HD_UNROLL for (int f = 0; f < 2; f++) {
            const uint4* src = reinterpret_cast<const uint4*>((f == 0 ? in.value32 : in.from32) + 32 * (size_t)i);
            const uint4 u0 = src[0], u1 = src[1];
            const uint32_t w[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
            HD_UNROLL for (int k = 0; k < 8; k++) {
                L[off + 4 * k] = (uint8_t)w[k];
                L[off + 4 * k + 1] = (uint8_t)(w[k] >> 8);
                L[off + 4 * k + 2] = (uint8_t)(w[k] >> 16);
                L[off + 4 * k + 3] = (uint8_t)(w[k] >> 24);
            }
            off += 32;
        }
        if (SIG) {
            const uint8_t* s = in.sig65 + 65 * (size_t)i;
            for (int k = 0; k < 65; k++) L[off + k] = s[k];
        }
    }
    __syncthreads();
    // LDS -> HBM: whole 16-byte words inside [byte0, byte1) as vectors; the
    // two partial boundary words (shared with the neighbouring workgroups)
    // byte by byte, so no byte outside this block's records is written.
    for (uint64_t w = t; a0 + 16 * w < byte1; w += HD_CODEC_BLOCK) {
        const uint64_t addr = a0 + 16 * w;
        if (addr >= byte0 && addr + 16 <= byte1) {
            *reinterpret_cast<uint4*>(buf + addr) = lds[w];
        } else {
            const uint8_t* s = reinterpret_cast<const uint8_t*>(&lds[w]);
            for (int k = 0; k < 16; k++)
                if (addr + k >= byte0 && addr + k < byte1) buf[addr + k] = s[k];
        }
    }
}

extern "C" {

uint32_t hd_record_size(int type, int with_sig) {
    if (type < 1 || type > 3) return 0;
    return (type == T_PROPOSE ? 88u : 80u) + (with_sig ? 65u : 0u);
}

int hd_unmarshal_batch_device(hd_ctx* ctx, int type, int with_sig, const uint8_t* d_buf, uint64_t len, uint32_t n,
                              const hd_batch_out* d_out, uint8_t* d_status, void* stream) {
    if (!ctx || hd_record_size(type, with_sig) == 0) return HD_EINVAL;
    if (n == 0) return HD_OK;
    if (!d_out) return HD_EINVAL;
    if (!d_buf || !d_status || !d_out->type || !d_out->height || !d_out->round || !d_out->value32 || !d_out->from32)
        return HD_EINVAL;
    if (type == T_PROPOSE && !d_out->valid_round) return HD_EINVAL;
    if (with_sig && !d_out->sig65) return HD_EINVAL;
    // k_unmarshal writes 16-byte words into value32, from32 and a block's
    // contiguous sig65 range
    if (((uintptr_t)d_buf & 15) || ((uintptr_t)d_out->value32 & 15) || ((uintptr_t)d_out->from32 & 15) ||
        (with_sig && ((uintptr_t)d_out->sig65 & 15)))
        return HD_EINVAL;
    (void)hipSetDevice(ctx->device);
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    const uint32_t blocks = (n + HD_DEC_BLOCK - 1) / HD_DEC_BLOCK;
    const uint8_t t = (uint8_t)type;
    if (type == T_PROPOSE) {
        if (with_sig) k_unmarshal<true, true><<<blocks, HD_DEC_BLOCK, 0, s>>>(d_buf, len, n, t, *d_out, d_status);
        else k_unmarshal<true, false><<<blocks, HD_DEC_BLOCK, 0, s>>>(d_buf, len, n, t, *d_out, d_status);
    } else {
        if (with_sig) k_unmarshal<false, true><<<blocks, HD_DEC_BLOCK, 0, s>>>(d_buf, len, n, t, *d_out, d_status);
        else k_unmarshal<false, false><<<blocks, HD_DEC_BLOCK, 0, s>>>(d_buf, len, n, t, *d_out, d_status);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? HD_OK : hd_ctx_fail(ctx, e, "k_unmarshal");
}

int hd_marshal_batch_device(hd_ctx* ctx, int type, int with_sig, const hd_batch* d_in, uint8_t* d_buf, uint64_t cap,
                            void* stream) {
    const uint32_t S = hd_record_size(type, with_sig);
    if (!ctx || !d_in || S == 0) return HD_EINVAL;
    const uint32_t n = d_in->n;
    if (n == 0) return HD_OK;
    if (!d_buf || !d_in->height || !d_in->round || !d_in->value32 || !d_in->from32) return HD_EINVAL;
    if (with_sig && !d_in->sig65) return HD_EINVAL;
    if (((uintptr_t)d_buf & 15) || ((uintptr_t)d_in->value32 & 15) || ((uintptr_t)d_in->from32 & 15))
        return HD_EINVAL;
    if (cap < (uint64_t)n * S) return HD_ECAP;
    (void)hipSetDevice(ctx->device);
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    const uint32_t blocks = (n + HD_CODEC_BLOCK - 1) / HD_CODEC_BLOCK;
    if (type == T_PROPOSE) {
        if (with_sig) k_marshal<true, true><<<blocks, HD_CODEC_BLOCK, 0, s>>>(*d_in, n, d_buf);
        else k_marshal<true, false><<<blocks, HD_CODEC_BLOCK, 0, s>>>(*d_in, n, d_buf);
    } else {
        if (with_sig) k_marshal<false, true><<<blocks, HD_CODEC_BLOCK, 0, s>>>(*d_in, n, d_buf);
        else k_marshal<false, false><<<blocks, HD_CODEC_BLOCK, 0, s>>>(*d_in, n, d_buf);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? HD_OK : hd_ctx_fail(ctx, e, "k_marshal");
}

}  // extern "C"
