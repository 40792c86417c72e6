// hd_digest.hip -- batch digest lanes (include/hd_digest.h).
//
//   k_digest<ALGO>   one message per lane: the surge preimage of message i
//                    (process/message.go:53-78, 165-186, 263-284) through
//                    SHA-256 (hd_sha256.h) or the Keccak-f[1600] sponge
//                    (hd_keccak.h), 32 B out.  VALU bound: ~2.2k (SHA-256
//                    vote) to ~5k (Keccak-f, 64-bit ops as 32-bit pairs)
//                    int32 ops per message against ~120 B of HBM traffic.
//   k_hash_bytes<PAD> one byte string per lane through the Keccak sponge;
//                    lanes are fetched as aligned dwords funnel-shifted into
//                    place, never touching a dword that starts past the end
//                    of the string.  SHA-256 strings take the compact
//                    streaming path of hd_sha256.h (k_hash_bytes_sha256).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/hd_digest.h"
#include "hd_internal.h"
#include "hd_keccak.h"
#include "hd_sha256.h"

using namespace hd;

namespace {

__device__ __forceinline__ uint32_t ld_be32(const uint8_t* p) { return load_be32(p); }

template <int ALGO>
__global__ __launch_bounds__(256) void k_digest(DevBatch b, uint8_t* __restrict__ out) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += stride) {
        const uint32_t type = b.type[i];
        uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (type >= 1 && type <= 3) {
            uint32_t v[8];
            HD_UNROLL for (int w = 0; w < 8; w++) v[w] = ld_be32(b.value32 + 32 * (size_t)i + 4 * w);
            const int64_t h = b.height[i], r = b.round[i];
            if (type == T_PROPOSE) {
                const int64_t vr = b.valid_round ? b.valid_round[i] : -1;
                if (ALGO == HD_DIGEST_SHA256) sha256_propose(d, h, r, vr, v);
                else keccak256_propose(d, h, r, vr, v, ALGO == HD_DIGEST_KECCAK256 ? 0x01 : 0x06);
            } else {
                if (ALGO == HD_DIGEST_SHA256) sha256_vote(d, h, r, v);
                else keccak256_vote(d, h, r, v, ALGO == HD_DIGEST_KECCAK256 ? 0x01 : 0x06);
            }
        }
        uint4* o = reinterpret_cast<uint4*>(out + 32 * (size_t)i);
        // digest words are big-endian: byte-swap into memory order
        o[0] = make_uint4(__builtin_bswap32(d[0]), __builtin_bswap32(d[1]), __builtin_bswap32(d[2]),
                          __builtin_bswap32(d[3]));
        o[1] = make_uint4(__builtin_bswap32(d[4]), __builtin_bswap32(d[5]), __builtin_bswap32(d[6]),
                          __builtin_bswap32(d[7]));
    }
}

// 8 bytes at p (any alignment) as a little-endian lane; dwords that start at
// or past `end` are not read (they hold no byte of the string).
struct LaneGet {
    const uint8_t* base;
    const uint8_t* end;
    __device__ __forceinline__ uint64_t operator()(uint64_t off) const {
        const uint8_t* p = base + off;
        const uintptr_t a = (uintptr_t)p;
        const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(a & 3);
        uint32_t w0 = 0, w1 = 0, w2 = 0;
        if ((const uint8_t*)q < end) w0 = q[0];
        if ((const uint8_t*)(q + 1) < end) w1 = q[1];
        if (sh && (const uint8_t*)(q + 2) < end) w2 = q[2];
        // alignbyte(hi, lo, s) = bytes s..s+3 of the 8-byte pair (lo first)
        const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
        const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
        return ((uint64_t)hi << 32) | lo;
    }
};

template <int PAD>
__global__ __launch_bounds__(256) void k_hash_bytes(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offs,
                                                    uint32_t n, uint8_t* __restrict__ out) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t s = offs[i], e = offs[i + 1];
        uint32_t d[8];
        keccak256_bytes(d, e - s, (uint8_t)PAD, LaneGet{data + s, data + e});
        uint4* o = reinterpret_cast<uint4*>(out + 32 * (size_t)i);
        o[0] = make_uint4(__builtin_bswap32(d[0]), __builtin_bswap32(d[1]), __builtin_bswap32(d[2]),
                          __builtin_bswap32(d[3]));
        o[1] = make_uint4(__builtin_bswap32(d[4]), __builtin_bswap32(d[5]), __builtin_bswap32(d[6]),
                          __builtin_bswap32(d[7]));
    }
}

// SHA-256 of one byte string per lane: 64-byte blocks assembled from aligned
// dword fetches (big-endian words), FIPS 180-4 padding with the bit length.
__global__ __launch_bounds__(256) void k_hash_bytes_sha256(const uint8_t* __restrict__ data,
                                                           const uint64_t* __restrict__ offs, uint32_t n,
                                                           uint8_t* __restrict__ out) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t s = offs[i], e = offs[i + 1];
        const uint64_t len = e - s;
        const LaneGet get{data + s, data + e};
        uint32_t st[8];
        sha256_init(st);
        // total blocks: the message, 0x80, zero fill, 8-byte length
        const uint64_t nblk = (len + 9 + 63) / 64;
        HD_NOUNROLL for (uint64_t blk = 0; blk < nblk; blk++) {
            uint32_t w[16];
            HD_UNROLL for (int k = 0; k < 8; k++) {
                const uint64_t off = 64 * blk + 8 * k;
                uint64_t lane = off < len ? get(off) : 0;
                if (off < len && len - off < 8) lane &= (1ull << (8 * (len - off))) - 1;
                if (off <= len && len - off < 8) lane |= 0x80ull << (8 * (len - off));   // the 0x80 byte
                w[2 * k] = __builtin_bswap32((uint32_t)lane);
                w[2 * k + 1] = __builtin_bswap32((uint32_t)(lane >> 32));
            }
            if (blk == nblk - 1) {
                w[14] = (uint32_t)((len * 8) >> 32);
                w[15] = (uint32_t)(len * 8);
            }
            sha256_compress(st, w);
        }
        uint4* o = reinterpret_cast<uint4*>(out + 32 * (size_t)i);
        o[0] = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]), __builtin_bswap32(st[2]),
                          __builtin_bswap32(st[3]));
        o[1] = make_uint4(__builtin_bswap32(st[4]), __builtin_bswap32(st[5]), __builtin_bswap32(st[6]),
                          __builtin_bswap32(st[7]));
    }
}

uint32_t grid_for(const hd_ctx* ctx, uint32_t n) {
    const uint32_t blocks = (n + 255) / 256;
    return std::min(blocks, (uint32_t)std::max(ctx->n_cu, 1) * 8u);
}

}  // namespace

extern "C" {

int hd_digest_batch_device(hd_ctx* ctx, int algo, const hd_batch* db, uint8_t* d_digest32, void* stream) {
    if (!ctx || !db || algo < HD_DIGEST_SHA256 || algo > HD_DIGEST_SHA3_256) return HD_EINVAL;
    if (db->n == 0) return HD_OK;
    if (!d_digest32) return HD_EINVAL;
    if (!db->type || !db->height || !db->round || !db->value32) return HD_EINVAL;
    if ((uintptr_t)d_digest32 & 15) return HD_EINVAL;   // 16-byte stores
    (void)hipSetDevice(ctx->device);
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    DevBatch b{db->n, db->type, db->height, db->round, db->valid_round, db->value32, db->from32, db->sig65};
    const uint32_t g = grid_for(ctx, db->n);
    if (algo == HD_DIGEST_SHA256) k_digest<HD_DIGEST_SHA256><<<g, 256, 0, s>>>(b, d_digest32);
    else if (algo == HD_DIGEST_KECCAK256) k_digest<HD_DIGEST_KECCAK256><<<g, 256, 0, s>>>(b, d_digest32);
    else k_digest<HD_DIGEST_SHA3_256><<<g, 256, 0, s>>>(b, d_digest32);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? HD_OK : hd_ctx_fail(ctx, e, "k_digest launch");
}

int hd_hash_bytes_device(hd_ctx* ctx, int algo, const uint8_t* d_data, const uint64_t* d_offsets, uint32_t n,
                         uint8_t* d_out32, void* stream) {
    if (!ctx || algo < HD_DIGEST_SHA256 || algo > HD_DIGEST_SHA3_256) return HD_EINVAL;
    if (n == 0) return HD_OK;
    if (!d_offsets || !d_out32) return HD_EINVAL;
    if ((uintptr_t)d_out32 & 15) return HD_EINVAL;
    (void)hipSetDevice(ctx->device);
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    const uint32_t g = grid_for(ctx, n);
    if (algo == HD_DIGEST_SHA256) k_hash_bytes_sha256<<<g, 256, 0, s>>>(d_data, d_offsets, n, d_out32);
    else if (algo == HD_DIGEST_KECCAK256) k_hash_bytes<0x01><<<g, 256, 0, s>>>(d_data, d_offsets, n, d_out32);
    else k_hash_bytes<0x06><<<g, 256, 0, s>>>(d_data, d_offsets, n, d_out32);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? HD_OK : hd_ctx_fail(ctx, e, "k_hash_bytes launch");
}

}  // extern "C"
