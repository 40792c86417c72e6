/* hd_digest.h -- batch digest lanes and verification over
 * caller-supplied digests.
 *
 * The reference digests every message with SHA-256 of its surge preimage
 * (id.NewHash = sha256.Sum256; process/message.go:53-78 Propose,
 * 165-186 Prevote, 263-284 Precommit) and that is what hd_verify_batch*
 * compute internally.  These entry points expose the digest step on its own,
 * with a choice of hash, and let the recovery run over digests produced
 * elsewhere (e.g. a Keccak-256 lane):
 *
 *   HD_DIGEST_SHA256     FIPS 180-4 SHA-256 (the reference's id.NewHash)
 *   HD_DIGEST_KECCAK256  Keccak-256, pad byte 0x01 (Ethereum's legacy Keccak;
 *                        the north star's "Keccak digesting"; the reference
 *                        itself never calls it)
 *   HD_DIGEST_SHA3_256   FIPS 202 SHA3-256, pad byte 0x06
 *
 * Device pointers, stream-ordered, no synchronisation, like
 * hd_verify_batch_device. */
#ifndef HD_DIGEST_H
#define HD_DIGEST_H

#include <stdint.h>

#include "hd_verify.h"

#ifdef __cplusplus
extern "C" {
#endif

#define HD_DIGEST_SHA256 0
#define HD_DIGEST_KECCAK256 1
#define HD_DIGEST_SHA3_256 2

/* d_digest32[i] = algo(surge preimage of message i): BE64(h) || BE64(r) ||
 * value for Prevote/Precommit (48 B), BE64(h) || BE64(r) || BE64(vr) || value
 * for Propose (56 B; valid_round NULL = -1).  Messages of any other type get
 * 32 zero bytes.  from32 and sig65 of the batch are not read (may be NULL). */
int hd_digest_batch_device(hd_ctx* ctx, int algo, const hd_batch* d_batch, uint8_t* d_digest32, void* stream);

/* d_out32[i] = algo(d_data[d_offsets[i] .. d_offsets[i+1])) for i < n: n
 * byte strings of any length (0 included) packed back to back; d_offsets
 * holds n+1 non-decreasing byte offsets. */
int hd_hash_bytes_device(hd_ctx* ctx, int algo, const uint8_t* d_data, const uint64_t* d_offsets, uint32_t n,
                         uint8_t* d_out32, void* stream);

/* hd_verify_batch_device with message i's digest read from d_digest32[i]
 * instead of computed: recovery (libsecp256k1 semantics), signatory,
 * Equal(From) and the admitted check are unchanged.  type must still be
 * 1..3 (else BAD_TYPE); height/round/valid_round/value32 are not read (may
 * be NULL). */
int hd_verify_batch_digest_device(hd_ctx* ctx, const hd_batch* d_batch, const uint8_t* d_digest32,
                                  uint8_t* d_verdict, uint8_t* d_recovered32, int32_t* d_signer,
                                  uint32_t* d_valid_bitmap, void* stream);

#ifdef __cplusplus
}
#endif
#endif
