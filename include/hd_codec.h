/* hd_codec.h -- batch surge codec of hyperdrive's messages on the GPU.
 *
 * Restates process/message.go Marshal / Unmarshal for arrays of messages:
 *   Propose   (message.go:102-149)  Height ‖ Round ‖ ValidRound ‖ Value ‖ From = 88 B
 *   Prevote   (message.go:208-247)  Height ‖ Round ‖ Value ‖ From              = 80 B
 *   Precommit (message.go:306-345)  Height ‖ Round ‖ Value ‖ From              = 80 B
 * surge v1.2.5 writes int64 as 8 big-endian bytes and [32]byte raw, with no
 * length prefixes or type tags.  With with_sig != 0 each record is followed by
 * its 65-byte id.Signature (R ‖ S ‖ V): the surge encoding of the
 * {message, signature} pair that INTEGRATION.md's verify.Signed carries.
 *
 * A wire buffer holds n records of ONE message type back to back (record i at
 * byte i * hd_record_size(type, with_sig)).  All pointers are device memory of
 * the ctx's device; buffers must be 16-byte aligned.  Calls are enqueued on
 * `stream` (a hipStream_t, NULL = the ctx's stream) and are asynchronous. */
#ifndef HD_CODEC_H
#define HD_CODEC_H

#include <stdint.h>

#include "hd_verify.h"

#ifdef __cplusplus
extern "C" {
#endif

/* bytes per record; 0 for a type other than 1 (Propose), 2 (Prevote), 3 (Precommit) */
uint32_t hd_record_size(int type, int with_sig);

/* Decode n records from d_buf[0, len) into the SoA fields of *d_out (type[]
 * := type; valid_round[] := ValidRound for proposes, -1 for votes, and may be
 * NULL for votes; sig65 may be NULL when with_sig == 0).  d_status[i] := 0 for
 * a decoded record, 1 when the buffer ends before record i is complete (the
 * "unmarshaling ...: unexpected end of buffer" error of message.go); such
 * records' fields are zeroed.  HD_EINVAL for a bad type, NULL or unaligned
 * pointers. */
int hd_unmarshal_batch_device(hd_ctx* ctx, int type, int with_sig, const uint8_t* d_buf, uint64_t len, uint32_t n,
                              const hd_batch_out* d_out, uint8_t* d_status, void* stream);

/* Encode the first n messages of *d_in as records into d_buf (capacity cap
 * bytes).  HD_ECAP if cap < n * hd_record_size(type, with_sig). */
int hd_marshal_batch_device(hd_ctx* ctx, int type, int with_sig, const hd_batch* d_in, uint8_t* d_buf, uint64_t cap,
                            void* stream);

#ifdef __cplusplus
}
#endif
#endif
