/* hd_mq.h -- bulk MessageQueue on the GPU (mq/mq.go), SURVEY §8(f)3.
 *
 * Per-sender queues ordered by (height, round), stable for equal keys
 * (mq.go:116-135), at most max_capacity messages per sender: inserting into a
 * full queue drops its largest element (mq.go:137-142).  A batch insert has
 * the effect of inserting the batch's messages one at a time in batch
 * (= arrival) order: every sender keeps the max_capacity smallest of its old
 * and new messages under (height, round, arrival).
 *
 * Senders are int32 indices (e.g. the signer index hd_verify_batch_device
 * writes for VALID messages).  Messages with a negative sender are not
 * inserted: in the reference they could only be dropped by the procsAllowed
 * filter of Consume (mq.go:49-51).  Messages are copied into device memory
 * owned by the queue.  Like mq.MessageQueue, an hd_mq is not safe for
 * concurrent use. */
#ifndef HD_MQ_H
#define HD_MQ_H

#include <stdint.h>

#include "hd_verify.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hd_mq hd_mq;

/* mq.New(Options{MaxCapacity: max_capacity}) (mq.go:25-30, opt.go:19 default 1000) */
int hd_mq_create(hd_ctx* ctx, uint32_t max_capacity, hd_mq** out);
int hd_mq_destroy(hd_mq* q);

/* InsertPropose / InsertPrevote / InsertPrecommit (mq.go:87-101) of every
 * message i of the device batch with d_sender[i] >= 0, in batch order.
 * valid_round may be NULL (then -1); sig65 may be NULL (then zeros).
 * Synchronises `stream` (a hipStream_t, NULL = the ctx's stream). */
int hd_mq_insert_device(hd_mq* q, const hd_batch* d_batch, const int32_t* d_sender, void* stream);

/* Replica.Run ingress of a verified batch (replica/replica.go:117-131):
 * message i is inserted iff d_verdict[i] == HD_VERDICT_VALID and its height
 * >= min_height (filterHeight, replica.go:247-249; min_height = the Process's
 * CurrentHeight), with sender d_signer[i] (the admitted index written by
 * hd_verify_batch_device).  Synchronises `stream`. */
int hd_mq_insert_verified_device(hd_mq* q, const hd_batch* d_batch, const uint8_t* d_verdict, const int32_t* d_signer,
                                 int64_t min_height, void* stream);

/* number of buffered messages */
int hd_mq_size(hd_mq* q, uint64_t* n);

/* Consume (mq.go:36-66): remove every message with height <= h and write
 * them to the HOST arrays of *out (valid_round, sig65 and adv_class may be
 * NULL) and out_sender (may be NULL), in consumption order: senders
 * ascending (the reference walks a Go map, i.e. an unspecified sender
 * order), each sender's messages by (height, round, arrival).  *n_out = the
 * number consumed.  HD_ECAP, with nothing removed and *n_out = the number
 * that would be returned, when that exceeds cap. */
int hd_mq_consume(hd_mq* q, int64_t h, const hd_batch_out* out, int32_t* out_sender, uint32_t cap, uint32_t* n_out);

/* DropMessagesBelowHeight (mq.go:70-83): remove every message with height < h */
int hd_mq_drop_below(hd_mq* q, int64_t h);

#ifdef __cplusplus
}
#endif
#endif
