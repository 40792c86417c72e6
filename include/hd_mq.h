/* hd_mq.h -- bulk MessageQueue on the GPU (mq/mq.go), SURVEY §8(f)3.
 *
 * Replaces mq.MessageQueue (mq/mq.go:19-143) for batch ingress:
 *   - one queue per sender, keyed by the message's From (id.Signatory, the
 *     32 bytes themselves), like mq.go's map[id.Signatory][]interface{}
 *     (mq.go:19-22, 107-110).  A sender's queue exists from its first insert
 *     until the hd_mq is destroyed, as the map entry does in the reference;
 *   - each queue ordered by (height, round), stable for equal keys
 *     (mq.go:116-135), at most max_capacity messages: inserting into a full
 *     queue drops its largest element (mq.go:137-142).  A batch insert has the
 *     effect of inserting the batch's messages one at a time in batch
 *     (= arrival) order;
 *   - the admitted-signatory filter is applied at CONSUME time against the set
 *     passed then (mq.go:49-51, procsAllowed), so messages buffered from a
 *     sender that a later ResetHeight admits are delivered
 *     (replica/replica.go:132-145).
 *
 * Messages are copied into device memory owned by the queue.  Like
 * mq.MessageQueue, an hd_mq is not safe for concurrent use. */
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
 * message i of the device batch with d_insert[i] != 0 (d_insert NULL: every
 * message), in batch order, into the queue of its from32.  The reference
 * assumes the caller authenticated the sender (mq.go:85-106).
 * valid_round may be NULL (then -1); sig65 may be NULL (then zeros).
 * Returns once every kernel the insert queued on `stream` (a hipStream_t,
 * NULL = the ctx's stream), and all work queued there before it, has
 * completed: the host spins on a word the insert's last kernel writes to
 * mapped memory instead of synchronising the stream, so d_batch may be
 * reused at once. */
int hd_mq_insert_device(hd_mq* q, const hd_batch* d_batch, const uint8_t* d_insert, void* stream);

/* Replica.Run ingress of a verified batch (replica/replica.go:117-131):
 * message i is inserted iff it is authenticated -- d_verdict[i] is
 * HD_VERDICT_VALID or HD_VERDICT_NOT_ADMITTED, i.e. the recovered signatory
 * equals From -- and its height >= min_height (filterHeight,
 * replica.go:247-249; min_height = the Process's CurrentHeight).  Membership
 * is NOT checked here: hd_mq_consume applies procsAllowed (mq.go:49-51).
 * Returns as hd_mq_insert_device does. */
int hd_mq_insert_verified_device(hd_mq* q, const hd_batch* d_batch, const uint8_t* d_verdict, int64_t min_height,
                                 void* stream);

/* number of buffered messages; number of sender queues created so far */
int hd_mq_size(hd_mq* q, uint64_t* n);
int hd_mq_senders(hd_mq* q, uint32_t* n);

/* Consume (mq.go:36-66): remove every message with height <= h.  Those whose
 * sender is in procsAllowed are written to the HOST arrays of *out
 * (valid_round, sig65 and adv_class may be NULL) and out_sender (may be NULL:
 * the sender queue's id, 0, 1, ... in queue-creation order), in consumption
 * order: sender queues in creation order (the reference walks a Go map, an
 * unspecified order), each queue by (height, round, arrival); the others are
 * dropped.  procsAllowed: allowed32 = n_allowed x 32 bytes (host, any order);
 * allowed32 == NULL uses the ctx's admitted set (hd_set_signatories) as it is
 * at this call.  *n_out = messages delivered; *n_removed (may be NULL) =
 * messages removed, delivered or not (Consume's return value n).  HD_ECAP,
 * with nothing removed and *n_out = the number that would be delivered, when
 * that exceeds cap. */
int hd_mq_consume(hd_mq* q, int64_t h, const uint8_t* allowed32, uint32_t n_allowed, const hd_batch_out* out,
                  int32_t* out_sender, uint32_t cap, uint32_t* n_out, uint32_t* n_removed);

/* The replica's flush (replica.go:251-264: Consume the current height into
 * the Process) in one call: hd_mq_consume into *out, then
 * hd_votes_insert_batch of the delivered messages into the vote logs v
 * (status / double_of / events per delivered message, as
 * hd_votes_insert_batch; proposes get HD_VOTE_NOT_VOTE and are left to the
 * caller).  One host round trip and one foreign call per flush.  HD_ECAP as
 * hd_mq_consume (nothing removed or inserted). */
struct hd_votes;
int hd_mq_consume_votes(hd_mq* q, struct hd_votes* v, int64_t h, const uint8_t* allowed32, uint32_t n_allowed,
                        const hd_batch_out* out, int32_t* out_sender, uint32_t cap, uint32_t* n_out,
                        uint32_t* n_removed, uint8_t* status, uint32_t* double_of, uint8_t* events,
                        uint32_t* n_inserted);

/* DropMessagesBelowHeight (mq.go:70-83): remove every message with height < h */
int hd_mq_drop_below(hd_mq* q, int64_t h);

#ifdef __cplusplus
}
#endif
#endif
