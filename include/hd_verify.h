/*
 * hd_verify.h -- C ABI of the MI355X batch authenticator + tallier for
 * hyperdrive consensus messages (libhdverify.so).
 *
 * Plain C: pointers and sizes only, no HIP/torch types in the signatures, so
 * that hyperdrive's Go packages can bind it through cgo (INTEGRATION.md shows
 * the binding).  What each entry point replaces in the reference
 * (tuanggolt/hyperdrive @ /root/reference):
 *
 *   hd_verify_batch     the authentication precondition the reference leaves to
 *                       its caller before Replica.Propose/Prevote/Precommit
 *                       (replica/replica.go:153-181; "assumes that the sender
 *                       has already been authenticated", mq/mq.go:85-101,
 *                       process/process.go:95-98): per message
 *                       NewProposeHash / NewPrevoteHash / NewPrecommitHash
 *                       (process/message.go:53-78, 165-186, 263-284) ->
 *                       id.Signature.Signatory(&hash) (message_test.go:152) ->
 *                       Signatory.Equal(From) (message_test.go:154) ->
 *                       procsAllowed[From] (mq/mq.go:49-51).
 *   hd_set_signatories  building procsAllowed from the signatory set
 *                       (replica/replica.go:69-72) and its rebuild on
 *                       ResetHeight (replica/replica.go:136-144).
 *   hd_tally            the first-wins vote logs (process/process.go:823-892)
 *                       and the counting loops of the 2f+1 / f+1 rules
 *                       (process.go:486-494, 534, 574-582, 626-632, 658,
 *                       696-702, 751), for every (height, round) of a batch.
 *
 * Ownership: all host buffers are caller-owned; the library copies what it
 * needs and keeps no pointer after a call returns.  Device buffers passed to
 * the *_device variants are caller-owned device memory (HBM) on the ctx's
 * device.  Threading: one hd_ctx per caller thread (the reference's Process is
 * single-goroutine, process.go:100-101); distinct contexts may share a device.
 * Errors: per-message failures are verdicts, never error returns; a negative
 * return is an HD_E* code (invalid argument, allocation, device failure).
 */
#ifndef HD_VERIFY_H
#define HD_VERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes ---------------------------------------------------- */
#define HD_OK 0
#define HD_EINVAL (-1)   /* bad argument (NULL pointer, size mismatch)       */
#define HD_ENOMEM (-2)   /* host or device allocation failed                 */
#define HD_EDEVICE (-3)  /* HIP runtime / kernel failure                     */
#define HD_ECAP (-4)     /* hd_tally_out capacity too small (n_* hold need)  */
#define HD_EAGAIN (-5)   /* hd_tally_collect: more groups than were staged;
                            run hd_tally_device_bitmap on the same inputs   */

/* ---- message types (process/message.go:11-22) ------------------------ */
#define HD_TYPE_PROPOSE 1
#define HD_TYPE_PREVOTE 2
#define HD_TYPE_PRECOMMIT 3

/* ---- per-message verdicts -------------------------------------------- */
#define HD_VERDICT_VALID 0              /* recovered signatory == From, From admitted */
#define HD_VERDICT_BAD_RECID 1          /* V >= 4 (go-ethereum checkSignature)       */
#define HD_VERDICT_BAD_RS 2             /* r or s == 0 or >= n                         */
#define HD_VERDICT_NO_POINT 3           /* x = r (+n) not a curve x-coordinate        */
#define HD_VERDICT_INFINITY 4           /* recovered point at infinity                */
#define HD_VERDICT_SIGNATORY_MISMATCH 5 /* recovered signatory != From                */
#define HD_VERDICT_NOT_ADMITTED 6       /* From not in the admitted signatory set     */
#define HD_VERDICT_BAD_TYPE 7           /* type not Propose/Prevote/Precommit         */
#define HD_VERDICT_NOT_AUTHENTIC 8      /* hd_authenticate_batch_device only: From's
                                           known key does not verify the signature;
                                           the recovery that would name the reason
                                           (NO_POINT, INFINITY or SIGNATORY_MISMATCH)
                                           was skipped                                 */

typedef struct hd_ctx hd_ctx;

/* Structure-of-arrays batch.  Strings are raw bytes: value32 = process.Value
 * ([32]byte), from32 = id.Signatory ([32]byte), sig65 = id.Signature
 * (R || S || V, [65]byte).  valid_round may be NULL when the batch carries no
 * Proposes (then -1 = InvalidRound is used). */
typedef struct {
    uint32_t n;
    const uint8_t* type;
    const int64_t* height;
    const int64_t* round;
    const int64_t* valid_round;
    const uint8_t* value32;
    const uint8_t* from32;
    const uint8_t* sig65;
} hd_batch;

/* ---- context --------------------------------------------------------- */
int hd_ctx_create(int device, hd_ctx** out);
/* Destroy first waits for the context's own stream, its verify calls, and the
 * last work of every caller stream that used its scratch or tables (routes,
 * tallies, digests, codec, generator); other work on the device is not waited
 * for.
 * Streams: a `stream` argument of NULL means the context's own stream, which
 * is created non-blocking: it is NOT ordered after work on the legacy NULL
 * stream (e.g. torch's default stream).  Device inputs produced on another
 * stream must be ordered by the caller (pass that stream, or an event). */
int hd_ctx_destroy(hd_ctx* ctx);
/* The pubkey encoding id.NewSignatory hashes [renproject/id v0.4.2; not
 * confirmable in this container, SURVEY §8(c)]:
 *   HD_PUBKEY_COMPRESSED   (1, default) SHA-256(02|03 || X), 33 bytes
 *   HD_PUBKEY_UNCOMPRESSED (0)          SHA-256(04 || X || Y), 65 bytes
 *   HD_PUBKEY_RAW64        (2)          SHA-256(X || Y), 64 bytes (X, Y 32-byte big-endian)
 *   HD_PUBKEY_XY_STRIPPED  (3)          SHA-256(X.Bytes() || Y.Bytes()), Go big.Int minimal
 *                                       big-endian encodings (leading zero bytes dropped), <= 64 bytes
 * Changing it drops the learned keys of the known-key fast path. */
#define HD_PUBKEY_UNCOMPRESSED 0
#define HD_PUBKEY_COMPRESSED 1
#define HD_PUBKEY_RAW64 2
#define HD_PUBKEY_XY_STRIPPED 3
int hd_ctx_set_pubkey_format(hd_ctx* ctx, int format);
/* Admitted set = procsAllowed.  sigs32: n x 32 bytes, any order, duplicates
 * allowed.  Signer indices reported by the library index this array.
 * Blocking: waits for the context's device work in flight (a verify call
 * still learning keys must not see its slots reassigned), so call it between
 * batches, as ResetHeight does (replica/replica.go:136-144). */
int hd_set_signatories(hd_ctx* ctx, const uint8_t* sigs32, uint32_t n);
/* Known-key fast path (on by default; HD_VERIFY_FASTPATH=0 in the
 * environment turns it off for new contexts).  The first message of an
 * admitted signatory that verifies VALID through the full recovery teaches
 * the context that signatory's public key; later messages claiming that
 * signatory are checked against the key with fixed-base tables
 * (R == s^-1 (m G + r P)) and only fall back to the full recovery when the
 * check fails.  Verdicts, recovered signatories, signer indices and bitmaps
 * are identical either way.  Keys are kept across hd_set_signatories for
 * signatories that stay admitted and dropped when the pubkey format changes. */
int hd_ctx_set_fastpath(hd_ctx* ctx, int enable);
/* known_keys: admitted signatories whose key tables are built;
 * last_fallback: messages of the last verify call that took the full
 * recovery (either may be NULL; synchronises the device) */
int hd_ctx_fastpath_stats(hd_ctx* ctx, uint32_t* known_keys, uint32_t* last_fallback);
/* Foreign-key slots (HD_VAR_FOREIGN_KEYS): ready_slots = foreign slots whose
 * tables are built; evictions = slotless Froms promoted so far into the slot
 * of a colder foreign key (a From with more recoveries since the last check
 * than twice the slot holder's known-key checks + 4; hd_fastverify.hip
 * fb_evict); checks = eviction checks so far (each waited for the context's
 * earlier verify calls).  Any may be NULL; synchronises the context's calls. */
int hd_ctx_foreign_stats(hd_ctx* ctx, uint32_t* ready_slots, uint32_t* evictions, uint32_t* checks);
/* Shape of the known-key check as the context runs it now (for cost models):
 * g_windows / key_windows: fixed-base windows of the G table and of the
 * per-key tables (one table point each; the first is loaded, the rest are
 * mixed additions); msgs_per_inversion: messages that share one inversion of
 * each kind in the last verify call (the split check takes 16 from 2^20 - 2^16
 * messages up, else 8; 2 for the paired kernel).
 * Host-only (no device access); any pointer may be NULL. */
int hd_ctx_fastpath_geometry(hd_ctx* ctx, int* g_windows, int* key_windows, int* msgs_per_inversion);
/* Device-time profile for roofline reports.  While enabled, every verify
 * call of the context records HIP events on its stream around the whole call
 * and around the known-key check's sums kernel (k_fast_sums, the dominant
 * kernel).  hd_ctx_profile_read waits for the recorded events, returns the
 * calls recorded since the last read with their summed milliseconds (either
 * pointer may be NULL; sums_ms covers the calls that ran the kernel, counted
 * in *sums_launches) and clears the record. */
int hd_ctx_profile(hd_ctx* ctx, int enable);
/* Kernel variants of a context, for A/B measurements and for the tests that
 * run every compiled instantiation against the golden fixtures.  Defaults
 * come from the environment at context creation (the variable in brackets);
 * HD_EINVAL for an unknown key or value. */
#define HD_VAR_VERIFY_WAVES 0   /* k_verify register budget, waves per SIMD: 2, 3 (default) or 4 (compressed
                                   pubkeys; the other formats run the 3-wave build) [HD_VERIFY_WAVES] */
#define HD_VAR_SUM_WAVES 1      /* k_fast_sums waves per SIMD: 2, 3 or 4 (128 VGPRs, table points loaded when
                                   used); 0 (default) 4 for batches under two rounds at 3, else 3 [HD_SUM_WAVES] */
#define HD_VAR_SUM_PREFETCH 2   /* k_fast_sums table-point prefetch depth: 1 (default) or 2 [HD_SUM_PF] */
#define HD_VAR_SPLIT_K 4        /* messages per inversion of the known-key check: -1 by batch size (default),
                                   8 or 16 [HD_FAST_K] */
#define HD_VAR_RECOVER_G 5      /* the full recovery's u1 G: 0 from the fixed-base G table (default), 1 from the
                                   GLV ladder's own 12-bit table [HD_RECOVER_GLV_G] */
#define HD_VAR_KEY_WIDTH 7      /* per-key table windows: 0 by the table budget (default: 22 while every key's
                                   1.48 GB table fits, else 20 (407 MB), else 16 (36 MB), else 13 (5 MB); the
                                   budget is HD_FB_MAX_BYTES or 64 GiB per device, shared by the
                                   process's contexts and bounded by the free memory), or 13, 16, 20, 22;
                                   applies from the next hd_set_signatories [HD_FB_PW] */
#define HD_VAR_WAVE_PRIO 8      /* wave issue priority (s_setprio 0..3) of the known-key check's short kernels
                                   (prep, s / Z inversions, comparison, lift, the leftovers' k_verify): above
                                   k_fast_sums' 0 they keep
                                   their SIMD share while the next call's sums waves share the SIMD
                                   [HD_WAVE_PRIO] */
#define HD_VAR_FOREIGN_KEYS 10  /* table slots (0..64) reserved for authenticated Froms outside the admitted set:
                                   a NOT_ADMITTED recovery teaches the context its key, and later messages of
                                   that From take the known-key check (verdict NOT_ADMITTED, identical to the
                                   recovery's); applies from the next hd_set_signatories (reserved once per
                                   context, when the table budget allows; a later 0 stops using the block); 16 (default),
                                   0 = off [HD_FOREIGN_KEYS] */
#define HD_VAR_SLOW_LIFT 11     /* the known-key check's leftovers: 1 (default) a lift kernel first (x^3 + 7 a
                                   square, else NO_POINT), then the full recovery over the rest; 0 the full
                                   recovery over every leftover (it checks the lift itself) [HD_SLOW_LIFT] */
/* Keys 3, 6, 9, 12, 13 and 14 (the digit pass, the paired kernel's waves, the
 * sums residency cap, the fused comparison, the lean inversions and the sums
 * chain) were measured without gain and removed in round 5: set returns
 * HD_EINVAL for them, get returns their fixed value. */
#define HD_VAR__COUNT 15
int hd_ctx_set_variant(hd_ctx* ctx, int which, int value);
int hd_ctx_get_variant(hd_ctx* ctx, int which, int* value);
int hd_ctx_profile_read(hd_ctx* ctx, uint32_t* calls, double* verify_ms, uint32_t* sums_launches, double* sums_ms);

/* ---- verification ------------------------------------------------------
 * verdict:     n bytes (HD_VERDICT_*), required.
 * recovered32: n x 32 bytes or NULL: recovered signatory (zeros when the
 *              recovery itself failed).
 * valid_bitmap: ceil(n/32) words or NULL: bit i set iff verdict[i] == VALID.
 * Host pointers; synchronous. */
int hd_verify_batch(hd_ctx* ctx, const hd_batch* batch, uint8_t* verdict, uint8_t* recovered32,
                    uint32_t* valid_bitmap);

/* Same, with every pointer (batch fields and outputs) in device memory of the
 * ctx's device; signer (n x int32 or NULL) receives the index of From in the
 * hd_set_signatories array for VALID messages, -1 otherwise.  Enqueued on
 * `stream` (a hipStream_t, NULL = the ctx's stream); asynchronous.  The
 * context keeps three scratch sets used round robin.  Once every admitted
 * signatory's key tables are built, calls issued on different streams run
 * concurrently on the device (a call waits only for the last call that used
 * its scratch set), so a caller that alternates two streams fills the SIMDs
 * one call's low-occupancy kernels leave idle; while keys are still being
 * learned, a call on another stream first waits for the previous call. */
int hd_verify_batch_device(hd_ctx* ctx, const hd_batch* dbatch, uint8_t* d_verdict, uint8_t* d_recovered32,
                           int32_t* d_signer, uint32_t* d_valid_bitmap, void* stream);

/* Authentication only, for the replica ingress: the reference buffers a
 * message only once it is authenticated (process/process.go:95-98,
 * mq/mq.go:85-101) and drops it otherwise, whatever the reason.  Same inputs
 * and ordering as hd_verify_batch_device with verdicts only.  VALID and
 * NOT_ADMITTED are exactly hd_verify_batch_device's; every other message gets
 * a verdict that is neither of them: the same as hd_verify_batch_device's, or
 * HD_VERDICT_NOT_AUTHENTIC where From's key is known and the known-key check
 * fails (then the recovered key is not From's, so the message is not
 * authentic; the full recovery that would classify it is skipped). */
int hd_authenticate_batch_device(hd_ctx* ctx, const hd_batch* dbatch, uint8_t* d_verdict, void* stream);

/* Asynchronous host-buffer verification (the cgo caller's path,
 * replica/replica.go:156-181, without its synchronous upload -> verify ->
 * download): hd_verify_submit queues the upload of `batch`, the verification
 * and the download of the outputs on one of the context's HD_HOST_SLOTS
 * pipelines and returns a ticket; hd_verify_wait(ticket) blocks until the
 * outputs are in the caller's buffers.  Consecutive submits overlap: batch
 * k+1's upload runs under batch k's kernels, and the two pipelines' verify
 * calls under each other.  Inputs in pinned memory (hd_host_alloc) are
 * uploaded by DMA straight from the caller's buffers; pageable inputs are
 * first copied into pinned staging by host threads.  The input buffers must
 * stay unchanged, and the output buffers valid, until the ticket's wait
 * returns.  A submit that reuses a pipeline first completes its previous
 * ticket.  Tickets start at 1; waiting on a completed ticket returns at once. */
#define HD_HOST_SLOTS 3   /* a caller keeps up to 3 in flight: upload, verify and output store of three
                             batches overlap (2 in flight serialise upload + verify + store); more
                             pipelines than the device's 4 hardware queues (with the context's own
                             stream) would share queues and serialise behind each other */
int hd_verify_submit(hd_ctx* ctx, const hd_batch* batch, uint8_t* verdict, uint8_t* recovered32,
                     uint32_t* valid_bitmap, uint64_t* ticket);
int hd_verify_wait(hd_ctx* ctx, uint64_t ticket);
/* Compact host batch (PCIe-lean form of hd_verify_submit, 86 B per vote
 * instead of 146 B).  A replica knows its signatory set and a batch carries
 * few distinct values, so From and value cross PCIe as 16-bit indices:
 *   from_idx[i] <  n_sig: From = row from_idx[i] of the array last passed to
 *                         hd_set_signatories (caller order, duplicates kept;
 *                         n_sig = its length)
 *   from_idx[i] >= n_sig: From = escape32 row from_idx[i] - n_sig (senders
 *                         outside the set, e.g. the NOT_ADMITTED ones)
 *   value_idx[i]:         value = values32 row value_idx[i]
 * The rows are expanded on the device, then verified as hd_verify_submit
 * verifies the expanded batch: verdicts, recovered signatories and bitmaps
 * are byte-identical.  HD_EINVAL (nothing queued) when an index names no
 * row, n_sig + n_escape > 65536 or n_values is 0 or > 65536.  Same ticket
 * semantics as hd_verify_submit; the dictionaries must stay unchanged until
 * the ticket's wait returns too. */
typedef struct {
    uint32_t n;
    const uint8_t* type;
    const int64_t* height;
    const int64_t* round;
    const int64_t* valid_round;   /* NULL: no Proposes (-1 = InvalidRound) */
    const uint16_t* from_idx;     /* n */
    const uint16_t* value_idx;    /* n */
    const uint8_t* sig65;         /* n x 65 */
    uint32_t n_escape;
    const uint8_t* escape32;      /* n_escape x 32 (may be NULL when 0) */
    uint32_t n_values;
    const uint8_t* values32;      /* n_values x 32 */
} hd_batch_compact;
int hd_verify_submit_compact(hd_ctx* ctx, const hd_batch_compact* batch, uint8_t* verdict, uint8_t* recovered32,
                             uint32_t* valid_bitmap, uint64_t* ticket);
/* pinned (page-locked) host memory for inputs the caller fills directly */
int hd_host_alloc(size_t bytes, void** out);
int hd_host_free(void* p);

/* A stream on a hardware queue of its own (a CU-mask stream with every CU
 * set), for a caller's verify or tally streams.  Ordinary streams share the
 * device's few hardware queues (GPU_MAX_HW_QUEUES, 4) round robin, and a
 * cross-stream wait queued in a shared queue holds back the other streams
 * mapped to it.  Destroy with hd_stream_destroy. */
int hd_stream_create_dedicated(hd_ctx* ctx, void** stream);
int hd_stream_destroy(hd_ctx* ctx, void* stream);

/* ---- tally --------------------------------------------------------------
 * Input: a batch and its verdicts.  Candidates are VALID Prevotes and
 * Precommits.  Per (height, round, type, signer) the lowest batch index wins
 * (first-wins, process.go:834-847); later ones are duplicates: identical
 * value -> dropped silently, different value -> what the reference hands to
 * Catcher.CatchDoublePrevote/Precommit (process.go:838-843, 875-880).
 * All output arrays are caller-owned with the given capacities.
 * Values are grouped by their 32 bytes themselves (count_rep names a message
 * carrying the value), so the caller-interned value_id argument SURVEY §8(b)
 * sketches is not needed and not taken. */
typedef struct {
    /* (height, round, type, value) groups, in the batch order of each group's
     * first message (deterministic) */
    uint32_t cap_counts;
    uint32_t n_counts;
    int64_t* count_height;
    int64_t* count_round;
    uint8_t* count_type;
    uint32_t* count_rep;   /* batch index of a message with that value */
    uint32_t* count_n;     /* number of first-wins votes for the value  */
    /* (height, round) groups, in the batch order of each round's first
     * candidate */
    uint32_t cap_hr;
    uint32_t n_hr;
    int64_t* hr_height;
    int64_t* hr_round;
    uint32_t* hr_prevotes;   /* len(PrevoteLogs[r])   */
    uint32_t* hr_precommits; /* len(PrecommitLogs[r]) */
    uint32_t* hr_any;        /* distinct vote signers (TraceLogs[r] without proposes) */
    /* n bytes or NULL: 0 logged, 1 identical duplicate, 2 conflicting
     * duplicate (double vote), 3 not a candidate (of this partition) */
    uint8_t* dup;
    /* cap_hr entries or NULL: batch index of each round's first candidate */
    uint32_t* hr_rep;
} hd_tally_out;

int hd_tally(hd_ctx* ctx, const hd_batch* batch, const uint8_t* verdict, hd_tally_out* out);

/* Same on device-resident inputs (pointers as in hd_verify_batch_device).
 * The logs are keyed by From itself, which equals the recovered signatory of
 * every VALID message.  Results land in the host arrays of `out`;
 * synchronises `stream`. */
int hd_tally_device(hd_ctx* ctx, const hd_batch* dbatch, const uint8_t* d_verdict, hd_tally_out* out, void* stream);

/* Same, with validity given as the valid bitmap of hd_verify_batch_device
 * (e.g. after an all-gather of per-GPU bitmaps over RCCL). */
int hd_tally_device_bitmap(hd_ctx* ctx, const hd_batch* dbatch, const uint32_t* d_valid_bitmap, hd_tally_out* out,
                           void* stream);

/* Asynchronous form of hd_tally_device_bitmap, for a caller that pipelines
 * batches (the cgo binding's VerifyBatchAsync, bench.py): the tally's kernels
 * and ONE download of its results into the ticket's pinned stage are queued on
 * `stream`, and nothing is waited for.  Once the stream has passed that point
 * (an event recorded after this call, or a stream sync), hd_tally_collect
 * fills `out` exactly as hd_tally_device_bitmap would.  The inputs must stay
 * unchanged until then.  The tallies of one context share device scratch, so
 * issue them all on ONE stream (they then run in its order).  Collect waits
 * (on the host, for the ticket's event) until the download has landed.
 *  - The rows are staged at capacities guessed from earlier tallies (the
 *    largest counts seen + 1/4).  A batch with more groups makes collect return
 *    HD_EAGAIN with nothing written; run hd_tally_device_bitmap on the same
 *    inputs instead.  Collect raises the guesses, so the next submit stages more.
 *  - stage / stage_cap: pinned host memory (hd_host_alloc) of at least
 *    hd_tally_stage_bytes(ctx, n, dup) bytes; a smaller stage makes the
 *    submit return HD_ECAP with `need` set.
 *  - dup != 0 stages the per-message classification too (out->dup of collect).
 * The partitioned and routed tallies (several GPUs) stay synchronous. */
typedef struct {
    void* stage;        /* caller: pinned host buffer                          */
    size_t stage_cap;   /* caller: its size in bytes                           */
    int dup;            /* caller: stage the classification                    */
    uint32_t n;         /* set by the submit: the batch size                   */
    uint32_t H, Cg;     /* set by the submit: staged row capacities            */
    size_t need;        /* set by the submit: stage bytes this submit needed   */
    void* done;         /* library: an event recorded after the download
                           (created by the first submit; hd_tally_ticket_release) */
} hd_tally_ticket;
int hd_tally_device_bitmap_async(hd_ctx* ctx, const hd_batch* dbatch, const uint32_t* d_valid_bitmap,
                                 hd_tally_ticket* ticket, void* stream);
int hd_tally_collect(hd_ctx* ctx, const hd_tally_ticket* ticket, hd_tally_out* out);   /* waits for `done` */
int hd_tally_ticket_release(hd_tally_ticket* ticket);
size_t hd_tally_stage_bytes(hd_ctx* ctx, uint32_t n, int dup);

/* Partitioned tally for G GPUs: only candidates with
 * hd_tally_partition_of(height, round, nparts) == part are tallied.
 * First-wins is per (height, round, type, signer), so the owner of an
 * (height, round) sees every duplicate of its keys and the partitions' groups
 * are exactly the unpartitioned tally's: their union, ordered by count_rep /
 * hr_rep, is the single-GPU output, and dup merges by taking the minimum over
 * partitions (a non-owner reports 3). */
int hd_tally_device_bitmap_part(hd_ctx* ctx, const hd_batch* dbatch, const uint32_t* d_valid_bitmap, uint32_t part,
                                uint32_t nparts, hd_tally_out* out, void* stream);
/* the partition of an (height, round) among nparts (host function) */
uint32_t hd_tally_partition_of(int64_t height, int64_t round, uint32_t nparts);

/* verify + tally with one upload of the batch */
int hd_process_batch(hd_ctx* ctx, const hd_batch* batch, uint8_t* verdict, uint8_t* recovered32,
                     uint32_t* valid_bitmap, hd_tally_out* tally);

/* ---- multi-GPU in one process ----------------------
 * A context per device plus an RCCL communicator over the devices
 * (ncclCommInitAll); for one caller (a Replica) that owns several GPUs.
 * hd_multi_verify_batch = hd_process_batch over the devices: message i is
 * uploaded to and verified on the device whose contiguous 32-aligned shard
 * holds i (each device receives 1/G of the batch over PCIe); with `tally`
 * non-NULL each device routes its shard's candidates to the owners of their
 * rounds (hd_route_candidates_device) with one grouped ncclSend / ncclRecv
 * over xGMI, every owner tallies what it received (hd_tally_routed_device)
 * and the host merges the disjoint tables into the single-device output
 * (same rows, same order).  Host buffers, synchronous; outputs as
 * hd_verify_batch / hd_tally.  devices: ngpus ordinals (NULL: 0 ..
 * ngpus-1); a device listed twice gets two contexts and the exchange uses
 * device copies (RCCL takes one rank per device).  Not thread-safe (one
 * hd_multi per caller thread). */
typedef struct hd_multi hd_multi;
int hd_multi_create(int ngpus, const int* devices, hd_multi** out);
int hd_multi_destroy(hd_multi* m);
/* number of devices; whether the exchange runs over RCCL (else copies) */
int hd_multi_size(hd_multi* m, int* ngpus, int* uses_rccl);
/* the context of device slot k (fast-path stats etc.), NULL if out of range */
hd_ctx* hd_multi_ctx(hd_multi* m, int k);
int hd_multi_set_signatories(hd_multi* m, const uint8_t* sigs32, uint32_t n);
int hd_multi_set_pubkey_format(hd_multi* m, int format);
int hd_multi_verify_batch(hd_multi* m, const hd_batch* batch, uint8_t* verdict, uint8_t* recovered32,
                          uint32_t* valid_bitmap, hd_tally_out* tally);

/* ---- synthetic workload (seeded; benchmarks/tests) --------
 * kind 0: votes (signer = i % S, type = 2 + (i/S)%2, h = 1 + i/(2S), r = 0)
 * kind 1: rounds (h = 1; per round 1 Propose + S Prevotes + S Precommits)
 * adv_pct: percentage of messages corrupted by the adversarial classes. */
int hd_gen_keys(hd_ctx* ctx, uint32_t S, uint8_t* signatories32, uint8_t* foreign32);
typedef struct {
    uint8_t* type;
    int64_t* height;
    int64_t* round;
    int64_t* valid_round;
    uint8_t* value32;
    uint8_t* from32;
    uint8_t* sig65;
    int8_t* adv_class; /* may be NULL */
} hd_batch_out;
/* device pointers; messages start .. start+n-1 of the workload. */
int hd_gen_batch_device(hd_ctx* ctx, uint32_t kind, uint64_t start, uint32_t n, uint32_t S, uint32_t adv_pct,
                        const uint8_t* d_signatories32, const uint8_t* d_foreign32, const hd_batch_out* d_out,
                        void* stream);

/* ---- multi-GPU tally routing (the C4 data path) -----------
 * The tally of a batch sharded over G GPUs without replicating the batch:
 * hd_route_candidates_device turns the candidates of one device's shard --
 * VALID Prevotes / Precommits per d_valid_bitmap, global index base_index + i
 * -- into HD_ROUTE_ROW_BYTES rows in d_rows (16-byte aligned, cap_rows rows),
 * grouped by the owner rank of their round (hd_tally_partition_of(h, r,
 * nparts), nparts <= 64) and in index order inside each group; counts[nparts]
 * (host) gets the group sizes (group o starts at row sum(counts[0..o))).
 * Synchronous (one small download); HD_ECAP when cap_rows is too small;
 * HD_EINVAL (nothing written) when a candidate's From is not in the context's
 * current admitted set (the set changed since verification): a row names its
 * signer by admitted index, so such a vote could not be told apart from
 * another non-admitted signer's on the owner.
 * The rows cross xGMI (grouped ncclSend/Recv or an all-to-all); the owner
 * concatenates what it received in source-rank order (= global index order)
 * and calls hd_unroute_device: a device batch (type, height, round, value32,
 * From rebuilt from the admitted set; valid_round -1 if given) and each
 * row's global index; hd_tally_routed_device then tallies it (every row is a
 * candidate; count_rep / hr_rep are global indices; dup is per received row).
 * The owners' tables are disjoint and their union ordered by count_rep /
 * hr_rep is the single-GPU tally.  All contexts need the same admitted set. */
#define HD_ROUTE_ROW_BYTES 64
int hd_route_candidates_device(hd_ctx* ctx, const hd_batch* dshard, const uint32_t* d_valid_bitmap,
                               uint32_t base_index, uint32_t nparts, uint8_t* d_rows, uint32_t cap_rows,
                               uint32_t* counts, void* stream);
/* The same, routing only candidates whose (height, round) is one of the
 * n_rounds pairs (d_round_h[k], d_round_r[k]), sorted lexicographically (as
 * signed int64): the rounds that appear in more than one shard.  A round
 * present in one shard only is complete there, so that shard tallies it
 * itself (hd_tally_device_bitmap, reps + base_index) and keeps only those
 * rows of its local tables; only the shared rounds cross xGMI, to their
 * owners (hd_tally_partition_of).  n_rounds = 0 routes nothing. */
int hd_route_candidates_listed_device(hd_ctx* ctx, const hd_batch* dshard, const uint32_t* d_valid_bitmap,
                                      uint32_t base_index, uint32_t nparts, const int64_t* d_round_h,
                                      const int64_t* d_round_r, uint32_t n_rounds, uint8_t* d_rows,
                                      uint32_t cap_rows, uint32_t* counts, void* stream);
int hd_unroute_device(hd_ctx* ctx, const uint8_t* d_rows, uint32_t n, const hd_batch_out* d_out, uint32_t* d_gidx,
                      void* stream);
int hd_tally_routed_device(hd_ctx* ctx, const hd_batch* dbatch, const uint32_t* d_gidx, hd_tally_out* out,
                           void* stream);

/* ---- misc ------------------------------------------------------------- */
const char* hd_strerror(int code);
/* last HIP error text recorded by the ctx (empty if none) */
const char* hd_ctx_last_error(hd_ctx* ctx);
/* ABI version, bumped on any signature change */
int hd_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* HD_VERIFY_H */
