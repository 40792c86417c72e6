/* hd_votes.h -- incremental vote logs and count table of one height
 * (process/state.go PrevoteLogs / PrecommitLogs / TraceLogs), SURVEY §8(f)1.
 *
 * The reference keeps map[Round]map[Signatory]Prevote (state.go:49-57) and
 * recounts a round's votes for a value with an O(n) loop every time a rule is
 * tried (process.go:486-491, 574-579, 626-631, 696-701), i.e. O(n^2) work per
 * round.  An hd_votes keeps the same logs plus, per (round, type), a count per
 * value, updated on insert, so every T-predicate of SURVEY §8(a) is O(1):
 *
 *   T1/T3/T4/T6  #votes of a type in a round for a value   hd_votes_count
 *   T2/T5        len(PrevoteLogs[r]) / len(PrecommitLogs[r])  hd_votes_len
 *   T7           len(TraceLogs[r])                         hd_votes_trace_len
 *
 * and, with f set (hd_votes_set_f), each insert reports the thresholds it
 * made a log reach exactly (HD_VOTE_EV_*).  L47 is an EQUALITY,
 * len(PrecommitLogs[CurrentRound]) == 2f+1 (process.go:658), tried after every
 * precommit insert (process.go:268) and at StartRound (process.go:310): it
 * fires on the insert that makes the log exactly 2f+1 when that round is the
 * current one, and a round entered with more than 2f+1 buffered precommits
 * never fires it.  A batch insert loses the intermediate lengths, so the
 * crossing is reported per message.
 *
 * Insertion follows insertPrevote / insertPrecommit (process.go:823-892):
 * accepted iff height == the table's height; first wins per (round, From); a
 * later vote from the same From in the same round is an identical duplicate
 * (same value -- Prevote.Equal over height, round, value, from, all but value
 * equal by construction) dropped silently, or a double vote (the caller's
 * Catcher.CatchDoublePrevote/Precommit, process.go:838-843, 875-880, gets the
 * logged value back); an accepted vote adds From to TraceLogs[round].
 * Proposes stay with the caller (scheduler / validator callbacks,
 * process.go:758-819); a VALID propose's signer is added to the trace with
 * hd_votes_trace_propose (process.go:810-815).
 *
 * Host memory only, no device calls.  Not safe for concurrent use (one per
 * Process, which is single-goroutine, process.go:100-101). */
#ifndef HD_VOTES_H
#define HD_VOTES_H

#include <stdint.h>

#include "hd_verify.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hd_votes hd_votes;

/* per-insert status */
#define HD_VOTE_INSERTED 0     /* logged (insert* returned true)                        */
#define HD_VOTE_WRONG_HEIGHT 1 /* height != the table's height (process.go:824, 861)    */
#define HD_VOTE_DUPLICATE 2    /* identical vote already logged: dropped                */
#define HD_VOTE_DOUBLE 3       /* different vote from the same From logged: dropped,
                                  the logged value is reported (CatchDouble*)           */
#define HD_VOTE_NOT_VOTE 4     /* type is not Prevote/Precommit (batch insert only)     */
#define HD_VOTE_SKIPPED 5      /* verdict != VALID (batch insert only)                  */

/* quorum events of one insert (bit mask) */
#define HD_VOTE_EV_PREVOTE_2F1 1u   /* len(PrevoteLogs[r]) became 2f+1 (L34's >= first true, process.go:534)  */
#define HD_VOTE_EV_PRECOMMIT_2F1 2u /* len(PrecommitLogs[r]) became 2f+1: L47's == (process.go:658)        */
#define HD_VOTE_EV_TRACE_F1 4u      /* len(TraceLogs[r]) became f+1 (L55's >= first true, process.go:751)   */

/* an empty table for `height` (NewProcess / State, state.go:66-78) */
int hd_votes_create(int64_t height, hd_votes** out);
/* f of the quorum events (replica.go:54, 138: len(signatories) / 3;
 * UINT32_MAX, the initial value, reports none).  Kept across resets. */
int hd_votes_set_f(hd_votes* v, uint32_t f);
int hd_votes_destroy(hd_votes* v);

/* empty every log and move to `height`: the reset of
 * tryCommitUponSufficientPrecommits (process.go:718-724) and of a
 * ResetHeight (replica.go:216-235) */
int hd_votes_reset(hd_votes* v, int64_t height);
int hd_votes_height(const hd_votes* v, int64_t* height);

/* insertPrevote / insertPrecommit of one vote.  existing_value32 (may be
 * NULL) receives the logged value when *status == HD_VOTE_DOUBLE; events
 * (may be NULL) the HD_VOTE_EV_* this insert caused. */
int hd_votes_insert(hd_votes* v, uint8_t type, int64_t height, int64_t round, const uint8_t* value32,
                    const uint8_t* from32, uint8_t* status, uint8_t* existing_value32, uint8_t* events);

/* the votes of a HOST batch in batch (= arrival) order: message i is
 * inserted iff verdict == NULL or verdict[i] == HD_VERDICT_VALID, and its
 * type is Prevote or Precommit.  status (N, may be NULL) gets each message's
 * HD_VOTE_*; double_of (N, may be NULL) gets, for HD_VOTE_DOUBLE, the batch
 * index of the logged vote if it came from this batch, else UINT32_MAX;
 * events (N, may be NULL) gets each message's HD_VOTE_EV_* mask;
 * *n_inserted (may be NULL) counts HD_VOTE_INSERTED. */
int hd_votes_insert_batch(hd_votes* v, const hd_batch* batch, const uint8_t* verdict, uint8_t* status,
                          uint32_t* double_of, uint8_t* events, uint32_t* n_inserted);

/* TraceLogs[round][from] = true for an accepted VALID propose
 * (process.go:810-815); events (may be NULL): HD_VOTE_EV_TRACE_F1 if this
 * made the trace reach f+1 */
int hd_votes_trace_propose(hd_votes* v, int64_t round, const uint8_t* from32, uint8_t* events);

/* #votes of `type` in `round` whose value equals value32 (T1/T3/T4/T6) */
int hd_votes_count(const hd_votes* v, uint8_t type, int64_t round, const uint8_t* value32, uint32_t* n);
/* len(PrevoteLogs[round]) / len(PrecommitLogs[round]) (T2/T5) */
int hd_votes_len(const hd_votes* v, uint8_t type, int64_t round, uint32_t* n);
/* len(TraceLogs[round]) (T7) */
int hd_votes_trace_len(const hd_votes* v, int64_t round, uint32_t* n);
/* the logged vote of `from32` in (type, round): *found = 0/1, value32 (may
 * be NULL) receives its value */
int hd_votes_get(const hd_votes* v, uint8_t type, int64_t round, const uint8_t* from32, uint8_t* value32,
                 int* found);

#ifdef __cplusplus
}
#endif
#endif
