"""Full-size bit-exactness of the product path against the CPU restatements
(test infrastructure: used by tests/ and bench.py's untimed check legs only).

`full_check` takes a batch the GPU verified and tallied and recomputes every
output on the host, independently of the library:
  * verdicts and recovered signatories: oracle/secp_port.cpp ('port-secp-class',
    bit-exact with the C oracle oracle/hd_oracle.c by
    tests/test_oracle.py::test_secp_class_port_equals_c_oracle), threaded;
  * tally rows: oracle_tally (oracle/hd_oracle.c) over the HOST verdicts --
    first-wins per (height, round, type, From) (process/process.go:823-892),
    counts per (h, r, type, value), distinct signers per (h, r, type) and per
    (h, r) (process.go:486-494, 534, 574-582, 626-632, 658, 696-702, 751);
  * decisions: oracle_tally's predicate bits per round (the C restatement of
    hd_pyoracle.decide_round) against hyperdrive_amd.quorum.decide on the
    library's tally, with the round's canonical value as the propose.
Nothing here feeds a product output; the GPU side is the library's own
(verify + hd_tally on the GPU verdicts).
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

DECIDE_BITS = ("timeout_prevote", "precommit_nil", "timeout_precommit_reached", "timeout_precommit_exact", "skip",
               "precommit_value", "commit")


def host_threads() -> int:
    """Threads this process may use: the affinity mask bounded by the
    cgroup's CPU quota (a GPU box shows the whole machine's CPUs but grants
    one GPU's share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, period = fh.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(period)))
    except (OSError, ValueError):
        pass
    return max(1, n)


def ports():
    """(SecpPort, COracle) built from oracle/ (make)."""
    import subprocess
    from oracle_c import COracle, SecpPort
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    b = os.path.join(ROOT, "oracle", "_build")
    return SecpPort(os.path.join(b, "libsecpport.so")), COracle(os.path.join(b, "liboracle.so"))


def full_check(v, batch, gpu_verdict: np.ndarray, gpu_recovered: np.ndarray, sigs: np.ndarray,
               threads: int = 0) -> dict:
    """v: the hyperdrive_amd.Verifier that verified `batch` (a host Batch);
    gpu_verdict [n] / gpu_recovered [n, 32]: its outputs.  Returns the four
    booleans (verdicts, signatories, tally_rows, decisions) plus sizes and
    host timings."""
    import hd_pyoracle as O
    from hyperdrive_amd import quorum
    threads = threads or host_threads()
    sp, co = ports()
    n = len(batch)
    f = len(sigs) // 3
    t0 = time.perf_counter()
    cv, crec = sp.verify(batch, sigs, True, threads=threads)
    t1 = time.perf_counter()
    ok_v = bool(np.array_equal(cv, np.asarray(gpu_verdict, np.uint8)))
    ok_s = bool(np.array_equal(crec, np.asarray(gpu_recovered, np.uint8).reshape(n, 32)))
    pv_cache = {}

    def pv(h, r):
        k = (h, r)
        if k not in pv_cache:
            pv_cache[k] = O.canonical_value(h, r)
        return pv_cache[k]

    tal = co.tally(batch, cv, f, propose_value=pv)        # the host's tally of the host's verdicts
    t2 = time.perf_counter()
    gt = v.tally(batch, np.asarray(gpu_verdict, np.uint8))  # the library's tally of the GPU's verdicts
    t3 = time.perf_counter()
    val = batch.value
    c_counts = {(int(h), int(r), int(t), val[rep].tobytes()): int(k) for h, r, t, rep, k in tal["counts"].tolist()}
    c_dist = {}
    for h, r, p, c, _, _ in tal["hr"].tolist():
        if p:
            c_dist[(h, r, 2)] = p
        if c:
            c_dist[(h, r, 3)] = c
    c_any = {(h, r): a for h, r, _, _, a, _ in tal["hr"].tolist()}
    ok_t = c_counts == gt.count and c_dist == gt.distinct and c_any == gt.distinct_any
    ok_d = True
    bad_rounds = 0
    for (h, r), d in zip(tal["hr"][:, :2].tolist(), tal["decide"].tolist()):
        want = {k: bool(d >> j & 1) for j, k in enumerate(DECIDE_BITS)}
        got = quorum.decide(gt, h, r, f, pv(h, r), True)
        if any(want[k] != got[k] for k in DECIDE_BITS):
            ok_d = False
            bad_rounds += 1
    t4 = time.perf_counter()
    return {"messages": n, "verdicts": ok_v, "signatories": ok_s, "tally_rows": bool(ok_t), "decisions": ok_d,
            "rounds": int(len(tal["hr"])), "count_rows": int(len(tal["counts"])), "rounds_differing": bad_rounds,
            "commits": int(sum(d >> 6 & 1 for d in tal["decide"].tolist())),
            "verdict_hist": np.bincount(cv, minlength=8).tolist(),
            "host_threads": threads, "host_verify_s": t1 - t0, "host_tally_s": t2 - t1, "gpu_tally_s": t3 - t2,
            "compare_s": t4 - t3,
            "checker": "verdicts/signatories: oracle/secp_port.cpp (bit-exact with oracle/hd_oracle.c); tally rows "
                       "and decisions: oracle_tally (oracle/hd_oracle.c) over the host verdicts vs hd_tally + "
                       "quorum.decide over the GPU verdicts"}
