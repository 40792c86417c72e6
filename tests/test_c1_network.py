"""BASELINE configs[0] (C1: "4 replicas (f=1), 100 heights") through one
replica's batch ingress -- see tests/c1_chain.py for the stream and the chain.

CPU: the committed stream (tests/golden/c1_stream.npz, tests/golden/make_c1.py)
through the chain of CPU restatements reproduces the committed flush records:
every height 1..100 commits its proposer's value at 2f+1 = 3, height 50 first
stalls at 2f = 2 precommits and commits when the third arrives (the
process_test.go 2f vs 2f+1 boundary), L47's exact crossing fires once per
committed height.
GPU: the same stream as wire bytes through hyperdrive_amd.Ingress (unmarshal
-> verify -> filterHeight -> mq -> consume -> vote logs) reproduces every
flush record bit for bit: delivered counts, vote statuses, the quorum-crossing
events and the decisions."""
import json
import os

import numpy as np
import pytest

from c1_chain import HEIGHTS, replica_view, run_gpu, run_oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load():
    z = dict(np.load(os.path.join(GOLDEN, "c1_stream.npz")))
    with open(os.path.join(GOLDEN, "c1_expected.json")) as fh:
        exp = json.load(fh)
    return z, exp


def _expected_shape(exp, oracle):
    commits = exp["commits"]
    assert [h for h, _ in commits] == list(range(1, HEIGHTS + 1))
    assert all(v == oracle.canonical_value(h, 0).hex() for h, v in commits)
    recs = exp["records"]
    at50 = [r for r in recs if r["height"] == 50]
    assert len(at50) == 2 and not at50[0]["decision"]["commit"] and at50[1]["decision"]["commit"]
    assert at50[0]["ev_precommit_2f1"] == 0 and at50[1]["ev_precommit_2f1"] == 1
    # one L47 crossing per height, over all its flushes
    per_h = {}
    for r in recs:
        per_h[r["height"]] = per_h.get(r["height"], 0) + r["ev_precommit_2f1"]
    assert per_h.pop(HEIGHTS + 1) == 0          # the final, empty flush at height 101
    assert set(per_h.values()) == {1}
    # the stream's adversarial parts were exercised: duplicates and double votes logged
    assert sum(r["status"][2] for r in recs) > 0 and sum(r["status"][3] for r in recs) > 0


def test_c1_oracle_chain_reproduces_fixture(coracle, oracle):
    z, exp = _load()
    _expected_shape(exp, oracle)
    rep = run_oracle(z, coracle)
    assert [list(c) for c in rep.commits] == exp["commits"]
    assert rep.records == exp["records"]


@pytest.mark.gpu
def test_c1_gpu_ingress_matches_chain(gpu):
    z, exp = _load()
    v = gpu.Verifier(0)
    try:
        rep = run_gpu(z, v)
    finally:
        v.close()
    assert [list(c) for c in rep.commits] == exp["commits"]
    for got, want in zip(rep.records, exp["records"]):
        assert got == want, (got, want)
    assert len(rep.records) == len(exp["records"])


def _canonical_commits(oracle):
    return [[h, oracle.canonical_value(h, 0).hex()] for h in range(1, HEIGHTS + 1)]


def test_c1_four_replicas_commit_identically(coracle, oracle):
    """C1 as the reference's network test states it (replica_test.go:414-423:
    every live replica commits the same values): 4 replicas, each with its
    own arrival order of the same broadcast stream, through the chain of CPU
    restatements -- every replica commits the proposer's value at every
    height 1..100."""
    z, _ = _load()
    want = _canonical_commits(oracle)
    for k in range(4):
        rep = run_oracle(replica_view(z, k), coracle)
        assert [list(c) for c in rep.commits] == want, k


@pytest.mark.gpu
def test_c1_four_replicas_gpu(gpu, coracle, oracle):
    """The same 4 replicas on the GPU, one context and one Ingress each (one
    hd_ctx per replica): every replica's flush records equal its
    own restatement chain's, and all four commit the same 100 values."""
    z, _ = _load()
    want = _canonical_commits(oracle)
    ctxs = [gpu.Verifier(0) for _ in range(4)]
    try:
        for k, v in enumerate(ctxs):
            view = replica_view(z, k)
            rep = run_gpu(view, v)
            ref = run_oracle(view, coracle)
            assert rep.records == ref.records, k
            assert [list(c) for c in rep.commits] == want, k
    finally:
        for v in ctxs:
            v.close()
