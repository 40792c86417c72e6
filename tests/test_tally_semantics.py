"""Tally semantics on CPU: the oracle's first-wins logs + the product's host
quorum predicates (hyperdrive_amd.quorum) on the process_test-style scenarios;
the GPU tally is checked against the same oracle in test_gpu_tally.py."""
import pytest

from hyperdrive_amd import quorum
from tally_cases import scenarios


def test_thresholds_f8():
    # n=4 -> 2f+1=3, n=100 -> 67, n=1000 -> 667; f+1 = 2 / 34 / 334
    assert quorum.thresholds(4) == (1, 3, 2)
    assert quorum.thresholds(100) == (33, 67, 34)
    assert quorum.thresholds(1000) == (333, 667, 334)
    assert quorum.thresholds(10) == (3, 7, 4)


@pytest.mark.parametrize("sc", scenarios(), ids=lambda s: s.name)
def test_scenario_predicates(oracle, sc):
    t = oracle.tally(sc.b, sc.verdicts())
    for h, r, pvalue, pvalid, want in sc.expect:
        got = quorum.decide(t, h, r, sc.f, pvalue, pvalid)
        ref = oracle.decide_round(t, h, r, sc.f, pvalue, pvalid)
        assert got == ref
        for k, v in want.items():
            assert got[k] == v, (sc.name, k)


def test_duplicate_classification(oracle):
    sc = [s for s in scenarios() if s.name == "dups_f5"][0]
    t = oracle.tally(sc.b, sc.verdicts())
    n = len(sc.b)
    assert t.dup[: 2 * 5] == [0] * 10
    assert t.dup[10:15] == [1] * 5     # identical: silently dropped (process_test.go:3931-3939)
    assert t.dup[15] == 2              # different value: CatchDoublePrevote
    assert len(t.dup) == n


def test_non_valid_and_proposes_are_not_candidates(oracle):
    b = oracle.Batch()
    v = oracle.canonical_value(1, 0)
    for k in range(6):
        b.append(oracle.PREVOTE, 1, 0, -1, v, bytes([k]) * 32, bytes(65))
    b.append(oracle.PROPOSE, 1, 0, -1, v, bytes([9]) * 32, bytes(65))
    verdicts = [0, 5, 0, 6, 0, 0, 0]
    t = oracle.tally(b, verdicts)
    assert t.distinct[(1, 0, oracle.PREVOTE)] == 4
    assert t.dup == [0, 3, 0, 3, 0, 0, 3]


DECIDE_BITS = ("timeout_prevote", "precommit_nil", "timeout_precommit_reached", "timeout_precommit_exact", "skip",
               "precommit_value", "commit")


def test_c_oracle_tally_and_decisions(coracle, oracle):
    """The C restatement of the tally and the quorum predicates (the CPU
    baseline's tally leg, oracle/hd_oracle.c oracle_tally) equals the Python
    restatement's rows and hyperdrive_amd.quorum.decide on every golden
    fixture and tally scenario."""
    import numpy as np
    from test_golden import CASES, load_case
    from test_multi_rank import tally_rows
    from util import from_np
    from hyperdrive_amd import quorum
    batches = [(load_case(c)[0], load_case(c)[1]["verdict"]) for c in CASES]
    from tally_cases import scenarios
    from util import to_np
    for sc in scenarios():
        batches.append((to_np(sc.b), np.array([0 if i % 7 else 5 for i in range(len(sc.b))], np.uint8)))
    for b, verdict in batches:
        ob = from_np(b)
        want = tally_rows(ob, verdict.tolist())
        for f in (1, 2, 33):
            pv = lambda h, r: oracle.canonical_value(h, r)
            got = coracle.tally(b, verdict, f, propose_value=pv)
            assert got["counts"].tolist() == want["counts"].tolist()
            assert got["hr"].tolist() == want["hr"].tolist()
            t = oracle.tally(ob, verdict.tolist())
            for (h, r), d in zip(got["hr"][:, :2].tolist(), got["decide"].tolist()):
                ref = quorum.decide(t, h, r, f, pv(h, r), True)
                assert {k: bool(d >> j & 1) for j, k in enumerate(DECIDE_BITS)} == \
                    {k: ref[k] for k in DECIDE_BITS}, (h, r, f)
