"""CompactBatch.from_batch (hyperdrive_amd/verify.py), the host side of
hd_verify_submit_compact: every From becomes the index of its first row in the
signatory array, or an escape row numbered after the array (each distinct
outsider once); every value an index into the batch's dictionary.  Expanding
the indices gives back the batch exactly (the device's k_compact_expand does
the same gather, tests/test_host_pipeline.py checks it on the GPU)."""
import numpy as np
import pytest

from hyperdrive_amd.verify import Batch, CompactBatch


def _batch(rng, n, frm, values):
    return Batch(rng.integers(2, 4, n).astype(np.uint8), rng.integers(0, 1 << 40, n), rng.integers(0, 9, n), None,
                 values, frm, rng.integers(0, 256, (n, 65), dtype=np.uint8))


def test_indices_expand_to_the_batch():
    rng = np.random.default_rng(3)
    sig = rng.integers(0, 256, (40, 32), dtype=np.uint8)
    sig[17] = sig[5]                                   # a repeated signatory: its first row is used
    outsiders = rng.integers(0, 256, (6, 32), dtype=np.uint8)
    n = 5000
    frm = np.where(rng.random((n, 1)) < 0.9, sig[rng.integers(0, 40, n)], outsiders[rng.integers(0, 6, n)])
    vals = rng.integers(0, 256, (300, 32), dtype=np.uint8)[rng.integers(0, 300, n)]
    b = _batch(rng, n, np.ascontiguousarray(frm), vals)
    c = CompactBatch.from_batch(b, sig)
    table = np.concatenate([sig, c.escape])
    assert (table[c.from_idx] == b.frm).all()
    assert (c.values[c.value_idx] == b.value).all()
    assert c.from_idx.dtype == np.uint16 and c.value_idx.dtype == np.uint16
    assert not (c.from_idx == 17).any()                # the repeat maps to row 5
    assert len(c.escape) == len({x.tobytes() for x in frm if x.tobytes() not in {s.tobytes() for s in sig}})
    assert len(np.unique(c.escape, axis=0)) == len(c.escape)
    assert len(c.values) == len(np.unique(vals, axis=0))
    assert (c.from_idx[(frm == sig[5]).all(1)] == 5).all()
    assert (c.sig == b.sig).all() and (c.height == b.height).all()


def test_limits_and_edges():
    rng = np.random.default_rng(4)
    sig = rng.integers(0, 256, (3, 32), dtype=np.uint8)
    b = _batch(rng, 0, np.zeros((0, 32), np.uint8), np.zeros((0, 32), np.uint8))
    c = CompactBatch.from_batch(b, sig)
    assert len(c) == 0 and len(c.escape) == 0
    n = 70000                                          # more distinct values than 16 bits can index
    frm = sig[rng.integers(0, 3, n)]
    vals = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    with pytest.raises(ValueError):
        CompactBatch.from_batch(_batch(rng, n, frm, vals), sig)
