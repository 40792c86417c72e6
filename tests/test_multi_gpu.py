"""The C-ABI multi-GPU path (include/hd_verify.h hd_multi_*,
hyperdrive_amd/multi.py) against the single-context path on the same batches:
verdicts, recovered signatories, the valid bitmap and the merged partitioned
tally are identical.  On a one-GPU box the device list [0] runs the RCCL
exchange (one rank) and [0, 0] / [0, 0, 0] run the copy exchange between
contexts sharing the GPU; an 8-GPU node runs the same code with one rank per
device."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same(a, b):
    ra, ta = a
    rb, tb = b
    assert ra.verdict.tolist() == rb.verdict.tolist()
    assert ra.recovered.tobytes() == rb.recovered.tobytes()
    assert ra.valid_bitmap.tolist() == rb.valid_bitmap.tolist()
    assert ta.count == tb.count and ta.distinct == tb.distinct and ta.distinct_any == tb.distinct_any
    assert ta.dup.tolist() == tb.dup.tolist()


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("kind,n,S,adv", [(0, 65536 + 17, 100, 30), (1, 128064, 1000, 10), (0, 37, 7, 50)])
def test_multi_equals_single(gpu, devices, kind, n, S, adv):
    from hyperdrive_amd.device import generate
    from hyperdrive_amd.multi import MultiVerifier
    v = gpu.Verifier(0)
    ks = v.gen_keys(S)
    v.set_signatories(ks[0])
    db, _, _ = generate(v, kind, n, S, adv, keys=ks)
    hb = db.to_host()
    single = v.process_batch(hb)
    m = MultiVerifier(devices)
    try:
        assert m.uses_rccl == (len(set(devices)) == len(devices))
        m.set_signatories(ks[0])
        for rnd in range(2):                   # pass 2: the per-device known-key tables
            _same(m.process_batch(hb), single)
        assert m.fastpath_stats(0)[0] > 0
    finally:
        m.close()
        v.close()


def test_multi_empty_and_errors(gpu):
    from hyperdrive_amd import _lib
    from hyperdrive_amd.multi import MultiVerifier
    from hyperdrive_amd.verify import Batch
    with pytest.raises(_lib.HDError):
        MultiVerifier([99])
    m = MultiVerifier([0, 0])
    e = Batch(np.zeros(0, np.uint8), np.zeros(0, np.int64), np.zeros(0, np.int64), None,
              np.zeros((0, 32), np.uint8), np.zeros((0, 32), np.uint8), np.zeros((0, 65), np.uint8))
    res, tal = m.process_batch(e)
    assert len(res.verdict) == 0 and tal.count == {}
    m.close()
