#!/usr/bin/env python3
"""Generate tests/golden/c1_stream.npz + c1_expected.json (test data only).

The C1 plumbing config (BASELINE configs[0]: n = 4, f = 1, 100 heights) as one
replica's arrival stream (tests/c1_chain.py make_stream, signed with the
pinned Python restatement's RFC6979 signer), and the flush records the chain
of CPU restatements produces for it (tests/c1_chain.py run_oracle).  The GPU
test (tests/test_c1_network.py) pushes the same stream through
hyperdrive_amd.Ingress and must reproduce the records.

Usage: python tests/golden/make_c1.py   (~15 s, deterministic)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import hd_pyoracle as O  # noqa: E402
from c1_chain import make_stream, run_oracle  # noqa: E402


def main():
    z = make_stream(O)
    np.savez_compressed(os.path.join(HERE, "c1_stream.npz"), **z)
    from conftest import build_coracle
    from oracle_c import COracle
    rep = run_oracle(z, COracle(build_coracle()))
    with open(os.path.join(HERE, "c1_expected.json"), "w") as fh:
        json.dump({"commits": rep.commits, "records": rep.records}, fh, indent=0)
    print(f"{len(z['type'])} messages, {len(rep.commits)} commits, {len(rep.records)} flushes")


if __name__ == "__main__":
    main()
