"""A per-key table allocation the device cannot serve: one context holds the
100-signatory 22-bit tables (~177 GB), a second is forced to the same width
(HD_VAR_KEY_WIDTH 22) and must fail its set change with HD_ENOMEM and no
crash; unforced, the same context then picks a width that fits and verifies
the batch identically to the first.  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch  # noqa: F401  (before the library: torch brings its own HIP runtime)

import hyperdrive_amd as hd
from hyperdrive_amd import _lib
from hyperdrive_amd.device import generate

v1 = hd.Verifier(0)
ks = v1.gen_keys(100)
v1.set_signatories(ks[0])
db, _, _ = generate(v1, 0, 4096 + 7, 100, 20, keys=ks)
hb = db.to_host()
r1, t1 = v1.process_batch(hb)
v2 = hd.Verifier(0)
v2.set_variant("key_width", 22)
err = None
try:
    v2.set_signatories(ks[0])
except _lib.HDError as e:
    err = str(e)
v2.set_variant("key_width", 0)
v2.set_signatories(ks[0])
out = []
for _ in range(2):
    r2, t2 = v2.process_batch(hb)
    out.append(r2.verdict.tolist() == r1.verdict.tolist() and r2.recovered.tobytes() == r1.recovered.tobytes()
               and t2.count == t1.count)
print(json.dumps({"forced_error": err, "geometry_v1": v1.fastpath_geometry(), "geometry_v2": v2.fastpath_geometry(),
                  "equal": out, "valid": int((r1.verdict == 0).sum())}), flush=True)
v2.close()
v1.close()
