"""The host-buffer (cgo) path alone: bench.py's host_buffers (hd_verify_submit /
hd_verify_wait, pinned and pageable host batches), for a rocprofv3
--kernel-trace --memory-copy-trace run."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch

import bench
import hyperdrive_amd as hd


class A:
    batch = 1 << 20
    signers = 100


dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
v = hd.Verifier(0)
sigs, foreign = v.gen_keys(100)
v.set_signatories(sigs)
print(json.dumps(bench.host_buffers(v, A, sigs, foreign, dev)), flush=True)
