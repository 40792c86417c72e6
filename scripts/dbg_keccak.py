import sys, hashlib
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/oracle"); sys.path.insert(0, "/root/repo/tests")
import numpy as np
import torch; torch.cuda.init()
import keccak_oracle as K
from hyperdrive_amd.verify import Verifier
from hyperdrive_amd.device import DeviceBatch
from hyperdrive_amd.digest import digest_device
from test_keccak import _rand_batch
v = Verifier(0)
for algo in (1, 2):
    b = _rand_batch(np.random.default_rng(11), 3001)
    d = digest_device(v, algo, DeviceBatch.from_host(b)).cpu().numpy()
    want = {}
    bad_valid = bad_invalid = 0
    ex = []
    for i in range(len(b)):
        t = int(b.type[i])
        if t in (1, 2, 3):
            pre = K.preimage(t, int(b.height[i]), int(b.round[i]), int(b.valid_round[i]), b.value[i].tobytes())
            w = K.sponge256(pre, 1 if algo == 1 else 6)
            want[w] = i
            if d[i].tobytes() != w:
                bad_valid += 1
                if len(ex) < 5: ex.append(("valid", i, t))
        elif d[i].any():
            bad_invalid += 1
            if len(ex) < 5: ex.append(("invalid", i, t))
    # do invalid digests match any valid message's digest?
    matches = [want.get(d[i].tobytes()) for i in range(len(b)) if int(b.type[i]) not in (1, 2, 3) and d[i].any()][:10]
    print(algo, "bad_valid", bad_valid, "bad_invalid", bad_invalid, ex, "matches", matches)
    print("types around", [int(x) for x in b.type[:20]])
