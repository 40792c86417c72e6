"""hyperdrive_amd -- MI355X-native batch authentication + 2f+1 tally for
hyperdrive consensus messages (tuanggolt/hyperdrive's data-parallel hot path).

The compute lives in ``_lib/libhdverify.so`` (HIP, gfx950) behind the C ABI of
``include/hd_verify.h``; this package is its host-side face.
"""
from .verify import (BAD_RECID, BAD_RS, BAD_TYPE, INFINITY, NO_POINT, NOT_ADMITTED, NOT_AUTHENTIC,
                     SIGNATORY_MISMATCH, VALID, Batch, TallyResult, Verifier, VerifyResult, probe_valu)

__all__ = ["Batch", "Verifier", "VerifyResult", "TallyResult", "probe_valu", "VALID", "BAD_RECID", "BAD_RS",
           "NO_POINT", "INFINITY", "SIGNATORY_MISMATCH", "NOT_ADMITTED", "BAD_TYPE", "NOT_AUTHENTIC"]
