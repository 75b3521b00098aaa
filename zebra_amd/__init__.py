"""zebra_amd -- MI355X-native batch Groth16 verifier (BLS12-381) for Zebra's Sapling
spend/output and Sprout-Groth16 JoinSplit proof checks.

The product is the HIP library ``zebra_amd/libzg.so`` behind the C ABI ``include/zg.h``;
``zebra_amd.zg`` is its ctypes binding. See DESIGN.md and INTEGRATION.md.
"""
from .zg import (Context, ZgError, KIND_SPEND, KIND_OUTPUT, KIND_SPROUT, KIND_NINPUTS, STATUS_OK,  # noqa: F401
                 STATUS_DECODE_INVALID, STATUS_MALFORMED_VK, STATUS_VERIFY_FAILED, STATUS_INPUT_NONCANONICAL,
                 STATUS_NAMES, pack_inputs, prep_spend, prep_output, prep_joinsplit, hsig, PrepError)
