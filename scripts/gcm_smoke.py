"""One AES-256-GCM message on the device against the oracle (first contact with a new kernel)."""
import sys

sys.path.insert(0, '.')
import torch  # noqa: E402,F401  (the HIP runtime as the tests see it)
from oracle import oracle as o  # noqa: E402
from replicat_amd.cipher import GpuAesGcm  # noqa: E402

g = GpuAesGcm()
k, v, d = bytes(range(32)), bytes(range(12)), bytes(range(200)) * 3
b = g.encrypt_many([d], [k], [v])[0]
want = v + o.gcm_encrypt(k, v, d)
print('got ', b[-20:].hex())
print('want', want[-20:].hex())
assert b == want, 'mismatch'
assert g.decrypt(b, k) == d
print('gcm smoke ok')
