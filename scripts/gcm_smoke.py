"""One AES-256-GCM message on the device against the oracle (first contact with a new kernel).
Each step is stamped, and a hang dumps every thread's stack (faulthandler) before the limit."""
import faulthandler
import os
import sys
import time

faulthandler.dump_traceback_later(25, repeat=True)
T0 = time.time()


def stamp(msg):
    print(f'[{time.time() - T0:7.2f}] {msg}', flush=True)


sys.path.insert(0, '.')
if os.environ.get('NO_TORCH') != '1':
    stamp('import torch')
    import torch  # noqa: E402,F401  (the HIP runtime as the tests see it)
stamp('import oracle')
from oracle import oracle as o  # noqa: E402
stamp('import cipher')
from replicat_amd.cipher import GpuAesGcm  # noqa: E402

g = GpuAesGcm()
stamp('handle')
g.handle()
k, v, d = bytes(range(32)), bytes(range(12)), bytes(range(200)) * 3
stamp('encrypt')
b = g.encrypt_many([d], [k], [v])[0]
stamp('oracle')
want = v + o.gcm_encrypt(k, v, d)
print('got ', b[-20:].hex())
print('want', want[-20:].hex())
assert b == want, 'mismatch'
stamp('decrypt')
assert g.decrypt(b, k) == d
stamp('gcm smoke ok')
