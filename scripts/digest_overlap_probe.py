"""Device-side steady state of the snapshot producer's per-batch work.

A batch's device work is: upload (pinned H2D) -> cut chain (rc_chunk_device, OPEN prefix) ->
chunk digests (rc_blake2b_chunks).  The digests of a batch end with the serial BLAKE2b chain
of its longest chunk (~40,000 blocks for a 5.12 MB chunk, ~55 ms) whatever the
batch size, so one batch at a time caps the device near batch / 55 ms.  The producer now keeps
`slots` batches in flight, each on its own HIP stream with its own digest handle; this probe
measures what that buys without the host's file reads in the way: NB batches of 1 GiB of
distinct synthetic bytes (splitmix64, generated in HBM), queued round-robin on S streams, with
and without the H2D upload of each batch from a pinned host buffer.  Digests of the first batch
are checked against hashlib.

    python scripts/digest_overlap_probe.py [--batches 8] [--slots 1,2,3,4] [--queues torch|own]

--queues own: each slot's stream has a hardware queue of its own (replicat_amd.chunker.QueueStream,
rc_stream_create) instead of a torch stream on the process's shared GPU_MAX_HW_QUEUES queues.
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, QueueStream, fill_splitmix  # noqa: E402
from replicat_amd.hashing import SLOT, GpuBlake2b  # noqa: E402

GIB = 1 << 30
MIN_LEN, MAX_LEN = 128_000, 5_120_000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batches', type=int, default=8)
    ap.add_argument('--batch-mib', type=int, default=1024)
    ap.add_argument('--slots', default='1,2,3,4')
    ap.add_argument('--queues', choices=['torch', 'own'], default='torch')
    args = ap.parse_args()
    torch.cuda.set_device(0)
    size = args.batch_mib << 20
    nb = args.batches
    dev = [torch.empty(size + 64, dtype=torch.uint8, device='cuda') for _ in range(nb)]
    hs0 = torch.cuda.current_stream().cuda_stream
    for i, t in enumerate(dev):
        fill_splitmix(t.data_ptr(), size, synth.DEFAULT_SEED, 1000 + i, hs0)
    pinned = torch.empty(size, dtype=torch.uint8, pin_memory=True)
    pinned.copy_(dev[0][:size].cpu())
    ch = GpuChunker(MIN_LEN, MAX_LEN, b'\xff' * 16)
    cap, _ = ch.capacity([size])
    smax = max(int(s) for s in args.slots.split(','))
    owned = [QueueStream.acquire() for _ in range(smax)] if args.queues == 'own' else []
    streams = [q.torch for q in owned] if owned else [torch.cuda.Stream() for _ in range(smax)]
    torch.cuda.set_stream(torch.cuda.Stream())  # keep the legacy NULL stream out of it
    hashers = [GpuBlake2b(length=64) for _ in range(smax)]
    cuts = [torch.zeros(cap, dtype=torch.int64, device='cuda') for _ in range(nb)]
    counts = [torch.zeros(1, dtype=torch.int64, device='cuda') for _ in range(nb)]
    digs = [torch.zeros((cap, SLOT), dtype=torch.uint8, device='cuda') for _ in range(nb)]
    staging = [torch.empty(size + 64, dtype=torch.uint8, device='cuda') for _ in range(smax)]
    torch.cuda.synchronize()

    def run(S, upload):
        t0 = time.perf_counter()
        for b in range(nb):
            k = b % S
            st = streams[k]
            with torch.cuda.stream(st):
                if upload:
                    # the slot's device copy is reused every S batches (stream order protects it)
                    buf = staging[k]
                    buf[:size].copy_(pinned, non_blocking=True)
                else:
                    buf = dev[b]
                ch.chunk_device([buf.data_ptr()], [size], [size], cuts[b].data_ptr(),
                                counts[b].data_ptr(), st.cuda_stream, open_=True)
                hashers[k].digest_chunks(ch, [buf.data_ptr()], [size], cuts[b].data_ptr(),
                                         counts[b].data_ptr(), digs[b].data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    # parity: batch 0's chunk digests against hashlib
    run(1, False)
    n0 = int(counts[0].item())
    ends = cuts[0][:n0].cpu().numpy()
    host = dev[0][:size].cpu().numpy()
    prev, ok = 0, True
    d0 = digs[0][:n0, :64].cpu().numpy()
    for i, e in enumerate(ends.tolist()):
        ok &= hashlib.blake2b(host[prev:e].tobytes()).digest() == d0[i].tobytes()
        prev = e
    print(json.dumps({'check': 'batch 0 digests vs hashlib', 'chunks': n0, 'ok': bool(ok),
                      'longest_chunk': int(np.diff(np.concatenate([[0], ends])).max())}),
          flush=True)
    if not ok:
        sys.exit(1)
    for upload in (False, True):
        for S in [int(s) for s in args.slots.split(',')]:
            run(S, upload)  # warm
            dt = min(run(S, upload) for _ in range(2))
            print(json.dumps({'slots': S, 'queues': args.queues,
                              'GPU_MAX_HW_QUEUES': os.environ.get('GPU_MAX_HW_QUEUES'),
                              'upload_from_pinned': upload, 'batches': nb,
                              'batch_bytes': size, 's': round(dt, 4),
                              'gib_s': round(nb * size / dt / GIB, 2),
                              'ms_per_batch': round(dt * 1e3 / nb, 2)}), flush=True)


if __name__ == '__main__':
    main()
