#!/usr/bin/env python
"""Debug (measurement only): run the large host-read fuzz cases in one process
and, when a read fails, compare every staged piece on the device with its
host bytes (which pieces arrived wrong, and whether they were DMA'd directly)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zarr-python_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import tempfile

    import torch

    from zarr_hip import staging
    from zarr_hip.store import FileRef
    import test_gpu_fuzz as F

    rec = []
    orig = staging.stage

    def stage(layout, device, post=(), defer=False):
        r = orig(layout, device, post, defer)
        rec.append((list(layout.pieces), r[0], staging.pinned_spans()))
        return r
    staging.stage = stage
    dev = torch.device("cuda:0")
    for rep in range(int(os.environ.get("REPS", "3"))):
        for seed in range(8):
            rec.clear()
            try:
                F.test_random_host_reads_large(dev, tempfile.mkdtemp(), seed)
            except (ValueError, AssertionError) as e:
                torch.cuda.synchronize()
                print("rep", rep, "seed", seed, "FAIL", type(e).__name__, str(e)[:80], flush=True)
                for pieces, dbuf, spans in rec[-6:]:
                    got = dbuf.cpu().numpy()
                    bad = []
                    for buf, off, n in pieces:
                        if isinstance(buf, FileRef):
                            continue
                        v = staging._host_view(buf)
                        if got[off: off + n].tobytes() != v.tobytes():
                            a = v.ctypes.data
                            pinned = any(lo <= a and a + n <= hi for lo, hi in spans)
                            d = np.nonzero(got[off: off + n] != v)[0]
                            bad.append((off, n, pinned, int(d[0]), int(d[-1]), len(d)))
                    print("   stage: pieces", len(pieces), "bad", bad[:5], flush=True)
    print("done", flush=True)


if __name__ == "__main__":
    main()
