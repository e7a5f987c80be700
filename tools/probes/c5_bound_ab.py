"""Config-5 A/B: consistent.run() with and without the walk's span bound
(diagnostic)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tools import zsdb_gen as zg  # noqa: E402
from zeroskip_amd import consistent as cs  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402

dev = torch.device("cuda:0")
db = zg.make_db(device=dev)
job = cs.Consistent(cs.open_db(db), 0, 1)
job.prepare()
cl = job.c_len
print("commits", len(cl), "max", int(cl.max()), "n>640", int((cl > 640).sum()), "pieces", len(job.pieces),
      "top", np.sort(cl)[-5:].tolist(), flush=True)
be = job.backend


def timed(tag):
    for _ in range(3):
        job.run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        job.run(events=(a, b))
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    print(tag, "kernel_ms median", round(sorted(ts)[5], 4), flush=True)


timed("bounded")
orig = be.verify
be.verify = lambda buf, off, ln, seed=None, max_len=None: zsfile.verify_commits(buf, off, ln, seed)
timed("unbounded")
