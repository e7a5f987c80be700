"""One 3 GiB record as a variable batch (the split-plan path), 10 passes
(rocprofv3 target)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from zeroskip_amd import device as zd  # noqa: E402

dev = torch.device("cuda:0")
big = torch.randint(0, 256, (3 << 30,), dtype=torch.uint8, device=dev)
offs = torch.zeros(1, dtype=torch.int64, device=dev)
lens = torch.full((1,), (3 << 30) - 77, dtype=torch.int64, device=dev)
for _ in range(13):
    zd.crc_batch(big, offs, lens)
torch.cuda.synchronize()
