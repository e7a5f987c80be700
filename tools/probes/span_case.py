"""A 3 GiB span, 10 passes after a marker dispatch (rocprofv3 target)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from zeroskip_amd import device as zd  # noqa: E402

dev = torch.device("cuda:0")
big = torch.randint(0, 256, (3 << 30,), dtype=torch.uint8, device=dev)
for _ in range(3):
    zd.crc_span(big)
torch.cuda.synchronize()
for _ in range(10):
    zd.crc_span(big)
torch.cuda.synchronize()
