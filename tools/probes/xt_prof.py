"""One fixed-stride case, 5 launches (rocprofv3 --pmc target).
usage: python tools/probes/xt_prof.py LEN N [XTEAM_MODE]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from zeroskip_amd._lib import check, lib  # noqa: E402

L, n = int(sys.argv[1]), int(sys.argv[2])
mode = int(sys.argv[3]) if len(sys.argv) > 3 else 1
lib().zscrc_set_xteam(mode, 4096)
dev = torch.device("cuda", 0)
big = torch.randint(0, 256, (4 << 30,), dtype=torch.uint8, device=dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream()
for _ in range(5):
    check(lib().zscrc_device_fixed(big.data_ptr(), L, L, 0, out.data_ptr(), n, 0, st.cuda_stream), "fixed")
torch.cuda.synchronize()
