"""The diagnostic block-store build keeps storing on every call: the count
of commits written (status 1) over three consecutive in-place writer calls
on config 4's image (with ZSCRC_LIB_PATH=zeroskip_amd/libzscrc_diagblock.so;
tools/probes/block_store_ab.sh)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools import zsdb_gen as zg  # noqa: E402
from zeroskip_amd import zsfile  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(7)
ppf = zg.pairs_per_file(True)
nfiles = -(-10_000_000 // ppf)
img = zg.log_files(bytes(range(16)), 0, nfiles, ppf, 0, True, g, dev).view(-1)
offs, lens = zg.log_spans(nfiles, ppf, True, True, dev)
live = lens > 0
ow, lw = offs[live].contiguous(), lens[live].contiguous()
counts = []
for _ in range(3):
    _, st = zsfile.write_commits(img, ow, lw, max_len=int(lw.max().item()), status=True)
    counts.append(int((st == 1).sum().item()))
print(json.dumps({"lib": os.environ.get("ZSCRC_LIB_PATH", "default"), "commits": int(ow.numel()),
                  "written_per_call": counts}))
