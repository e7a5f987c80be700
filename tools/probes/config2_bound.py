"""Config 2's bound: multi64_kernel over 64 batches of
1M x 64 B (4 GiB), forms and diagnostics interleaved block by block (10
launches back to back between two events per block, 7 blocks, medians), beside
the same-GPU streaming read of the same 4 GiB:
  0            the shipped form (unconditional result stores, lanes past the
               batch's end to a sink word)
  128          round 4's guarded stores (the compiler drained them with
               vmcnt(0) before every other chunk's loads)
  64           unconditional non-temporal result stores
  1<<20        no hashing (diagnostic)
  262144       result stores into one L2-resident window (diagnostic)
(round 5's first probe also had bit 64: no result stores -- 0.609 ms against
0.818 with them, the streaming read 0.618; profiles/r05/config2/bound_probe.jsonl)
usage: python tools/probes/config2_bound.py [opt ...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from zeroskip_amd import device as zd  # noqa: E402
from zeroskip_amd._lib import check, lib  # noqa: E402


def main():
    opts = [int(x) for x in sys.argv[1:]] or [0, 128, 64, 1 << 20, 262144]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(0x64)
    n, rot = 1 << 20, 64
    bufs = torch.randint(0, 256, (rot, n * 64), dtype=torch.uint8, device=dev, generator=g)
    blist = list(bufs)
    outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(rot)]
    st = torch.cuda.current_stream(dev)
    scratch = torch.zeros(4, dtype=torch.int32, device=dev)
    nbytes = bufs.numel()

    def multi():
        zd.crc_fixed_multi(blist, 64, 64, n, outs=outs)

    def sread():
        check(lib().zscrc_diag_stream_read(bufs.data_ptr(), nbytes, scratch.data_ptr(), 1, st.cuda_stream), "read")

    forms = [("opt%d" % o, o, multi) for o in opts] + [("stream_read", 0, sread)]
    ts = {k: [] for k, _, _ in forms}
    ref = None
    for blk in range(8):
        for name, o, fn in forms:
            lib().zscrc_set_opt(o)
            fn()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(10):
                fn()
            b.record(st)
            torch.cuda.synchronize()
            if blk:
                ts[name].append(a.elapsed_time(b) / 10)
            if name == "opt0" and ref is None:
                ref = torch.stack(outs).clone()
            if name == "opt128":
                assert torch.equal(torch.stack(outs), ref), "opt 128 results differ from the shipped form"
    lib().zscrc_set_opt(0)
    for name, _, _ in forms:
        med = sorted(ts[name])[len(ts[name]) // 2]
        print(json.dumps({"form": name, "ms_per_launch": round(med, 4), "us_per_batch": round(med * 1e3 / rot, 3),
                          "GBs": round(nbytes / (med * 1e-3) / 1e9, 1),
                          "frac_of_spec": round(nbytes / (med * 1e-3) / 1e9 / 8000.0, 4),
                          "blocks": [round(t, 4) for t in ts[name]]}), flush=True)


if __name__ == "__main__":
    main()
