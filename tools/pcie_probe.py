#!/usr/bin/env python3
"""PCIe probe (GPU box): H2D alone, D2H alone, and both at once on two streams, page-locked buffers of the
C4 e2e sizes (964 MB raster in, 639 MB frames out).  Tells whether the two copy directions overlap
(full duplex) under the current DMA configuration (run once with HSA_ENABLE_SDMA=0 to compare blit
kernels).  torch is used here only as plumbing for streams and page-locked tensors."""
import json
import os
import time

import torch


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    nin, nout = 964_483_200, 638_528_270
    hin = torch.empty(nin, dtype=torch.uint8).pin_memory()
    hout = torch.empty(nout, dtype=torch.uint8).pin_memory()
    din = torch.empty(nin, dtype=torch.uint8, device="cuda")
    dout = torch.empty(nout, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def h2d():
        with torch.cuda.stream(s1):
            din.copy_(hin, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            hout.copy_(dout, non_blocking=True)

    def both():
        h2d()
        d2h()

    def chunked_both(nb=11):
        for b in range(nb):
            a0, a1 = nin * b // nb, nin * (b + 1) // nb
            o0, o1 = nout * b // nb, nout * (b + 1) // nb
            with torch.cuda.stream(s1):
                din[a0:a1].copy_(hin[a0:a1], non_blocking=True)
            with torch.cuda.stream(s2):
                hout[o0:o1].copy_(dout[o0:o1], non_blocking=True)

    r = {"sdma": os.environ.get("HSA_ENABLE_SDMA", "default"), "h2d_ms": timed(h2d), "d2h_ms": timed(d2h),
         "both_ms": timed(both), "chunked_both_ms": timed(chunked_both)}
    r["h2d_GBps"] = round(nin / r["h2d_ms"] / 1e6, 1)
    r["d2h_GBps"] = round(nout / r["d2h_ms"] / 1e6, 1)
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
