#!/usr/bin/env python3
"""PCIe probe at C5 band sizes (GPU box): one host band of raster in (2 GiB, page-locked) and one band of frames
out (1.4 GB, page-locked or pageable), alone and at once -- whole copies or interleaved chunks, the pageable D2H
from its own thread (as fra_plan_encode_ring's D2H worker).  Tells what the ring path's per-band floor is.
torch is used here only as plumbing for streams and page-locked tensors."""
import json
import sys
import threading
import time

import torch


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / reps * 1e3, 2)


def main():
    nin, nout = 2 << 30, 1_400_000_000
    chunk = int(sys.argv[1]) << 20 if len(sys.argv) > 1 else 64 << 20
    hin = torch.empty(nin, dtype=torch.uint8).pin_memory()
    hout = torch.empty(nout, dtype=torch.uint8).pin_memory()
    pout = torch.empty(nout, dtype=torch.uint8)  # pageable
    pout.fill_(1)
    din = torch.empty(nin, dtype=torch.uint8, device="cuda")
    dout = torch.empty(nout, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def h2d(ch=0):
        with torch.cuda.stream(s1):
            if not ch:
                din.copy_(hin, non_blocking=True)
            else:
                for a in range(0, nin, ch):
                    din[a:a + ch].copy_(hin[a:a + ch], non_blocking=True)

    def d2h(dst, ch=0):
        with torch.cuda.stream(s2):
            if not ch:
                dst.copy_(dout, non_blocking=True)
            else:
                for a in range(0, nout, ch):
                    dst[a:a + ch].copy_(dout[a:a + ch], non_blocking=True)
        s2.synchronize()

    def both(dst, ch=0, thread=False):
        if thread:
            t = threading.Thread(target=d2h, args=(dst, ch))
            t.start()
            h2d(ch)
            t.join()
        elif ch:  # interleaved issue order
            for a in range(0, max(nin, nout), ch):
                with torch.cuda.stream(s1):
                    if a < nin:
                        din[a:a + ch].copy_(hin[a:a + ch], non_blocking=True)
                with torch.cuda.stream(s2):
                    if a < nout:
                        dst[a:a + ch].copy_(dout[a:a + ch], non_blocking=True)
        else:
            h2d()
            d2h(dst)

    r = {"chunk_MiB": chunk >> 20,
         "h2d_ms": timed(h2d), "h2d_chunked_ms": timed(lambda: h2d(chunk)),
         "d2h_pinned_ms": timed(lambda: d2h(hout)), "d2h_pageable_ms": timed(lambda: d2h(pout)),
         "d2h_pageable_chunked_ms": timed(lambda: d2h(pout, chunk)),
         "both_pinned_ms": timed(lambda: both(hout)), "both_pinned_chunked_ms": timed(lambda: both(hout, chunk)),
         "both_pinned_thread_ms": timed(lambda: both(hout, 0, True)),
         "both_pageable_thread_ms": timed(lambda: both(pout, 0, True)),
         "both_pageable_thread_chunked_ms": timed(lambda: both(pout, chunk, True))}
    r["h2d_GBps"] = round(nin / r["h2d_ms"] / 1e6, 1)
    r["d2h_pinned_GBps"] = round(nout / r["d2h_pinned_ms"] / 1e6, 1)
    r["d2h_pageable_GBps"] = round(nout / r["d2h_pageable_ms"] / 1e6, 1)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
