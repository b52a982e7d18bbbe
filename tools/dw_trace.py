"""Direct-write diagnostics: time a C4-like plan with and without direct write, dump one DW launch's
per-subframe s_memrealtime stamps (start, emit, look-back done, end) and summarise them."""
import os, sys, time
sys.path.insert(0, "flac-raster_amd")
import numpy as np
from flac_raster import _native as N
from flac_raster.synth import synth_window
from flac_raster.tiles import calculate_tiles

H = W = int(os.environ.get("DWT_SIZE", "8192"))
r = synth_window(4, 5, 4, H, W).astype(np.uint16)
wins = calculate_tiles(H, W, 1024)
out = os.environ.get("DWT_OUT", "gpurun_out/dw_trace")
os.makedirs(out, exist_ok=True)


def run(dw, trace):
    os.environ["FRA_DW"] = "1" if dw else "0"
    if trace:
        os.environ["FRA_DW_TRACE"] = out + "/trace.bin"
    else:
        os.environ.pop("FRA_DW_TRACE", None)
    plan = N.Plan(N.default_context(0), r.ctypes.data, False, r.dtype, 4, (H * W, W, 1), wins, 5, 4096, 16, 0,
                  keepalive=r)
    try:
        plan.execute(); plan.sync()
        plan.enable_timing(True)
        for _ in range(5):
            plan.execute()
        plan.sync()
        ms, n = plan.timing()
        return [m / n for m in ms], plan.download()[1]
    finally:
        plan.close()


if os.path.exists(out + "/trace.bin"):
    os.remove(out + "/trace.bin")
a, fa = run(False, False)
b, fb = run(True, True)
print("slot ms/phase", [round(x, 3) for x in a])
print("dw   ms/phase", [round(x, 3) for x in b], "bytes equal", fa == fb)
t = np.fromfile(out + "/trace.bin", np.uint64).reshape(-1, 4).astype(np.int64)
t = t[-(len(t) // 1):]
nsf = len(wins) and (len(t))
t0 = t[:, 0].min()
us = (t - t0) / 100.0
ana, crc, lbw, tail = us[:, 1] - us[:, 0], us[:, 2] - us[:, 1], us[:, 2] - us[:, 1], us[:, 3] - us[:, 2]
print("subframes", len(t), "span us", us[:, 2].max())
for name, v in [("analysis", us[:, 1] - us[:, 0]), ("emit->P", us[:, 2] - us[:, 1]), ("P->end(last ch)", tail[t[:, 3] > 0])]:
    print(name, "p10/50/90/99/max", np.percentile(v, [10, 50, 90, 99]).round(1), v.max().round(1))
# waiting WGs over time
ts = np.linspace(0, us[:, 2].max(), 40)
for x in ts[::4]:
    run_ = ((us[:, 0] <= x) & (us[:, 2] > x)).sum()
    wait = ((us[:, 1] <= x) & (us[:, 2] > x)).sum()
    print(f"t {x:8.1f} us resident {run_:5d} in look-back {wait:5d}")
