#!/usr/bin/env python3
"""Code-object statistics of the gfx950 kernels in an object or shared library.

For each kernel symbol: code bytes (ELF symbol size), and from the disassembly the static counts of
v_writelane_b32 / v_readlane_b32 (SGPR spill traffic into VGPR lanes), s_nop and s_waitcnt, plus the
VGPR / SGPR / LDS / spill numbers the compiler reports in the code object's metadata notes.

    python tools/codeobj_stats.py flac-raster_amd/flac_raster/_lib/libflac_raster_amd.so [name-filter]

Used to put code_bytes / vgpr / sgpr_spill of the dominant kernel on the bench line (bench.py) and to
check codegen changes on the CPU before any GPU run.
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def _device_objects(path: str, tmp: str) -> list[str]:
    """Unbundle the gfx950 code object(s) of an object file or shared library."""
    fat = os.path.join(tmp, "fat.bin")
    r = subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", path, os.path.join(tmp, "x.o")],
                       capture_output=True, text=True)
    if r.returncode != 0 or not os.path.exists(fat):
        raise RuntimeError(f"no .hip_fatbin in {path}: {r.stderr.strip()}")
    # a shared library's fatbin holds one bundle per linked object; the bundler takes the first, so
    # split on the bundle magic and unbundle each
    data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    outs = []
    for i, s in enumerate(starts):
        e = starts[i + 1] if i + 1 < len(starts) else len(data)
        part = os.path.join(tmp, f"b{i}.bin")
        with open(part, "wb") as f:
            f.write(data[s:e])
        co = os.path.join(tmp, f"b{i}.co")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                           capture_output=True, text=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            outs.append(co)
    return outs


def _metadata(co: str) -> dict[str, dict]:
    """Kernel records of the code object's metadata note (each kernel map starts at .agpr_count: the keys
    are sorted)."""
    r = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True)
    recs: list[dict] = []
    for line in r.stdout.splitlines():
        s = line.strip()
        if s.startswith("- .agpr_count"):
            recs.append({})
        if not recs:
            continue
        for key in ("name", "sgpr_count", "vgpr_count", "sgpr_spill_count", "vgpr_spill_count",
                    "group_segment_fixed_size", "private_segment_fixed_size"):
            m = re.match(rf"-?\s*\.{key}:\s+(\S+)$", s)
            if m and key not in recs[-1]:
                v = m.group(1)
                recs[-1][key] = v if key == "name" else int(v)
    return {r["name"]: r for r in recs if "name" in r}


def stats(path: str, filt: str = "") -> list[dict]:
    res = []
    with tempfile.TemporaryDirectory() as tmp:
        for co in _device_objects(path, tmp):
            meta = _metadata(co)
            sym = subprocess.run([f"{LLVM}/llvm-readelf", "-sW", co], capture_output=True, text=True).stdout
            sizes = {}
            for line in sym.splitlines():
                p = line.split()
                if len(p) >= 8 and p[3] == "FUNC":
                    sizes[p[7]] = int(p[2], 0) if p[2].startswith("0x") else int(p[2])
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                                 text=True).stdout
            counts: dict[str, dict[str, int]] = {}
            cur = None
            for line in dis.splitlines():
                m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
                if m:
                    cur = m.group(1)
                    counts[cur] = {"insts": 0, "writelane": 0, "readlane": 0, "s_nop": 0, "s_waitcnt": 0}
                    continue
                if cur is None or not line.startswith("\t"):
                    continue
                op = line.strip().split(" ")[0]
                c = counts[cur]
                c["insts"] += 1
                if op == "v_writelane_b32":
                    c["writelane"] += 1
                elif op == "v_readlane_b32":
                    c["readlane"] += 1
                elif op == "s_nop":
                    c["s_nop"] += 1
                elif op.startswith("s_waitcnt"):
                    c["s_waitcnt"] += 1
            for name, sz in sizes.items():
                if filt and filt not in name:
                    continue
                if name not in meta and name not in counts:
                    continue
                md = meta.get(name, {})
                row = {"kernel": name, "code_bytes": sz, "vgpr": md.get("vgpr_count"), "sgpr": md.get("sgpr_count"),
                       "sgpr_spill": md.get("sgpr_spill_count"), "vgpr_spill": md.get("vgpr_spill_count"),
                       "lds": md.get("group_segment_fixed_size"), "scratch": md.get("private_segment_fixed_size")}
                row.update(counts.get(name, {}))
                res.append(row)
    return res


def main() -> None:
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = stats(path, filt)
    if "--json" in sys.argv:
        print(json.dumps(rows))
        return
    hdr = ["kernel", "code_bytes", "vgpr", "sgpr", "sgpr_spill", "vgpr_spill", "lds", "scratch", "insts",
           "writelane", "readlane", "s_nop", "s_waitcnt"]
    print("\t".join(hdr))
    for r in sorted(rows, key=lambda r: -r["code_bytes"]):
        print("\t".join(str(r.get(h)) for h in hdr))


if __name__ == "__main__":
    main()
