#!/usr/bin/env python3
"""Code bytes per source line / phase of one kernel: build the file with -gline-tables-only first.
usage: code_lines.py <obj.o> [top]"""
import collections, os, re, subprocess, sys, tempfile
LLVM = "/opt/rocm/lib/llvm/bin"
obj, top = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40
with tempfile.TemporaryDirectory() as t:
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={t}/f.bin", obj, f"{t}/x.o"], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={t}/f.bin",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={t}/g.co"], check=True)
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "-l", f"{t}/g.co"], capture_output=True, text=True).stdout
cur = None
by = collections.Counter()
for line in dis.splitlines():
    m = re.match(r"; (/\S+):(\d+)", line)
    if m:
        cur = (os.path.basename(m.group(1)), int(m.group(2)))
        continue
    m = re.search(r"// ([0-9A-F]{12}): ((?:[0-9A-F]{8} ?)+)", line)
    if m and cur:
        by[cur] += len(m.group(2).split()) * 4
print("total", sum(by.values()))
for (f, l), b in sorted(by.items(), key=lambda x: -x[1])[:top]:
    print(f"{f}:{l}\t{b}")
