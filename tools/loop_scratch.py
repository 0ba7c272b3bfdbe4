"""Scratch (spill) instructions inside the MFMA loops of a kernel (dev aid).

python tools/loop_scratch.py LIB.so KERNEL_SUBSTRING
Disassembles the gfx950 code object of LIB.so and, for every backward branch
of the kernel, prints the loop's MFMA and scratch instruction counts: spills
inside a tile loop force vmcnt(0) waits behind the tile's stores."""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"
lib, name = sys.argv[1], sys.argv[2]
with tempfile.TemporaryDirectory() as d:
    subprocess.run([f"{B}/llvm-objcopy", f"--dump-section=.hip_fatbin={d}/f.bin", lib], check=True)
    subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={d}/f.bin",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={d}/k.co"], check=True)
    dis = subprocess.run([f"{B}/llvm-objdump", "-d", f"{d}/k.co"], check=True,
                         capture_output=True, text=True).stdout.split("\n")
starts = [i for i, l in enumerate(dis) if name in l and l.endswith(">:")]
for s in starts:
    e = s + 1
    while e < len(dis) and not re.match(r"^[0-9a-f]+ <", dis[e]):
        e += 1
    f = dis[s:e]
    addr = {}
    for i, l in enumerate(f):
        m = re.search(r"// ([0-9A-F]+):", l)
        if m:
            addr[int(m.group(1), 16)] = i
    loops = []
    for i, l in enumerate(f):
        m = re.search(r"s_c?branch\w*\s+(\d+)\s+// ([0-9A-F]+):", l)
        if m:
            off = int(m.group(1))
            off = off - 65536 if off >= 32768 else off
            tgt = addr.get(int(m.group(2), 16) + 4 + 4 * off)
            if tgt is not None and tgt < i:
                seg = f[tgt:i + 1]
                loops.append((tgt, i, sum("v_mfma" in x for x in seg), sum("scratch_" in x for x in seg)))
    print(f[0][:90])
    print("  scratch total", sum("scratch_" in x for x in f), "| loops with MFMAs (start, end, mfma, scratch):")
    for lp in loops:
        if lp[2]:
            print("   ", lp)
