"""dev: instruction mix of one kernel's innermost loop in the gfx950 ISA
(hipcc -S).  Usage: python tools/isa_count.py <kernel-substring> [file.s]
Prints each loop block (label .. back-edge) with its VALU/SALU/LDS counts."""
import collections
import re
import subprocess
import sys

name = sys.argv[1]
path = sys.argv[2] if len(sys.argv) > 2 else "/tmp/sh.s"
if len(sys.argv) <= 2:
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC",
                    "-ffp-contract=off", "-Iinclude", "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
                    "--cuda-device-only", "-S", "-o", path,
                    "mpi-hungarian-method_amd/csrc/santa_hip.hip"], check=True, stderr=subprocess.DEVNULL)
s = open(path).read()
m = re.search(r"^(_Z\S*" + re.escape(name) + r"\S*):", s, re.M)
body = s[m.end():s.index(".Lfunc_end", m.end())].splitlines()


def kind(op):
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
        return "lane"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("v_"):
        return "valu"
    return op


labels = {}
for i, l in enumerate(body):
    if re.match(r"^\.LBB\S+:", l):
        labels[l.split(":")[0]] = i
# loops: the last branch back to a loop header label (the header's comment
# names its depth); counted from the header to that back-edge
heads = {lab: i for lab, i in labels.items()
         if "Loop Header" in " ".join(body[i:i + 5])}
last_back = {}
for i, l in enumerate(body):
    t = l.strip().split()
    if t and t[0].startswith(("s_branch", "s_cbranch")) and t[-1] in heads and heads[t[-1]] < i:
        last_back[t[-1]] = i
for tgt, i in sorted(last_back.items(), key=lambda x: heads[x[0]]):
        depth = re.search(r"Depth=(\d+)", " ".join(body[heads[tgt]:heads[tgt] + 3]))
        if True:
            c = collections.Counter()
            for x in body[labels[tgt]:i + 1]:
                u = x.strip().split()
                if u and not u[0].startswith((".", ";")) and not u[0].endswith(":"):
                    c[kind(u[0])] += 1
            print(f"loop {tgt} depth {depth.group(1) if depth else '?'} lines {labels[tgt]}-{i}: {dict(c)}")
            if tgt in sys.argv[3:]:
                print("\n".join(x for x in body[labels[tgt]:i + 1] if not x.strip().startswith(";")))
