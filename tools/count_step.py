"""Static instruction mix of a kernel's innermost Dijkstra-step loop (dev tool).
usage: python tools/count_step.py <kernel-substring> [--dump]"""
import subprocess, sys
src = "mpi-hungarian-method_amd/csrc/santa_hip.hip"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                "-Iinclude"] + [x for x in __import__("os").environ.get("SH_DEFS","").split() if x] + ["--cuda-device-only", "-S", "-o", "/tmp/sh.s", src], check=True,
               stderr=subprocess.DEVNULL)
s = open("/tmp/sh.s").read()
name = sys.argv[1]
a = s.index(name)
b = s.index(".Lfunc_end", a)
body = s[a:b].splitlines()
dpp = [i for i, l in enumerate(body) if "v_min_u32_dpp" in l]
# the innermost step loop: a v_min_u32_dpp inside a block annotated as a depth-2 loop
def in_depth2(i):
    for j in range(i, -1, -1):
        if body[j].startswith((".LBB", "; %bb")):
            return "Depth=2" in body[j] or "Depth=2" in body[j + 1]
    return False
idx = [i for i in dpp if in_depth2(i)][0]
hdr = max(i for i in range(idx) if "Loop Header: Depth=2" in body[i])
lab = body[hdr - 1].split(":")[0] if body[hdr - 1].startswith(".LBB") else body[hdr].split(":")[0]
tag = lab.lstrip(".L")  # e.g. BB5_246
# basic blocks of the loop: the header, blocks annotated "in Loop: Header=<tag>" and
# child-loop blocks ("Parent Loop <tag>") -- the loop may be rotated above its header
blocks, curb = [], None
for i, l in enumerate(body):
    if l.startswith((".LBB", "; %bb")):
        curb = [l, []]
        blocks.append(curb)
    if curb is not None:
        curb[1].append(l)
seg = []
for head, lines in blocks:
    text = "\n".join(lines[:3])
    if head.startswith(lab + ":") or f"Header={tag} Depth=2" in text or f"Parent Loop {tag} " in text:
        seg.extend(lines)
ins = [l.strip() for l in seg if l.strip() and not l.strip().startswith((";", "."))]
kinds = {"VALU": lambda l: l.startswith("v_"), "SALU": lambda l: l.startswith("s_") and not l.startswith(("s_nop", "s_waitcnt", "s_cbranch", "s_branch")),
         "branch": lambda l: l.startswith(("s_cbranch", "s_branch")), "DS": lambda l: l.startswith("ds_"),
         "nop": lambda l: l.startswith("s_nop"), "wait": lambda l: l.startswith("s_waitcnt")}
print({k: sum(1 for l in ins if f(l)) for k, f in kinds.items()}, "total", len(ins))
if "--dump" in sys.argv:
    print("\n".join(ins))
