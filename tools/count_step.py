"""Static instruction mix of a kernel's innermost Dijkstra-step loop (dev tool).
usage: python tools/count_step.py <kernel-substring> [--dump]"""
import subprocess, sys
src = "mpi-hungarian-method_amd/csrc/santa_hip.hip"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                "-Iinclude", "--cuda-device-only", "-S", "-o", "/tmp/sh.s", src], check=True,
               stderr=subprocess.DEVNULL)
s = open("/tmp/sh.s").read()
name = sys.argv[1]
a = s.index(name)
b = s.index(".Lfunc_end", a)
body = s[a:b].splitlines()
idx = [i for i, l in enumerate(body) if "v_min_u32_dpp" in l][0]
hdr = max(i for i in range(idx) if "Loop Header: Depth=2" in body[i])
lab = body[hdr - 1].split(":")[0]
end = max(i for i, l in enumerate(body) if lab in l and "branch" in l)
seg = body[hdr:end + 1]
ins = [l.strip() for l in seg if l.strip() and not l.strip().startswith((";", "."))]
kinds = {"VALU": lambda l: l.startswith("v_"), "SALU": lambda l: l.startswith("s_") and not l.startswith(("s_nop", "s_waitcnt", "s_cbranch", "s_branch")),
         "branch": lambda l: l.startswith(("s_cbranch", "s_branch")), "DS": lambda l: l.startswith("ds_"),
         "nop": lambda l: l.startswith("s_nop"), "wait": lambda l: l.startswith("s_waitcnt")}
print({k: sum(1 for l in ins if f(l)) for k, f in kinds.items()}, "total", len(ins))
if "--dump" in sys.argv:
    print("\n".join(ins))
