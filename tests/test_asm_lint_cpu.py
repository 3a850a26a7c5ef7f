"""CPU lint of the kernels' inline asm and code object.

Round 5's one-wave solvers updated one slot of a four-register tuple per
Dijkstra step through GPR index mode (`s_set_gpr_idx_on ... gpr_idx(DST)`).
Round 6 pinned the tuples to fixed registers and declared the M0 clobber, and
the indexed instructions were then exactly round 5's -- yet every build whose
register allocation differed from round 5's corrupted results of other blocks
at random (a whole VGPR of a block's output stage, or a step), while the same
source without index mode was exact on every run (DESIGN §8a,
tools/diag_round.py).  The kernels now keep those tie bits in LDS.  This test
pins the rules that came out of it:

* no inline asm uses GPR index mode or M0-relative moves
  (`s_set_gpr_idx_*`, `v_movrel*`, `s_movrel*`);
* no kernel in the built code object writes through GPR index mode (the
  compiler's own indexed *reads* of register arrays, `gpr_idx(SRC0)`, stay:
  they were present in every exact build);
* an asm statement that names `m0` receives it as a `{m0}` input (the
  compiler loads it) or clobbers it.
"""
import os
import re
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "mpi-hungarian-method_amd", "csrc", "santa_hip.hip")
LIB = os.path.join(ROOT, "mpi-hungarian-method_amd", "santa_hip", "libsanta_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _asm_statements(text):
    """(line, body) of every `asm(...)` / `asm volatile(...)` statement."""
    out = []
    for m in re.finditer(r"\basm\s*(?:volatile\s*)?\(", text):
        i, depth, in_str = m.end(), 1, False
        while depth:
            c = text[i]
            if in_str:
                if c == "\\":
                    i += 1
                elif c == '"':
                    in_str = False
            elif c == '"':
                in_str = True
            elif c == "(":
                depth += 1
            elif c == ")":
                depth -= 1
            i += 1
        out.append((text.count("\n", 0, m.start()) + 1, text[m.end():i - 1]))
    return out


def _split_sections(body):
    """Split an asm body at top-level ':' into template/outputs/inputs/clobbers."""
    parts, cur, depth, in_str, i = [], [], 0, False, 0
    while i < len(body):
        c = body[i]
        if in_str:
            cur.append(c)
            if c == "\\":
                cur.append(body[i + 1])
                i += 1
            elif c == '"':
                in_str = False
        elif c == '"':
            in_str = True
            cur.append(c)
        elif c in "([":
            depth += 1
            cur.append(c)
        elif c in ")]":
            depth -= 1
            cur.append(c)
        elif c == ":" and depth == 0:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(c)
        i += 1
    parts.append("".join(cur))
    return parts + [""] * (4 - len(parts))


def _template(section):
    return "".join(re.findall(r'"((?:[^"\\]|\\.)*)"', section)).replace("\\n", "\n").replace("\\t", " ")


def _statements():
    text = open(SRC).read()
    return [(line, _split_sections(body)) for line, body in _asm_statements(text)]


def test_asm_found():
    assert len(_statements()) > 40


def test_no_gpr_index_mode_or_movrel_in_inline_asm():
    for line, (tmpl_s, _, _, _) in _statements():
        tmpl = _template(tmpl_s)
        assert not re.search(r"s_set_gpr_idx|v_movrel|s_movrel", tmpl), \
            f"santa_hip.hip:{line}: inline asm uses GPR index mode / M0-relative moves: {tmpl!r}"


def test_m0_is_an_input_or_clobbered():
    for line, (tmpl_s, outs_s, ins_s, clob_s) in _statements():
        if not re.search(r"\bm0\b", _template(tmpl_s)):
            continue
        ins = re.findall(r'"([^"]*)"\s*\(', ins_s)
        clobbers = re.findall(r'"([^"]*)"', clob_s)
        assert "{m0}" in ins or "m0" in clobbers, \
            f"santa_hip.hip:{line}: asm names m0 without a {{m0}} input or an m0 clobber"


def test_code_object_has_no_indexed_writes(tmp_path):
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")]
    if not os.path.exists(LIB) or not all(os.path.exists(t) for t in tools):
        pytest.skip("library or ROCm LLVM tools absent")
    objcopy, bundler, objdump = tools
    fb, co = str(tmp_path / "fb.bin"), str(tmp_path / "co.o")
    subprocess.run([objcopy, f"--dump-section=.hip_fatbin={fb}", LIB, str(tmp_path / "junk.so")], check=True)
    subprocess.run([bundler, "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}",
                    f"--output={co}", "--unbundle"], check=True)
    dis = subprocess.run([objdump, "-d", "--no-show-raw-insn", co], check=True, capture_output=True,
                         text=True).stdout
    modes = re.findall(r"s_set_gpr_idx_on\s+\S+,\s*gpr_idx\(([A-Z0-9,]*)\)", dis)
    assert not re.search(r"v_movrel|s_movrel|s_set_gpr_idx_mode", dis)
    bad = sorted({m for m in modes if "DST" in m})
    assert not bad, f"indexed writes in the code object: gpr_idx({bad})"
