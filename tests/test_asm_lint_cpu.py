"""CPU lint of the kernels' GPR-indexed inline asm and code object (VERDICT r05
weak #1).

A GPR-indexed instruction (between `s_set_gpr_idx_on` and `s_set_gpr_idx_off`)
addresses "the register it names + M0[7:0]".  The rules, each learned the hard
way:

* the indexed instruction is `v_mov_b32` (VOP1), the only form the compiler
  itself emits in index mode.  Round 5 also indexed `v_cndmask_b32_e64` and
  `v_xor_b32`; those were exact only under round 5's register allocation --
  every other allocation corrupted registers of other blocks at random, and
  so did a `v_cndmask_b32_e32` form -- while v_mov-only builds were exact on
  every run (tools/diag_round.py, profiles/r06_gpr_idx_diag.jsonl);
* the statement declares M0 clobbered (`s_set_gpr_idx_on` writes M0 bits 7:0
  and 15:12);
* the indexed operand names the FIRST register of a tuple literally
  (`SH_VREG(base)`), and that tuple is an operand of the same statement
  pinned to exactly those physical registers (`SH_VTUPLE(base, base + 3)`):
  in-out ("+") when the indexed v_mov writes it (DST), input or in-out when it
  reads it (SRC0).  A `%N` operand in an indexed slot is the bug this guards
  against: the compiler may give a scalar operand like `lo.x` its own
  register, and the indexed access then lands in an unrelated live register;
* any asm that names `m0` receives it as a `{m0}` input or clobbers it;
* the built code object holds no other instruction in index mode and no
  M0-relative moves (`v_movrel*`, `s_movrel*`), compiler-generated included.
"""
import os
import re
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "mpi-hungarian-method_amd", "csrc", "santa_hip.hip")
LIB = os.path.join(ROOT, "mpi-hungarian-method_amd", "santa_hip", "libsanta_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _defines(text):
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"^#define (\w+) (\d+)\b", text, re.M)}


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


def _expand(section, defs):
    """Resolve the register macros and concatenate adjacent string literals."""
    s = re.sub(r"SH_VREG\((\w+)\)", lambda m: '"v%d"' % defs[m.group(1)], section)
    s = re.sub(r"SH_VTUPLE\((\w+),\s*(\w+)\)",
               lambda m: '"{v[%d:%d]}"' % (defs[m.group(1)], defs[m.group(2)]), s)
    return re.sub(r'"\s*"', "", s)  # "a" "b" -> "ab"


def _template(section):
    return "".join(re.findall(r'"((?:[^"\\]|\\.)*)"', section)).replace("\\n", "\n").replace("\\t", " ")


def _operands(section):
    """[(constraint, expr)] of an operand list."""
    return [(m.group(1), m.group(2).strip())
            for m in re.finditer(r'"([^"]*)"\s*\(((?:[^()]|\([^()]*\))*)\)', section)]


def _statements():
    text = open(SRC).read()
    defs = _defines(text)
    for line, body in _asm_statements(text):
        yield line, [_expand(p, defs) for p in _split_sections(body)]


def test_pinned_tuple_bases_are_four_wide():
    defs = _defines(open(SRC).read())
    bases = [k for k in defs if re.fullmatch(r"\w+_V", k) and k + "E" in defs]
    assert bases, "no pinned tuple bases found"
    for k in bases:
        assert defs[k + "E"] == defs[k] + 3, f"{k}: tuple {defs[k]}..{defs[k + 'E']} is not 4 VGPRs"


def test_gpr_indexed_asm_is_well_defined():
    seen = 0
    for line, (tmpl_s, outs_s, ins_s, clob_s) in _statements():
        tmpl = _template(tmpl_s)
        if "s_set_gpr_idx_on" not in tmpl:
            continue
        seen += 1
        clobbers = re.findall(r'"([^"]*)"', clob_s)
        assert "m0" in clobbers, f"santa_hip.hip:{line}: s_set_gpr_idx_on without an m0 clobber"
        pinned = {}
        for c, expr in _operands(outs_s) + _operands(ins_s):
            m = re.fullmatch(r"([+=&]*)\{v\[(\d+):(\d+)\]\}", c)
            if m:
                pinned[int(m.group(2))] = (m.group(1), int(m.group(3)), expr)
        lines = [x.strip() for x in tmpl.split("\n") if x.strip()]
        for k, x in enumerate(lines):
            m = re.match(r"s_set_gpr_idx_on\s+\S+,\s*gpr_idx\(([A-Z0-9,]*)\)", x)
            if not m:
                continue
            mode = m.group(1)
            inst = lines[k + 1]
            assert lines[k + 2].startswith("s_set_gpr_idx_off"), \
                f"santa_hip.hip:{line}: more than one instruction in gpr-index mode"
            op, args = inst.split(None, 1)
            assert op == "v_mov_b32", f"santa_hip.hip:{line}: {op} in index mode (only v_mov_b32)"
            assert mode in ("SRC0", "DST"), f"santa_hip.hip:{line}: gpr_idx({mode}) on a v_mov"
            dst, src = [o.strip() for o in args.split(",")]
            reg = dst if mode == "DST" else src
            r = re.fullmatch(r"v(\d+)", reg)
            assert r, f"santa_hip.hip:{line}: indexed operand {reg!r} of {inst!r} is not a literal register"
            base = int(r.group(1))
            assert base in pinned, f"santa_hip.hip:{line}: v{base} is not the base of a pinned tuple operand"
            mod, end, expr = pinned[base]
            assert end == base + 3
            if mode == "DST":
                assert "+" in mod, f"santa_hip.hip:{line}: indexed write into {expr}, not an in-out operand"
    assert seen >= 6, f"expected the six gpr-indexed statements of sp3/dt, found {seen}"


def test_no_movrel_in_inline_asm_and_m0_declared():
    for line, (tmpl_s, _, ins_s, clob_s) in _statements():
        tmpl = _template(tmpl_s)
        assert not re.search(r"v_movrel|s_movrel|s_set_gpr_idx_mode|s_set_gpr_idx_idx", tmpl), \
            f"santa_hip.hip:{line}: M0-relative move / index-mode change outside the v_mov pattern"
        if re.search(r"\bm0\b", tmpl):
            ins = [c for c, _ in _operands(ins_s)]
            clobbers = re.findall(r'"([^"]*)"', clob_s)
            assert "{m0}" in ins or "m0" in clobbers, \
                f"santa_hip.hip:{line}: asm names m0 without a {{m0}} input or an m0 clobber"


def test_code_object_indexes_only_v_mov(tmp_path):
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
    lines = [x.split("//")[0].strip() for x in dis.splitlines()]
    assert not any(re.match(r"(v_movrel|s_movrel|s_set_gpr_idx_mode|s_set_gpr_idx_idx)", x) for x in lines)
    inside = [lines[k + 1].split()[0] for k, x in enumerate(lines) if x.startswith("s_set_gpr_idx_on")]
    assert inside, "no GPR indexing found at all (test out of date?)"
    assert set(inside) == {"v_mov_b32_e32"}, f"instructions in index mode: {sorted(set(inside))}"
