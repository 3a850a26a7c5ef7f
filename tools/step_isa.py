"""dev: static instruction count of one sap_solve_mw step in a gfx950 listing
(hipcc -S, as tools/isa_count.py makes it): the row read + relax + key +
lane/row argmin, from the loader's barrier to the step word's ds_min.
    python tools/step_isa.py LISTING.s KERNEL_SUBSTRING K [label]
Prints one JSON line; per_column = the first part / K (the slots per thread)."""
import collections
import json
import re
import sys


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
    return "other"


def count(lines):
    c = collections.Counter()
    for x in lines:
        u = x.strip().split()
        if u and not u[0].startswith((".", ";")) and not u[0].endswith(":"):
            c[kind(u[0])] += 1
    return dict(c)


def main():
    path, name, K = sys.argv[1], sys.argv[2], int(sys.argv[3])
    label = sys.argv[4] if len(sys.argv) > 4 else path
    s = open(path).read()
    m = re.search(r"^(_Z\S*" + re.escape(name) + r"\S*):", s, re.M)
    body = s[m.end():s.index(".Lfunc_end", m.end())].splitlines()
    i_min = next(i for i, l in enumerate(body) if "ds_min_u64" in l)
    i_bar = max(i for i in range(i_min) if "s_barrier" in body[i])
    step = count(body[i_bar:i_min + 1])
    print(json.dumps({"label": label, "kernel": name, "K": K, "relax_key_argmin": step,
                      "per_column_valu": round(step.get("valu", 0) / K, 1)}))


if __name__ == "__main__":
    main()
