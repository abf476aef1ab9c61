"""Basic-block VALU/LDS/SALU counts of one kernel in a hipcc --save-temps .s
file: python tools/isa_blocks.py file.s <kernel-substring> [min_valu]."""
import re
import sys

path, name = sys.argv[1], sys.argv[2]
minv = int(sys.argv[3]) if len(sys.argv) > 3 else 20
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + name + r"\S*:", l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.size") or lines[i].startswith(".Lfunc_end"))
blocks, cur = [], ["entry", []]
for l in lines[start + 1:end]:
    m = re.match(r"^(\.LBB\S+):", l)
    if m:
        blocks.append(cur)
        cur = [m.group(1), []]
        continue
    s = l.strip()
    if s and not s.startswith(";") and not s.startswith("."):
        cur[1].append(s)
blocks.append(cur)
tot = {}
for lab, ins in blocks:
    ops = [i.split()[0] for i in ins]
    v = [o for o in ops if o.startswith("v_")]
    f64 = [o for o in v if "f64" in o]
    ds = [o for o in ops if o.startswith("ds_")]
    br = [i for i in ins if i.startswith("s_cbranch") or i.startswith("s_branch")]
    if len(v) >= minv or br and any(lab in b for b in br):
        print(f"{lab:14s} valu={len(v):5d} f64={len(f64):5d} ds={len(ds):4d} n={len(ins):5d} br={[b for b in br]}")
    for o in v:
        tot[o] = tot.get(o, 0) + 1
if "-v" in sys.argv:
    for k, c in sorted(tot.items(), key=lambda t: -t[1])[:60]:
        print(f"{c:6d} {k}")
