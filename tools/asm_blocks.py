"""Per-basic-block instruction counts of one kernel (find the hot loop bodies).

usage: python tools/asm_blocks.py FILE.s KERNEL_SUBSTRING [N] [--dump LABEL]
"""
import re
import sys

src, pat = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3].isdigit() else 12
s = open(src).read()
m = re.search(r"^(_Z[^ :]*%s[^ :]*):" % re.escape(pat), s, re.M)
body = s[m.start(): s.find(".Lfunc_end", m.start())]
blocks, cur, name = [], [], "entry"
for line in body.splitlines():
    lm = re.match(r"^(\.LBB\S+):", line)
    if lm:
        blocks.append((name, cur))
        name, cur = lm.group(1), []
        continue
    t = line.strip().split()
    if t and not t[0].startswith((";", ".")):
        cur.append(line.strip())
blocks.append((name, cur))
if "--dump" in sys.argv:
    want = sys.argv[sys.argv.index("--dump") + 1]
    for n, ins in blocks:
        if n == want:
            print("\n".join(ins))
    sys.exit()


def stat(ins):
    f64 = sum(1 for i in ins if re.match(r"v_\w*f64", i) and not i.startswith("v_cmp"))
    cmp64 = sum(1 for i in ins if i.startswith("v_cmp") and "f64" in i)
    valu = sum(1 for i in ins if i.startswith("v_"))
    salu = sum(1 for i in ins if i.startswith("s_") and not i.startswith(("s_waitcnt", "s_nop", "s_cbranch", "s_branch")))
    lds = sum(1 for i in ins if i.startswith("ds_"))
    return f64, cmp64, valu, salu, lds, len(ins)


rows = sorted(((stat(ins), n) for n, ins in blocks), key=lambda r: -r[0][0])
print("block               f64  cmpf64  valu  salu  lds  total")
for (f64, c, v, sa, l, t), n in rows[:top]:
    print(f"{n:18s} {f64:5d} {c:6d} {v:5d} {sa:5d} {l:4d} {t:6d}")
