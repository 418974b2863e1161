"""Instruction mix of one kernel in a device assembly file (hipcc --cuda-device-only -S).

usage: python tools/asm_stats.py FILE.s KERNEL_SUBSTRING
"""
import collections
import re
import sys

src, pat = sys.argv[1], sys.argv[2]
s = open(src).read()
m = re.search(r"^(_Z[^ :]*%s[^ :]*):" % re.escape(pat), s, re.M)
body = s[m.start(): s.find(".Lfunc_end", m.start())]
cnt = collections.Counter()
for line in body.splitlines():
    t = line.strip().split()
    if t and re.match(r"^[vsd]_|^ds_|^global_|^buffer_|^flat_", t[0]):
        cnt[t[0]] += 1
tot = sum(cnt.values())
print(m.group(1), "instructions:", tot)
for k, v in cnt.most_common(40):
    print(f"  {k:32s} {v}")
