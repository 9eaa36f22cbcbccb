"""Prints the global-memory instruction stream of one kernel from a device .s file, with runs of
identical opcodes collapsed -- to spot loads serialised by s_waitcnt (e.g. a load inside a
branch followed by vmcnt(0)).   usage: python tools/isa_loads.py file.s SYMBOL_SUBSTRING [max_lines]"""
import re
import sys

src, pat = sys.argv[1], sys.argv[2]
lim = int(sys.argv[3]) if len(sys.argv) > 3 else 200
s = open(src).read()
names = [m.group(1) for m in re.finditer(r"^(_Z\S+):", s, flags=re.M) if pat in m.group(1)]
name = names[0]
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
ops = []
for line in s[i:j].split("\n"):
    t = line.strip()
    if re.match(r"(global_load|global_store|global_atomic|flat_load|flat_store|s_waitcnt\s+vmcnt|v_mfma|ds_write|ds_read|s_cbranch)", t):
        ops.append(t.split(";")[0].strip())
print(name, len(ops), "ops")
out, prev, cnt = [], None, 0
for o in ops:
    k = o.split()[0] if not o.startswith("s_waitcnt") else o
    if k == prev:
        cnt += 1
        continue
    if prev is not None:
        out.append(f"{cnt:3d}x {prev}")
    prev, cnt = k, 1
out.append(f"{cnt:3d}x {prev}")
print("\n".join(out[:lim]))
