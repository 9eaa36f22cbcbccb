"""Per-kernel VGPR / AGPR / scratch / occupancy and the number of global loads issued before the
first s_waitcnt vmcnt, from a device .s file (hipcc --cuda-device-only -S).
usage: python tools/isa_summary.py file.s [SYMBOL_SUBSTRING]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"^(_Z\S+):", s, flags=re.M):
    name = m.group(1)
    if pat not in name:
        continue
    i = m.end()
    j = s.index(".Lfunc_end", i)
    body = s[i:j]
    tail = s[j:j + 4000]
    g = lambda k: (re.search(k + r":\s*(\d+)", tail) or [None, "?"])[1]
    loads = len(re.findall(r"^\s*global_load", body, flags=re.M))
    waits = len(re.findall(r"^\s*s_waitcnt\s+vmcnt", body, flags=re.M))
    mfma = len(re.findall(r"^\s*v_mfma", body, flags=re.M))
    print(f"{name[:90]:90s} vgpr {g('NumVgprs'):>3} agpr {g('NumAgprs'):>3} scratch {g('ScratchSize'):>4} "
          f"occ {g('Occupancy'):>2} loads {loads:4d} vmcnt-waits {waits:4d} mfma {mfma:4d}")
