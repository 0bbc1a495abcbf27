"""Instruction counts of kernels in a device-only assembly file (hipcc
--cuda-device-only -S): total, SALU, VALU, LDS, v_mul_hi.  Usage:
python3 tools/isa_count.py file.s [name-substring]"""
import re
import sys

txt = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)\n\.Lfunc_end", txt, re.S):
    name = m.group(1)
    if pat not in name:
        continue
    ops = []
    for l in m.group(2).split("\n"):
        l = l.strip()
        if not l or l.startswith((".", ";")) or l.endswith(":"):
            continue
        ops.append(l.split()[0])
    c = lambda f: sum(1 for o in ops if f(o))
    print(f"{name[:70]:70s} total {len(ops):5d} salu {c(lambda o: o.startswith('s_')):5d} "
          f"valu {c(lambda o: o.startswith('v_')):5d} ds {c(lambda o: o.startswith('ds_')):4d} "
          f"mul_hi {c(lambda o: 'mul_hi' in o):3d}")
