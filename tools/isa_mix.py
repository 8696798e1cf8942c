#!/usr/bin/env python3
"""Instruction mix per kernel of a device .s file: isa_mix.py FILE.s [name-substring ...]"""
import re
import sys
from collections import Counter

text = open(sys.argv[1]).read()
subs = sys.argv[2:]
starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\w+):", text, flags=re.M)]
for i, (pos, name) in enumerate(starts):
    if subs and not any(x in name for x in subs):
        continue
    end = starts[i + 1][0] if i + 1 < len(starts) else len(text)
    body = text[pos:end]
    ops = [l.split()[0] for l in body.split("\n") if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
    c = Counter(ops)
    pick = lambda pre: sum(v for k, v in c.items() if k.startswith(pre))
    print(f"{name[:60]:60s} total {len(ops):5d} valu {pick('v_'):5d} salu {pick('s_'):5d} "
          f"vmem {pick('global_') + pick('buffer_'):4d} ds {pick('ds_'):3d} min3 {c['v_min3_f32']} max3 {c['v_max3_f32']} "
          f"cndmask {pick('v_cndmask')} fma {pick('v_fma') + pick('v_fmac')} div_scale {c['v_div_scale_f32']} "
          f"f64 {pick('v_fma_f64') + pick('v_mul_f64') + pick('v_add_f64')}")
