#!/usr/bin/env python3
"""One line per tools/ab.py log: median ms per build (!DIFF = frame differs from the first build)."""
import json,sys
for f in sys.argv[1:]:
    t=open(f).read(); d=json.loads(t[t.index('{'):])
    print(f.split('/')[-1], ' '.join(f"{k.replace('.so','')}={v['median_ms']}{'' if v.get('same_image_as_first', True) else '!DIFF'}" for k,v in d['results'].items()))
