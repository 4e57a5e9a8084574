"""Medians of scripts/ab_inproc.py's JSON (its log file) per library, one line each."""
import json
import sys

t = open(sys.argv[1]).read()
j = json.loads(t[t.index("{"):])
for k, v in j.items():
    print(f"{k:32s} " + " ".join(f"{x} {v[x]['median']:.4f}" for x in v))
