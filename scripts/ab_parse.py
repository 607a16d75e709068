"""Summarise interleaved A/B logs: a label line, then the JSON line of that run."""
import collections
import json
import sys

r = collections.defaultdict(list)
key = None
for line in open(sys.argv[1]):
    line = line.strip()
    if line.startswith("{"):
        r[key].append(json.loads(line)["ms_per_step"])
    elif line:
        key = line
for k, v in r.items():
    print(f"{k:44s}", " ".join(f"{x:.4f}" for x in v), " min", round(min(v), 4))
