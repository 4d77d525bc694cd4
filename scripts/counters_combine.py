#!/usr/bin/env python3
"""Merge counters_*.json records (scripts/gpu_profile.sh) into one list: profiles/counters.json."""
import glob
import json
import os
import sys

recs = []
for d in sys.argv[1:]:
    for f in sorted(glob.glob(os.path.join(d, "counters_*.json"))):
        recs.append(json.load(open(f)))
print(json.dumps(recs, indent=1))
