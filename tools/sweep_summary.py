#!/usr/bin/env python3
"""Table of a ratio_sweep JSON (bench.py / tools/ratio_sweep.py output)."""
import json
import sys

d = json.load(open(sys.argv[1]))
d = d.get("ratio_sweep", d)
print(f"{d['single_pass_cases']}/{d['cases']} single-pass, min speedup {d['min_speedup_vs_two_launch']}")
for r in d["rows"]:
    print(f"{r['L']}/{r['M']} K{r['K']:<4} {r['path']:<12} TS {r['tile_len']:<3} {r['ms']:8.4f} ms "
          f"{r['msamples_s']:10.1f} Ms/s  two-launch {r.get('two_launch_ms', 0):8.4f} ms  "
          f"x{r.get('speedup_vs_two_launch', 0)}")
