"""Min / median CLI convergence time per (workload, variant) from tools/gpu.sh cli output (cli.txt)."""
import collections
import re
import statistics
import sys

d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    m = re.match(r"(\S+) (\d+ \S+ \S+): Convergence Time: ([\d.]+) ms Rounds: (\d+)", line)
    if m:
        d[(m.group(2), m.group(1))].append(float(m.group(3)))
for (wl, v), xs in sorted(d.items()):
    print(f"{wl:28s} {v:10s} min {min(xs):9.1f}  median {statistics.median(xs):9.1f}  ({' '.join(f'{x:.1f}' for x in xs)})")
