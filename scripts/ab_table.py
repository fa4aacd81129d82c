"""Median table of scripts/potrf_ab.sh / knob_ab.sh output: python3 scripts/ab_table.py FILE..."""
import re, sys, collections
d = collections.defaultdict(list)
for fn in sys.argv[1:]:
    for l in open(fn):
        m = re.match(r"(\S+) potrf n=(\d+).*median ([\d.]+) ms", l)
        if m:
            d[(m.group(1), int(m.group(2)))].append(float(m.group(3)))
specs = sorted({k[0] for k in d}, key=lambda s: list(d).index((s, [k for k in d if k[0] == s][0][1])))
sizes = sorted({k[1] for k in d}, reverse=True)
print("spec".ljust(40) + "".join(f"n={n}".rjust(22) for n in sizes))
for sp in specs:
    print(sp.ljust(40) + "".join(("/".join(f"{v:.3f}" for v in d.get((sp, n), []))).rjust(22) for n in sizes))
