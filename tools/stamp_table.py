"""Side-by-side table of tools/tile_stamps.py blocks ("== name" headers) from one or more logs."""
import re
import sys
tab = {}
for i, path in enumerate(sys.argv[1:]):
    for b in open(path).read().split('== ')[1:]:
        lines = b.strip().split('\n')
        rows = {}
        for l in lines:
            m = re.match(r'wave0 (.+?)\s+(\d+)\s+wave1\s+(\d+)', l)
            if m:
                rows[m.group(1).strip()] = (int(m.group(2)), int(m.group(3)))
        tab[("%d:" % i if len(sys.argv) > 2 else "") + lines[0].strip()] = rows
names = list(tab)
keys = list(tab[names[0]])
print("%-24s" % "" + "".join("%17s" % n for n in names))
for k in keys:
    print("%-24s" % k + "".join("%8d/%-8d" % tab[n].get(k, (0, 0)) for n in names))
print("%-24s" % "total w0" + "".join("%17d" % sum(v[0] for v in tab[n].values()) for n in names))
