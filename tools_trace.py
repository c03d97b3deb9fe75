"""Per-kernel durations from a rocprofv3 kernel trace: isolated (no other kernel overlapping) vs overlapped."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
keys = {'occupancy': 'OCC', 'tile_kernel': 'TILE', 'compress_gate': 'CG', 'score_list': 'SCORE', 'replay': 'REPLAY'}
ks = []
for r in rows:
    for k, v in keys.items():
        if k in r['Kernel_Name']:
            ks.append((v, int(r['Start_Timestamp']), int(r['End_Timestamp']), int(r['Grid_Size_Y']) * int(r['Grid_Size_Z'])))
iso, ovl = defaultdict(list), defaultdict(list)
for i, (n, s, e, fr) in enumerate(ks):
    others = [(s2, e2) for j, (_, s2, e2, _) in enumerate(ks) if j != i and s2 < e and e2 > s]
    (ovl if others else iso)[n].append((e - s) / 1e3)
for n in keys.values():
    for lab, d in (('isolated', iso), ('overlapped', ovl)):
        v = sorted(d[n])
        if v:
            print("%-6s %-10s n=%3d med=%7.1f us min=%7.1f" % (n, lab, len(v), v[len(v) // 2], v[0]))
