"""Average duration per (kernel, grid size) from a rocprofv3 kernel trace:
separates the k_pair launches of one bench run (the hot launch and the row
launches of the overlapped steps, and the full-grid roofline probe)."""
import collections, csv, glob, json, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    name = r['Kernel_Name']
    if 'k_' not in name:
        continue
    short = name.split('(')[0].replace('void ', '').replace('lqro::', '')
    grid = int(r.get('Grid_Size_X') or r.get('Grid_Size'))
    wg = int(r.get('Workgroup_Size_X') or r.get('Workgroup_Size'))
    acc[(short, grid // wg, wg)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
out = []
for (k, nwg, wg), v in sorted(acc.items()):
    out.append({"kernel": k, "workgroups": nwg, "threads": wg, "launches": len(v),
                "avg_ms": sum(v) / len(v), "min_ms": min(v), "max_ms": max(v)})
    print(f"{k:22s} wg {nwg:5d} x {wg:4d}  n {len(v):3d}  avg {sum(v)/len(v):8.3f} ms  "
          f"min {min(v):8.3f}  max {max(v):8.3f}")
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], 'w'), indent=1)
