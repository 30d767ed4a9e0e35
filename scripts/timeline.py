"""Print the kernel timeline of the last step(s) in a rocprofv3 kernel trace."""
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if 'k_' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
starts = [k for k, r in enumerate(rows) if 'k_prio' in r['Kernel_Name']]
for idx in starts[-int(sys.argv[2]) if len(sys.argv) > 2 else -1:]:
    t0 = int(rows[idx]['Start_Timestamp'])
    print('---')
    for r in rows[idx:idx + 8]:
        if r is not rows[idx] and 'k_prio' in r['Kernel_Name']:
            break
        print("%-28s q%-3s start %8.3f end %8.3f dur %8.3f grid %s" % (
            r['Kernel_Name'][:28], r['Queue_Id'], (int(r['Start_Timestamp']) - t0) / 1e6,
            (int(r['End_Timestamp']) - t0) / 1e6,
            (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6, r.get('Grid_Size_X', r.get('Grid_Size'))))
