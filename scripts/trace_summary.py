"""Per-bounce kernel durations from rocprofv3 kernel-trace CSVs (one row per pass position)."""
import csv, sys, collections
for path in sys.argv[1:]:
    rows = [r for r in csv.DictReader(open(path)) if 'k_bounce' in r['Kernel_Name'] or 'k_shade' in r['Kernel_Name']]
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    per = collections.defaultdict(list)
    depth = 8
    for i, r in enumerate(rows):
        per[i % depth].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
    med = [sorted(v)[len(v) // 2] for k, v in sorted(per.items())]
    print(path.split('/')[-3] if '/' in path else path, ' '.join(f'{x:7.1f}' for x in med), ' sum', f'{sum(med):.1f}')
