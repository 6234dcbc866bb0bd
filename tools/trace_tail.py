import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'hs_' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
t0 = int(rows[-n]['Start_Timestamp'])
for r in rows[-n:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{r['Kernel_Name'][:70]:70s} start {(s - t0) / 1e3:9.2f} us  dur {(e - s) / 1e3:8.2f} us")
