"""Print one graph replay's kernel timeline from a rocprofv3 kernel-trace CSV."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
first = sys.argv[2] if len(sys.argv) > 2 else 'stem_kernel'
idx = [i for i, r in enumerate(rows) if first in r['Kernel_Name']]
s, e = idx[-4], idx[-3]
win = rows[s:e]
t0 = int(win[0]['Start_Timestamp'])
tl = int(win[-1]['End_Timestamp'])
busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in win)
print(f"kernels {len(win)} span {(tl - t0) / 1e3:.1f} us busy {busy / 1e3:.1f} us")
for r in win:
    st, en = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    nm = r['Kernel_Name'].replace('void ', '').replace('fce::', '')[:48]
    print(f"{(st - t0) / 1e3:8.1f} {(en - st) / 1e3:7.1f}  {nm:48s} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']} vgpr={r['VGPR_Count']} agpr={r['Accum_VGPR_Count']}")
