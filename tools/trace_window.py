"""Print a steady-state window of a rocprofv3 kernel trace (times in us relative to one k_analyze start).
usage: python tools/trace_window.py <run_kernel_trace.csv> [analyze_index] [span_us]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
idx = int(sys.argv[2]) if len(sys.argv) > 2 else 10
span = float(sys.argv[3]) if len(sys.argv) > 3 else 3000.0
ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:44], r['Grid_Size_X']) for r in rows)
ana = [k for k in ks if 'analyze' in k[2]]
st = ana[idx][0]
for s, e, n, g in ks:
    if st - span * 1000 < s < st + span * 1000:
        print(f"{(s - st) / 1000:9.1f} {(e - st) / 1000:9.1f} {(e - s) / 1000:8.1f}  {n}  grid {g}")
