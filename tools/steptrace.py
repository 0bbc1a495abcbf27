"""Timeline of one step from a rocprofv3 kernel_trace.csv: the kernels around
the n-th launch of a marker kernel, with start offsets and durations (us)."""
import csv
import sys

path, marker = sys.argv[1], sys.argv[2]
nth = int(sys.argv[3]) if len(sys.argv) > 3 else 30
span = int(sys.argv[4]) if len(sys.argv) > 4 else 8
r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(r) if marker in x["Kernel_Name"]]
i0 = idx[nth]
t0 = int(r[i0 - span // 2]["Start_Timestamp"])
for x in r[i0 - span // 2:i0 + span]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    print(f"{x['Kernel_Name'][:50]:50s} start {(s - t0) / 1000:8.1f} dur {(e - s) / 1000:7.1f}")
