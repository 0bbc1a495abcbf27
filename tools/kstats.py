"""Print rocprofv3 kernel-stats rows (name, calls, average us) whose name
contains any of the given substrings.  python3 tools/kstats.py FILE [SUBSTR...]"""
import csv
import sys

keys = sys.argv[2:]
for r in csv.DictReader(open(sys.argv[1])):
    if not keys or any(k in r["Name"] for k in keys):
        print(f'{r["Name"][:70]:70s} {r["Calls"]:>5s} {float(r["AverageNs"]) / 1e3:10.1f} us')
