"""Print a rocprofv3 kernel_stats.csv as a short table (name, calls, avg us, %)."""
import csv
import sys

for x in list(csv.DictReader(open(sys.argv[1])))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{x['Name'][:80]:80s} {x['Calls']:>6s} {float(x['AverageNs'])/1000:9.1f} us {float(x['Percentage']):6.2f}%")
