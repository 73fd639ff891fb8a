"""Print the per-kernel averages of rocprofv3 --stats CSVs (one per argument)."""
import csv
import sys

for f in sys.argv[1:]:
    print(f)
    for r in csv.DictReader(open(f)):
        if float(r["Percentage"]) > 1.0:
            print(f"  {r['Name'][:70]:70s} calls {r['Calls']:>5s}  avg {float(r['AverageNs'])/1e3:9.2f} us")
