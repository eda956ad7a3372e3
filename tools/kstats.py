"""Per-call summary of a rocprofv3 kernel_stats.csv: python tools/kstats.py <csv> <calls-per-unit>"""
import csv
import sys
rows = list(csv.DictReader(open(sys.argv[1])))
per = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(r['Name'][:64].ljust(64), r['Calls'].rjust(6), f"{float(r['TotalDurationNs']) / per / 1e3:8.1f} us/unit",
          f"{float(r['AverageNs']) / 1e3:8.2f} us avg")
print(f"total {tot / per / 1e3:.1f} us/unit")
