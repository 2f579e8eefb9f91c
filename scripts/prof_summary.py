import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 14]:
    print(f"{r['Name'][:95]:95s} calls={r['Calls']:>4s} avg={float(r['AverageNs'])/1e3:9.1f}us per_step={float(r['TotalDurationNs'])/steps/1e6:7.3f}ms {float(r['Percentage']):5.1f}%")
print("total per step ms", tot/steps/1e6)
