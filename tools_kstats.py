import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
frames = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 22]:
    n = r["Name"].replace("void ", "")[:80]
    print(f'{float(r["TotalDurationNs"])/1e6/frames:8.3f} ms/fr {int(r["Calls"])/frames:8.1f} c/fr avg {float(r["AverageNs"])/1e3:8.2f} us  {n}')
print("total ms/frame", tot/1e6/frames)
