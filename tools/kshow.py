import csv, re, sys
for f in sys.argv[1:]:
    print("==", f)
    for r in csv.DictReader(open(f)):
        n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        m = re.match(r"([\w:<>, ]+?)\(", n)
        short = (m.group(1) if m else n)[:48]
        print(f"  {short:48s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
