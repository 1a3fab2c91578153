import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    try:
        d = json.load(open(f))
    except Exception as e:
        print(f, "unreadable", e); continue
    k = d["kernels"]
    print(f"{f.split('/')[-1]:28s} value={d['value']:8.1f} ser={k['serialize_execute']['GBps']:7.1f} "
          f"de={k['deserialize_execute']['GBps']:7.1f} copy={d.get('copy_ceiling',{}).get('GBps')} ms/step={d['ms_per_step']}")
