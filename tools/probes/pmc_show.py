import csv, collections, glob, sys, os
for d in sorted(glob.glob(sys.argv[1] + "/*")):
    f = os.path.join(d, "p_counter_collection.csv")
    if not os.path.exists(f): continue
    agg = collections.defaultdict(float); disp = set()
    for r in csv.DictReader(open(f)):
        agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
    last = sorted(disp, key=int)[-1]
    print(os.path.basename(d), {c: "%.3g" % v for (dd, c), v in sorted(agg.items()) if dd == last})
