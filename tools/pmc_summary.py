import csv, glob, os, sys, collections
d = sys.argv[1]
k = sys.argv[2] if len(sys.argv) > 2 else "dfa_fwd"
acc = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "p*", "pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if k in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c, v in sorted(acc.items()):
    print("%-26s %16.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))
