"""Average PMC counters per dispatch of the dominant kernel in a gpu_pmc_cfg.sh output dir."""
import collections, csv, glob, sys
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{d}/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "_kernel" in r["Kernel_Name"] and "gen_kernel" not in r["Kernel_Name"]:
            agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for c, v in sorted(agg.items()):
    print(f"{c:24s} {sum(v.values()) / len(v):16.4g}")
