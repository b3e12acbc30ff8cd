"""Print the state kernel's average time per ablation variant (gpurun_out/abl/p*/)."""
import csv
import glob
import re

for d in sorted(glob.glob("gpurun_out/abl/p*"), key=lambda p: int(re.sub(r"\D", "", p.split("/")[-1]))):
    for f in glob.glob(d + "/*kernel_stats.csv"):
        for r in csv.DictReader(open(f)):
            n = r["Name"]
            if "fb_lti_kernel<2, 64, 2" in n or "fb_lti_gemm" in n:
                k = n[n.find("fb_"):n.find("(", n.find("fb_"))]
                print("%-6s %-34s %8.1f us" % (d.split("/")[-1], k, float(r["AverageNs"]) / 1e3))
