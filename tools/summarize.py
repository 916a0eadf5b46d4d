"""Summarize gpurun_out logs: test lines, bench JSON, kernel profile."""
import csv, collections, glob, json, os, sys
out = "gpurun_out"
for f in sorted(glob.glob(f"{out}/t_*.log")):
    for l in open(f):
        if any(k in l for k in ("token-exact", "passed", "failed", "Error", "sampler:", "mid row")):
            print(os.path.basename(f), l.rstrip()[:200])
for f in sorted(glob.glob(f"{out}/micro*.log")):
    for l in open(f):
        if "us/step" in l or "Error" in l:
            print(l.rstrip())
b = f"{out}/bench.log"
if os.path.exists(b):
    lines = [l for l in open(b) if l.startswith("{")]
    if lines:
        d = json.loads(lines[-1])
        print("BENCH", d["value"], d.get("ms_per_step"), json.dumps(d.get("roofline")), json.dumps(d.get("cpu_baseline")))
    else:
        print(open(b).read()[-3000:])
t = f"{out}/prof/run_kernel_trace.csv"
if os.path.exists(t):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(t)):
        key = (r["Kernel_Name"][:45], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        d[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in d.values())
    print(f"kernel total {tot/1e6:.1f} ms")
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[1]) if len(sys.argv) > 1 else 16]:
        v = sorted(v)
        print(f"{sum(v)/1e6:8.1f} ms n={len(v):6d} med={v[len(v)//2]/1e3:7.2f}us", k)
