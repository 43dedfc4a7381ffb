"""How much the compute stream's kernels stretch when the side stream's weight gradients share the CUs.

python tools/overlap_stretch.py gpurun_out/prof_<tag>/run_kernel_trace.csv
Steps end at the SGD kernel. bench.py runs one serialised calibration step (every launch on the compute
queue) before the timed steps, so each compute-queue launch of the last timed step is matched by position
with the same launch of the calibration step: in-step duration / solo duration, and the share of its
in-step duration during which a side-queue kernel ran."""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], []
    for r in rows:
        cur.append(r)
        if "sgd_mom" in r["Kernel_Name"]:
            steps.append(cur)
            cur = []
    queues = lambda st: {r["Queue_Id"] for r in st}  # noqa: E731
    def top_share(st):
        c = defaultdict(int)
        for r in st:
            c[r["Queue_Id"]] += 1
        return max(c.values()) / len(st)
    calib = [s for s in steps if top_share(s) > 0.95 and len(s) > 100]
    timed = [s for s in steps if top_share(s) < 0.95]
    if not calib or not timed:
        print("no calibration / timed step found", len(steps))
        return
    # (the step before the last timed one when there is one: bench.py's last timed step carries the HIP
    # event packets that time the kernel families)
    cal, last = calib[-1], timed[-2] if len(timed) >= 2 else timed[-1]
    qcount = defaultdict(int)
    for r in last:
        qcount[r["Queue_Id"]] += 1
    main_q = max(qcount, key=lambda q: sum(1 for r in last if r["Queue_Id"] == q and "igemm" in r["Kernel_Name"]))
    side = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in last if r["Queue_Id"] != main_q]
    mains = [r for r in last if r["Queue_Id"] == main_q]
    # the calibration step's launches in order, minus the side-stream kernels (match by kernel name sequence)
    cal_by_name = defaultdict(list)
    for r in cal:
        cal_by_name[r["Kernel_Name"]].append(r)
    used = defaultdict(int)
    agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for r in mains:
        nm = r["Kernel_Name"]
        k = used[nm]
        used[nm] += 1
        lst = cal_by_name.get(nm, [])
        if k >= len(lst):
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        solo = int(lst[k]["End_Timestamp"]) - int(lst[k]["Start_Timestamp"])
        ov = 0
        for a, b in side:
            ov += max(0, min(b, e) - max(a, s))
        short = nm.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]
        g = agg[short]
        g[0] += 1
        g[1] += (e - s) / 1e3
        g[2] += solo / 1e3
        g[3] += min(ov, e - s) / 1e3
    tot = [0.0, 0.0]
    print("%-70s %4s %9s %9s %6s %8s" % ("compute-stream kernel", "n", "step us", "solo us", "x", "ovl"))
    for k, (n, d, so, ov) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        tot[0] += d
        tot[1] += so
        print("%-70s %4d %9.1f %9.1f %6.2f %7.0f%%" % (k, n, d, so, d / max(so, 1e-9), 100 * ov / max(d, 1e-9)))
    print("total compute-stream kernel time %.3f ms in-step vs %.3f ms solo (x%.3f)" % (tot[0] / 1e3, tot[1] / 1e3,
                                                                                  tot[0] / max(tot[1], 1e-9)))


if __name__ == "__main__":
    main(sys.argv[1])
