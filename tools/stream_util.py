"""Per-queue busy time and idle gaps over the LAST uninstrumented training step of a rocprofv3 kernel trace (steps end
with the SGD kernel): how much of the step each HIP stream (queue) is busy, and the main queue's gaps.
usage: python tools/stream_util.py gpurun_out/prof_<tag>/run_kernel_trace.csv"""
import collections
import csv
import re
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "sgd_mom" in r["Kernel_Name"]]
    # the step before the last when there is one: bench.py's last timed step carries the HIP event
    # packets that time the kernel families (gaps of their own around every launch they wrap)
    k = -2 if len(idx) >= 3 else -1
    a, b = idx[k - 1] + 1, idx[k] + 1
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in step)
    print("step span %.3f ms, %d launches" % ((t1 - t0) / 1e6, len(step)))
    byq = collections.defaultdict(list)
    for r in step:
        byq[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    for q, ks in sorted(byq.items(), key=lambda kv: -len(kv[1])):
        busy = sum(e - s for s, e, _ in ks)
        gaps = [(ks[i + 1][0] - ks[i][1], ks[i][2], ks[i + 1][2]) for i in range(len(ks) - 1)]
        gsum = sum(max(g, 0) for g, _, _ in gaps)
        print("queue %s: %d launches, busy %.3f ms, gaps %.3f ms (first %.3f ms after step start, ends %.3f ms "
              "before step end)" % (q, len(ks), busy / 1e6, gsum / 1e6, (ks[0][0] - t0) / 1e6, (t1 - ks[-1][1]) / 1e6))
        big = sorted(gaps, key=lambda g: -g[0])[:8]
        for g, k1, k2 in big:
            nm = lambda k: re.sub(r"\(.*", "", k.replace("(anonymous namespace)::", "").replace("void ", ""))[:60]
            print("    gap %7.1f us  after %s  before %s" % (g / 1e3, nm(k1), nm(k2)))


if __name__ == "__main__":
    main(sys.argv[1])
