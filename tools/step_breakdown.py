"""Per-kernel breakdown of the LAST uninstrumented training step in a rocprofv3 kernel trace (steps end with the
SGD kernel). usage: python tools/step_breakdown.py gpurun_out/prof_<tag>/run_kernel_trace.csv"""
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
    fam = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in rows[a:b]:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        n = re.sub(r"\(.*", "", n).replace("void ", "").replace("unsigned short", "bf16")
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        fam[n] += d
        cnt[n] += 1
    span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e6
    print("kernel sum %.3f ms, wall span %.3f ms, launches %d" % (sum(fam.values()), span, b - a))
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print("%8.3f ms %4d  %s" % (v, cnt[k], k[:100]))


if __name__ == "__main__":
    main(sys.argv[1])
