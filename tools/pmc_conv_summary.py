"""Summarise tools/pmc_conv.sh output: per kernel family, the mean of each SQ counter per dispatch,
plus the derived fractions (WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY of WAVE_CYCLES, LDS bank
conflict cycles / LDS active cycles). usage: python tools/pmc_conv_summary.py gpurun_out/pmcc_<tag>"""
import collections
import csv
import glob
import re
import sys


def fam(n):
    m = re.search(r"(igemm_big_kernel<[^>]*>|igemm_kernel<[^>]*>|wgrad_big_kernel<[^>]*>|wgrad_kernel<[^>]*>)", n)
    return m.group(1) if m else None


def main(base):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sorted(glob.glob(base + "_*/run_counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            f = fam(r["Kernel_Name"])
            if f:
                vals[f][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f, cs in vals.items():
        mean = {k: sum(v) / len(v) for k, v in cs.items()}
        print(f, "dispatches", len(next(iter(cs.values()))))
        for k in sorted(mean):
            print("   %-28s %14.4g" % (k, mean[k]))
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if k in mean:
                    print("   %-28s %13.1f%%" % (k + " / WAVE", 100 * mean[k] / wc))
        if mean.get("SQ_LDS_IDX_ACTIVE"):
            print("   %-28s %13.1f%%" % ("LDS_BANK_CONFLICT / ACTIVE", 100 * mean.get("SQ_LDS_BANK_CONFLICT", 0) /
                                           mean["SQ_LDS_IDX_ACTIVE"]))


if __name__ == "__main__":
    main(sys.argv[1])
