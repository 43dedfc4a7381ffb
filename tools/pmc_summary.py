"""Summarise rocprofv3 --pmc passes (tools/pmc_bench.sh) per kernel family and for the last step.

Usage: python tools/pmc_summary.py gpurun_out/pmc_<tag>  [--json out.json]
Reads <dir>_fetch/, <dir>_write/ and (when present) <dir>_sq/run_counter_collection.csv.
MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) (rocprofv3's
MfmaUtil formula: GRBM_GUI_ACTIVE comes summed over the 8 XCDs); LDS bank-conflict share =
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles / all LDS-array cycles).
Units: rocprofv3 reports both counters in KiB. gfx950 correction (MI355X_MICROARCH.md, HBM
section): FETCH_SIZE counts half the bytes of a 16-B/lane streaming read -> doubled here;
WRITE_SIZE is exact for 16-B stores and fp32 atomics.
"""
import csv, json, re, sys, collections


def family(name):
    m = re.search(r"igemm_big_kernel<(\d+), \d+, \d+(?:, (?:true|false), (\d+))?", name)
    if m:
        return "igemm_big_kernel<%sx%s>" % (m.group(2) or "256", m.group(1))
    m = re.search(r"(igemm_kernel|wgrad_kernel)<([^>]*)>", name)
    if m:
        args = [a.strip() for a in m.group(2).split(",")]
        tname = {"__hip_bfloat16": "bf16", "float": "f32", "unsigned short": "bf16"}
        args = [tname.get(a, a) for a in args]
        if m.group(1) == "igemm_kernel":
            return "igemm_kernel<%s,%s,%sx%s>" % tuple(args[:4])
        return "wgrad_kernel<%s,%s,%s>" % tuple(args[:3])
    name = re.sub(r"^void\s+", "", name).replace("(anonymous namespace)::", "")
    m = re.match(r"(?:\w+::)*(\w+)", name)
    return m.group(1) if m else name[:40]


def load(path, counter):
    out = collections.defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            out[family(row["Kernel_Name"])].append(float(row["Counter_Value"]) * 1024.0)
    return out


def aggregate(name):
    """bench.py's family for a kernel family: every bf16 weight-gradient kernel is one family there."""
    if name.startswith("wgrad_big_kernel") or name.startswith("wgrad_kernel<bf16"):
        return "wgrad_kernel<bf16,*>"
    return None


def summarise(base):
    fetch = load(base + "_fetch/run_counter_collection.csv", "FETCH_SIZE")
    write = load(base + "_write/run_counter_collection.csv", "WRITE_SIZE")
    for src in (fetch, write):
        for k in list(src):
            a = aggregate(k)
            if a:
                src.setdefault(a, []).extend(src[k])
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        fb = 2.0 * sum(f) / max(1, len(f))
        wb = sum(w) / max(1, len(w))
        res[k] = {"launches": len(f), "fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb}
    return res


SQ = ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
      "SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_INSTS_LDS")


def load_dispatches(path):
    """{dispatch id: {"name", "start", counters...}} from a counter-collection csv."""
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            d = out.setdefault(int(row["Dispatch_Id"]), {"name": row["Kernel_Name"],
                                                          "start": int(row["Start_Timestamp"])})
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return out


def last_step_bytes(base):
    """HBM bytes of the last training step: 2 x FETCH_SIZE + WRITE_SIZE summed over its dispatches."""
    tot = 0.0
    for name, counter, scale in (("fetch", "FETCH_SIZE", 2.0), ("write", "WRITE_SIZE", 1.0)):
        rows = sorted(load_dispatches(base + "_%s/run_counter_collection.csv" % name).values(),
                      key=lambda d: d["start"])
        sgd = [i for i, d in enumerate(rows) if "sgd_mom" in d["name"]]
        if len(sgd) < 2:
            return None
        tot += scale * 1024.0 * sum(d.get(counter, 0.0) for d in rows[sgd[-2] + 1:sgd[-1] + 1])
    return tot


def sq_ratios(acc):
    simd_cycles = acc.get("GRBM_GUI_ACTIVE", 0.0) / 8.0 * 1024.0
    return {"mfma_util": acc.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / simd_cycles if simd_cycles else None,
            "lds_conflict_share": (acc.get("SQ_LDS_BANK_CONFLICT", 0.0) / acc["SQ_LDS_IDX_ACTIVE"]
                                   if acc.get("SQ_LDS_IDX_ACTIVE") else None),
            "mfma_bf16_tflop": acc.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512 / 1e12,
            "busy_ms_at_2.4GHz": acc.get("GRBM_GUI_ACTIVE", 0.0) / 8.0 / 2.4e9 * 1e3}


def summarise_sq(base):
    """Per family (summed over launches) and over the last training step (dispatches between the
    last two SGD launches): MFMA utilisation of the kernels' own busy time, LDS conflict share."""
    path = base + "_sq/run_counter_collection.csv"
    try:
        disp = load_dispatches(path)
    except FileNotFoundError:
        return None
    rows = sorted(disp.values(), key=lambda d: d["start"])
    sgd = [i for i, d in enumerate(rows) if "sgd_mom" in d["name"]]
    fam = collections.defaultdict(lambda: collections.defaultdict(float))
    step = collections.defaultdict(float)
    for i, d in enumerate(rows):
        f = family(d["name"])
        a = aggregate(f)
        for k in SQ:
            fam[f][k] += d.get(k, 0.0)
            if a:
                fam[a][k] += d.get(k, 0.0)
            if len(sgd) >= 2 and sgd[-2] < i <= sgd[-1]:
                step[k] += d.get(k, 0.0)
        fam[f]["launches"] += 1
        if a:
            fam[a]["launches"] += 1
    out = {"families": {k: dict(sq_ratios(v), launches=int(v["launches"])) for k, v in fam.items()}}
    if step:
        out["last_step"] = sq_ratios(step)
    return out


if __name__ == "__main__":
    base = sys.argv[1]
    res = summarise(base)
    sq = summarise_sq(base)
    sb = last_step_bytes(base)
    if sb:
        print("last step HBM bytes (2 x FETCH_SIZE + WRITE_SIZE): %.2f GB" % (sb / 1e9))
    if sq:
        print("last step (kernels serialised under PMC): MFMA util %.3f of the kernels' busy time, "
              "%.1f TFLOP bf16 MFMA, busy %.2f ms at 2.4 GHz, LDS conflict share %.3f" % (
                  sq["last_step"]["mfma_util"], sq["last_step"]["mfma_bf16_tflop"],
                  sq["last_step"]["busy_ms_at_2.4GHz"], sq["last_step"]["lds_conflict_share"] or 0))
        for k, v in sorted(sq["families"].items(), key=lambda kv: -kv[1]["busy_ms_at_2.4GHz"]):
            if v["mfma_util"] is None:
                continue
            print("  %-42s n=%5d MFMA util %.3f  LDS conflict %.3f  busy %.2f ms" % (
                k, v["launches"], v["mfma_util"], v["lds_conflict_share"] or 0, v["busy_ms_at_2.4GHz"]))
        res = {"hbm": res, "sq": sq, "last_step_hbm_bytes": sb}
    hbm = res["hbm"] if sq else res
    for k, v in sorted(hbm.items(), key=lambda kv: -kv[1]["hbm_bytes"] * kv[1]["launches"]):
        print("%-42s n=%5d fetch %9.2f MB  write %9.2f MB  per launch" %
              (k, v["launches"], v["fetch_bytes"] / 1e6, v["write_bytes"] / 1e6))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(res, f, indent=1)
