"""Sum rocprofv3 --pmc counters per kernel (name pattern groups) from *_counter_collection.csv
files. usage: python tools/pmc_sum.py out.json csv [csv ...]
Derived: mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs);
valu/mfma/lds instruction ratios; LDS bank-conflict share of LDS-array cycles."""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(\w+_kernel)(?:I|<|\()", name) or re.search(r"(\w+_kernel)", name)
    k = m.group(1) if m else name[:40]
    k = re.sub(r"^_ZN\d+_GLOBAL__N_1\d+", "", k)
    k = re.sub(r"^\d+", "", k)
    g = re.search(r"GCfg<([^>]*)>", name) or re.search(r"GCfgILi(\d)ELi(\d)ELi(\d)ELi(\d)", name)
    if g:
        k += "[" + ",".join(x.strip() for x in g.groups() if x) + "]" if g.lastindex and g.lastindex > 1 else "[" + g.group(1).replace(" ", "") + "]"
    wp = re.search(r"WPGeoILi(\d+)E", name)
    if wp:
        k += f"<W{wp.group(1)}>"
    kind = re.search(r"conv_glds_kernelI(\w+?)Li(\d)E", name)
    if kind:
        k += f"<{kind.group(1)},{kind.group(2)}>"
    return k


out = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((path, r.get("Dispatch_Id", r.get("Correlation_Id"))))
res = {}
for k, c in acc.items():
    d = dict(c)
    d["dispatches"] = len(disp[k])
    if c.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        # MFMA pipe busy share of the SIMD cycles: GRBM_GUI_ACTIVE sums the 8 XCDs' cycle counts
        d["mfma_util"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
    if c.get("SQ_INSTS_MFMA"):
        for x in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SALU"):
            if x in c:
                d[x.replace("SQ_INSTS_", "").lower() + "_per_mfma"] = round(c[x] / c["SQ_INSTS_MFMA"], 3)
    if c.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in c:
        d["lds_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
    if c.get("SQ_WAVE_CYCLES"):
        for x in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_ANY"):
            if x in c:
                d[x.lower() + "_frac"] = round(c[x] / c["SQ_WAVE_CYCLES"], 4)
    res[k] = d
json.dump(res, open(out, "w"), indent=1, sort_keys=True)
for k in sorted(res, key=lambda k: -res[k].get("GRBM_GUI_ACTIVE", 0))[:30]:
    d = res[k]
    print(f"{k[:60]:60s} n={d['dispatches']:4d} mfma_util={d.get('mfma_util', '-')} "
          f"valu/mfma={d.get('valu_per_mfma', '-')} lds/mfma={d.get('lds_per_mfma', '-')} "
          f"ldsconf={d.get('lds_conflict_frac', '-')} wait={d.get('sq_wait_any_frac', '-')} "
          f"waitinst={d.get('sq_wait_inst_any_frac', '-')}")
