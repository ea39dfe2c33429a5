"""MFMA utilisation per forward kernel from a rocprofv3 --pmc pass of bench.py with
SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE.

Per dispatch (MI355X_MICROARCH.md, SQ PMC units / DVFS rows): SQ_VALU_MFMA_BUSY_CYCLES counts
MFMA pipe cycles summed over every SIMD; GRBM_GUI_ACTIVE is summed over the 8 XCDs, so the
dispatch's GPU cycles = GRBM_GUI_ACTIVE / 8 and the effective clock = that / duration.
    mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs)
Dispatches are grouped by kernel template (the same kernel at different layers averages).
Usage: python tools/mfma_util.py run_counter_collection.csv [--last N] [--json out.json]"""
import csv
import json
import sys
from collections import defaultdict

FWD = ("stem_", "conv_", "head_pred", "spp_maxpool", "focus_pack", "dwconv")
path = sys.argv[1]
last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 3
disp = defaultdict(dict)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if not any(k in name for k in FWD):
        continue
    d = disp[(int(r["Dispatch_Id"]), name)]
    d[r["Counter_Name"]] = float(r["Counter_Value"])
    d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
# only the last `last` forwards (each starts at its stem launch): autotune candidates and
# warm-up dispatches before them are dropped
stems = sorted(k[0] for k in disp if "stem_" in k[1] and "pack" not in k[1])
first = stems[-last] if len(stems) >= last else 0
disp = {k: v for k, v in disp.items() if k[0] >= first}
fam = defaultdict(lambda: defaultdict(float))
for (_, name), d in disp.items():
    f = fam[name]
    for k, v in d.items():
        f[k] += v
    f["n"] += 1
# optional second pass (--stalls CSV: SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY,
# SQ_INSTS_LDS, ...): where the waves' cycles go, per kernel template (dispatch ids of another run
# differ, so it is matched by name; the whole pass is averaged per dispatch)
stall = defaultdict(lambda: defaultdict(float))
if "--stalls" in sys.argv:
    for r in csv.DictReader(open(sys.argv[sys.argv.index("--stalls") + 1])):
        if any(k in r["Kernel_Name"] for k in FWD):
            stall[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
rows = []
for name, f in fam.items():
    cyc = f["GRBM_GUI_ACTIVE"] / 8
    util = f["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 256 * 4) if cyc else 0.0
    clk = cyc / f["ns"] if f["ns"] else 0.0
    rows.append({"kernel": name[:110], "dispatches": int(f["n"]), "time_us": f["ns"] / 1e3 / last, "mfma_util": util,
                 "clock_ghz": clk, "mfma_insts": f["SQ_INSTS_MFMA"], "valu_insts": f["SQ_INSTS_VALU"],
                 "valu_per_mfma": f["SQ_INSTS_VALU"] / max(f["SQ_INSTS_MFMA"], 1)})
    st = stall.get(name)
    if st and st.get("SQ_WAVE_CYCLES"):
        wc = st["SQ_WAVE_CYCLES"]
        rows[-1].update({"wait_any": st["SQ_WAIT_ANY"] / wc, "wait_inst_any": st["SQ_WAIT_INST_ANY"] / wc,
                         "active_inst_any": st["SQ_ACTIVE_INST_ANY"] / wc,
                         "wait_inst_lds": st.get("SQ_WAIT_INST_LDS", 0.0) / wc,
                         "lds_bank_conflict_cycles": st.get("SQ_LDS_BANK_CONFLICT", 0.0)})
rows.sort(key=lambda r: -r["time_us"])
tot_t = sum(r["time_us"] for r in rows)
tot_busy = sum(fam[n]["SQ_VALU_MFMA_BUSY_CYCLES"] for n in fam)
tot_cyc = sum(fam[n]["GRBM_GUI_ACTIVE"] / 8 for n in fam)
print(f"last {last} forwards; time per forward")
print(f"{'time us':>9} {'share':>6} {'util':>6} {'GHz':>5} {'VALU/MFMA':>9} {'wait':>5} {'stall':>5} {'issue':>5}  kernel"
      "   (wait / stall / issue: SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES)")
for r in rows:
    w = (f"{r['wait_any']:5.0%} {r['wait_inst_any']:5.0%} {r['active_inst_any']:5.0%}" if "wait_any" in r
         else f"{'-':>5} {'-':>5} {'-':>5}")
    print(f"{r['time_us']:9.1f} {r['time_us'] / tot_t:6.1%} {r['mfma_util']:6.1%} {r['clock_ghz']:5.2f} "
          f"{r['valu_per_mfma']:9.1f} {w}  {r['kernel'][:80]}")
print(f"all forward kernels: MFMA utilisation {tot_busy / (tot_cyc * 1024):.1%} (time-weighted)")
if "--json" in sys.argv:
    json.dump({"source": path, "formula": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs)",
               "overall_mfma_util": tot_busy / (tot_cyc * 1024), "kernels": rows},
              open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
