"""MFMA utilisation per kernel from one rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CU_CYCLES and GRBM_GUI_ACTIVE (tools/gpu_r2_mfma.sh).

  util = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x 256 CUs x GRBM_GUI_ACTIVE / 8)

(GRBM_GUI_ACTIVE is summed over the 8 XCDs, MI355X_MICROARCH.md §DVFS; MFMA busy cycles
are counted per SIMD and summed over the chip.) Kernels with fewer than 1e6 MFMA busy
cycles per dispatch are left out.

  python tools/pmc_mfma.py <counter_collection.csv> <out.json>
"""
import csv
import json
import sys
from collections import defaultdict


def main(path, dst):
    per = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for k, c in per.items():
        if not all(n in c for n in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE")):
            continue
        busy = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(c["SQ_VALU_MFMA_BUSY_CYCLES"])
        gui = sum(c["GRBM_GUI_ACTIVE"]) / len(c["GRBM_GUI_ACTIVE"]) / 8
        if busy < 1e6 or gui <= 0:
            continue
        cu = sum(c.get("SQ_BUSY_CU_CYCLES", [0])) / max(len(c.get("SQ_BUSY_CU_CYCLES", [1])), 1)
        rows.append({"kernel": k[:140], "dispatches": len(c["GRBM_GUI_ACTIVE"]),
                     "mfma_busy_cycles": busy, "gui_active_cycles_per_xcd": gui,
                     "mfma_util": round(busy / (1024 * gui), 4),
                     "sq_busy_cu_cycles": cu})
    rows.sort(key=lambda r: -r["mfma_busy_cycles"] * r["dispatches"])
    res = {"formula": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)", "kernels": rows}
    json.dump(res, open(dst, "w"), indent=1)
    for r in rows:
        print(f'{r["mfma_util"]:7.3f}  x{r["dispatches"]:<4d} {r["kernel"][:100]}')


if __name__ == "__main__":
    main(*sys.argv[1:])
