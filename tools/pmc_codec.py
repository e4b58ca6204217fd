"""MFMA utilisation of the codec's large-M GEMMs (gemm_glds_kernel, gemm_bf16_kernel) from a
rocprofv3 --pmc pass.

usage: python tools/pmc_codec.py COUNTER_CSV KEY [OUT_JSON]

The pass collects SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (one SQ and one GRBM slot) over
bench.py, whose codec calls all decode the same S x chunk frames. Over every large-M GEMM dispatch:
busy = sum of SQ_VALU_MFMA_BUSY_CYCLES (MFMA-busy cycles summed over the SIMDs, MI355X_MICROARCH.md), active = sum of GRBM_GUI_ACTIVE / 8 (GRBM sums the
8 XCDs), util = busy / (active x 1024 SIMDs). KEY = bench.py's codec key
"<dtype>/F<frames>/L<frames per stream>".
"""
import csv
import json
import os
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    dst = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "pmc_codec.json")
    per = {}
    for r in csv.DictReader(open(path)):
        if "gemm_bf16_kernel" not in r["Kernel_Name"] and "gemm_glds_kernel" not in r["Kernel_Name"]:
            continue
        d = per.setdefault(r["Dispatch_Id"], {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    busy = sum(d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for d in per.values())
    active = sum(d.get("GRBM_GUI_ACTIVE", 0.0) for d in per.values()) / 8.0
    util = busy / (active * 1024.0) if active else None
    res = json.load(open(dst)) if os.path.exists(dst) else {}
    res[key] = {"dispatches": len(per), "mfma_busy_cycles": busy, "active_cycles": active,
                "mfma_util": round(util, 4) if util is not None else None,
                "mfma_flops_equiv": busy * 1024.0}
    print(key, res[key])
    json.dump(res, open(dst, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
