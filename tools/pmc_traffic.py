"""Per-launch HBM traffic of bench.py's probed kernels from rocprofv3 --pmc passes.

usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV DTYPE [OUT_JSON]

bench.py's roofline probe (``probe_kernels``) runs, for each op k = 0..5, one
``ar_rowinfo_init_kernel`` + 10 warm launches, then one ``ar_rowinfo_init_kernel`` + 200 timed
launches.  The last 12 rowinfo-init dispatches therefore delimit the probe segments; the
timed segment of op k is the (2k+1)-th.  Bytes per launch = counter sum over the segment / 200.

Corrections (MI355X_MICROARCH.md, "HBM"): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE counts half the bytes of a 16-B/lane coalesced read, so it is doubled; WRITE_SIZE
is taken as is.  Our loads on these kernels are 16 B/lane.
"""
import csv
import json
import os
import sys

KNAMES = {0: "ar_gemv c_attn", 1: "ar_attn (split-KV decode)", 2: "ar_gemv c_proj(+merge)",
          3: "ar_gemv c_fc(+gelu)", 4: "ar_gemv mlp.c_proj", 5: "ar_gemv lm_head"}
ITERS = 200


def segments(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    marks = [i for i, r in enumerate(rows) if "ar_rowinfo_init_kernel" in r["Kernel_Name"]][-12:]
    out = {}
    for k in range(6):
        a = marks[2 * k + 1] + 1
        b = marks[2 * k + 2] if 2 * k + 2 < len(marks) else len(rows)
        seg = [r for r in rows[a:b] if not r["Kernel_Name"].startswith("__amd")]
        out[k] = (sum(float(r["Counter_Value"]) for r in seg) * 1024.0 / ITERS,
                  sorted({r["Kernel_Name"] for r in seg}), len(seg))
    return out


def main():
    fetch, write, dtype = sys.argv[1], sys.argv[2], sys.argv[3]
    dst = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "pmc_traffic.json")
    f, w = segments(fetch, "FETCH_SIZE"), segments(write, "WRITE_SIZE")
    res = json.load(open(dst)) if os.path.exists(dst) else {}
    for k in range(6):
        byts = 2.0 * f[k][0] + w[k][0]
        res[f"{dtype}:{KNAMES[k]}"] = round(byts)
        print(f"{KNAMES[k]:28s} fetch {2 * f[k][0] / 1e6:8.3f} MB  write {w[k][0] / 1e6:8.3f} MB  "
              f"launches/segment {f[k][2]}  kernels {f[k][1]}")
    json.dump(res, open(dst, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
