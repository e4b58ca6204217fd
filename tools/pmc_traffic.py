"""Per-launch HBM traffic of bench.py's probed kernels from rocprofv3 --pmc passes.

usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV DTYPE [OUT_JSON]

bench.py's roofline probe (``probe_kernels``) runs passes over the ops k = 0..5 (one untimed
capture pass, then the timed ones), each op one ``ar_rowinfo_init_kernel`` + 200 launches (a
replayed graph); the rowinfo-init dispatches delimit the segments and the last pass's segments
are used.  Bytes per launch = counter sum over the segment / 200.

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
    """{op: (bytes per launch, kernel names, launches)} over the timed probe segments (those with
    ITERS launches after an ar_rowinfo_init_kernel marker); an op with no kernel of its own at this
    B (the mlp c_proj of the fused MLP) has no segment and is reported with 0 launches."""
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    marks = [i for i, r in enumerate(rows) if "ar_rowinfo_init_kernel" in r["Kernel_Name"]] + [len(rows)]
    timed = []
    for a, b in zip(marks[:-1], marks[1:]):
        seg = [r for r in rows[a + 1:b] if not r["Kernel_Name"].startswith("__amd")]
        # a probe segment starts with ITERS launches of one op = ITERS x (1 kernel, or 2 kernels
        # alternating: rows + GEMM, merge + GEMM); anything after it (the codec probe behind the
        # last op) is cut off; decode-loop segments and warm-ups (10 launches) do not qualify
        nm = [r["Kernel_Name"] for r in seg]
        if len(nm) >= ITERS and all(x == nm[0] for x in nm[:ITERS]):
            timed.append(seg[:ITERS])
        elif (len(nm) >= 2 * ITERS and nm[0] != nm[1] and all(nm[2 * i] == nm[0] for i in range(ITERS))
              and all(nm[2 * i + 1] == nm[1] for i in range(ITERS))):
            timed.append(seg[:2 * ITERS])
    fused = any("mlp_fused" in r["Kernel_Name"] for t in timed for r in t[:1])
    timed = timed[-5:] if fused else timed[-6:]  # the fused MLP: five probed ops
    ops = list(range(6)) if len(timed) == 6 else [0, 1, 2, 3, 5]
    out = {k: (0.0, [], 0) for k in range(6)}
    for k, seg in zip(ops, timed[-len(ops):]):
        out[k] = (sum(float(r["Counter_Value"]) for r in seg) * 1024.0 / ITERS,
                  sorted({r["Kernel_Name"].split("(")[0] for r in seg}), len(seg))
    return out


def main():
    fetch, write, dtype = sys.argv[1], sys.argv[2], sys.argv[3]
    dst = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "pmc_traffic.json")
    f, w = segments(fetch, "FETCH_SIZE"), segments(write, "WRITE_SIZE")
    res = json.load(open(dst)) if os.path.exists(dst) else {}
    names = dict(KNAMES)
    if f[4][2] == 0:  # mlp c_proj has no kernel of its own (fused MLP at this B)
        names[3] = "ar_mlp fused (c_fc+gelu+c_proj)"
    for k in range(6):
        if f[k][2] == 0:
            continue
        byts = 2.0 * f[k][0] + w[k][0]
        res[f"{dtype}:{names[k]}"] = round(byts)
        print(f"{names[k]:32s} fetch {2 * f[k][0] / 1e6:8.3f} MB  write {w[k][0] / 1e6:8.3f} MB  "
              f"launches/segment {f[k][2]}  kernels {f[k][1]}")
    json.dump(res, open(dst, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
