"""Kernel durations of bench.py's roofline probe from a rocprofv3 --kernel-trace CSV of the same
bench command: the probe's 200-launch segments (delimited as in tools/pmc_traffic.py), last pass,
per op: the traced average duration of each kernel, the op's launch period (first start to last
end / 200, the HIP-event quantity bench.py reports as avg_us) and the gap between launches.
usage: python tools/probe_trace.py KERNEL_TRACE_CSV"""
import csv
import sys

KNAMES = {0: "ar_gemv c_attn", 1: "ar_attn (split-KV decode)", 2: "ar_gemv c_proj(+merge)",
          3: "ar_gemv c_fc(+gelu)", 4: "ar_gemv mlp.c_proj", 5: "ar_gemv lm_head"}
ITERS = 200


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "ar_rowinfo_init_kernel" in r["Kernel_Name"]] + [len(rows)]
    timed = []
    for a, b in zip(marks[:-1], marks[1:]):
        seg = [r for r in rows[a + 1:b] if not r["Kernel_Name"].startswith("__amd")]
        nm = [r["Kernel_Name"] for r in seg]
        if len(nm) >= ITERS and all(x == nm[0] for x in nm[:ITERS]):
            timed.append(seg[:ITERS])
        elif (len(nm) >= 2 * ITERS and nm[0] != nm[1] and all(nm[2 * i] == nm[0] for i in range(ITERS))
              and all(nm[2 * i + 1] == nm[1] for i in range(ITERS))):
            timed.append(seg[:2 * ITERS])
    fused = any("mlp_fused" in r["Kernel_Name"] for t in timed for r in t[:1])
    ops = [0, 1, 2, 3, 5] if fused else list(range(6))
    timed = timed[-len(ops):]
    print(f"{'op':28s} {'kernel':44s} {'traced avg us':>13s} {'period us':>10s}")
    for k, seg in zip(ops, timed):
        per = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3 / ITERS
        by = {}
        for r in seg:
            by.setdefault(r["Kernel_Name"].split("(")[0], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for i, (n, d) in enumerate(sorted(by.items())):
            print(f"{KNAMES[k] if i == 0 else '':28s} {n[-44:]:44s} {sum(d) / len(d) / 1e3:13.2f} {per if i == 0 else float('nan'):10.2f}")


if __name__ == "__main__":
    main()
