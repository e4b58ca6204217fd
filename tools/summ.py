"""Print the key fields of bench JSON lines (tools/gpu_r5_check.sh outputs)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    sr = d.get("step_roofline") or {}
    par = d.get("parity_mode_fp32") or {}
    print(f, d["value"], "tok/s", d["ms_per_step"], "ms/step | p50", d.get("p50_first_chunk_latency_ms"),
          "loaded", d.get("p50_first_chunk_latency_loaded_ms"), "| step", sr.get("us_per_step"), sr.get("frac"),
          "| parity", par.get("value"), par.get("ratio_to_headline"), "| codec", (d.get("codec_roofline") or {}).get("avg_ms"),
          "| head", d.get("tokens_head"))
