"""value / ms per step / group us of bench JSON lines: python tools/r5/show.py <files>"""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    r = d.get("roofline") or {}
    pk = r.get("per_kernel_us") or {k: v.get("avg_us") for k, v in r.get("per_kernel", {}).items()}
    print(f"{f:50s} {d.get('value', 0):10.2f} {d.get('ms_per_step', 0):8.4f}  group {pk.get('group')}")
