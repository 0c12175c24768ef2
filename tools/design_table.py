"""DESIGN.md §5's table from a profiles run: python tools/design_table.py r7z"""
import json
import sys

pre = sys.argv[1] if len(sys.argv) > 1 else "r7z"
names = {"c1": "reference Simple payload × 65 536", "c2": "65 536 × 196 B flat Simple",
         "c2x": "C2, flags 0x7 (reference benchmark options)", "c2s": "C2, keys shuffled per message",
         "c3": "65 536 × 2.2 KB nested", "c4": "4 096 × 85 KB (48 KiB base64 + 1 024 doubles)",
         "c5": "ONE 1 048 576-message mixed batch (90/9.5/0.5 %)", "t2j-c2": "Thrift of C2 -> JSON",
         "t2j-c3": "Thrift of C3 -> JSON"}
print("| config | workload | step ms (in flight) | GB/s JSON in (serial) | dominant kernel: ms, frac | serial step: ms, frac "
      "| traffic / alg | CPU GB/s: quota cores (n) / all affinity / 1 core |")
print("|---|---|---|---|---|---|---|---|")
for c in ["c1", "c2", "c2x", "c2s", "c3", "c4", "c5", "t2j-c2", "t2j-c3"]:
    try:
        d = json.loads(open(f"profiles/{pre}_{c}_bench.json").read().strip().splitlines()[-1])
    except OSError:
        continue
    r = d["roofline"] or {}
    st = r.get("step") or {"ms": r.get("kernel_ms"), "frac": r.get("frac")}
    cb = d.get("cpu_baseline") or {}
    tr, alg = r.get("traffic"), r.get("alg_bytes_per_launch")
    allv = (cb.get("all_affinity") or {}).get("value")
    cpu = (f"{cb.get('value', 0):.1f} ({cb.get('cores')}) / {'-' if allv is None else round(allv, 1)} / "
           f"{cb.get('one_core_gbs', 0):.2f}") if cb else "-"
    dom = f"{r.get('kernel', '')} {r.get('kernel_ms')}, {r.get('frac')}" if "kernel" in r else "-"
    bold = "**" if c == "c2" else ""
    print(f"| {bold}{c.upper() if c[0] == 'c' else c}{bold} | {names[c]} | {d['ms_per_step']} | "
          f"{bold}{d['value']}{bold} ({d['config'].get('serial_gbs')}) | {dom} | {st.get('ms')}, {st.get('frac')} | "
          f"{round(tr / alg, 2) if tr and alg else '-'} | {cpu} |")
