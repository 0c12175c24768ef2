"""DESIGN.md §5's table from a profiles run: python tools/design_table.py r5z"""
import json
import sys

pre = sys.argv[1] if len(sys.argv) > 1 else "r5z"
names = {"c1": "reference Simple payload × 65 536", "c2": "65 536 × 196 B flat Simple",
         "c2x": "C2, flags 0x7 (reference benchmark options)", "c2s": "C2, keys shuffled per message",
         "c3": "65 536 × 2.2 KB nested", "c4": "4 096 × 85 KB (48 KiB base64 + 1 024 doubles)",
         "c5": "ONE 1 048 576-message mixed batch (90/9.5/0.5 %)", "t2j-c2": "Thrift of C2 -> JSON",
         "t2j-c3": "Thrift of C3 -> JSON"}
print("| config | workload | step ms | GB/s JSON in (serial) | kernel ms (serial step) | roofline frac | traffic / alg | "
      "CPU 128-thread / 16 / 1 core GB/s (median; best of 5) |")
print("|---|---|---|---|---|---|---|---|")
for c in ["c1", "c2", "c2x", "c2s", "c3", "c4", "c5", "t2j-c2", "t2j-c3"]:
    try:
        d = json.loads(open(f"profiles/{pre}_{c}_bench.json").read().strip().splitlines()[-1])
    except OSError:
        continue
    r = d["roofline"] or {}
    cb = d.get("cpu_baseline") or {}
    tr, alg = r.get("traffic"), r.get("alg_bytes_per_launch")
    sh = (cb.get("share") or {}).get("value")
    best = (cb.get("range") or {}).get("best_of_5")
    cpu = f"{cb.get('value', 0):.1f} / {sh if sh is None else round(sh, 1)} / {cb.get('one_core_gbs', 0):.2f}"
    if best:
        cpu += f" (best {best:.1f})"
    bold = "**" if c == "c2" else ""
    print(f"| {bold}{c.upper() if c[0] == 'c' else c}{bold} | {names[c]} | {d['ms_per_step']} | "
          f"{bold}{d['value']}{bold} ({d['config'].get('serial_gbs')}) | {r.get('kernel_ms')} | {r.get('frac')} | "
          f"{round(tr / alg, 2) if tr and alg else '-'} | {cpu} |")
