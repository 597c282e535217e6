"""Summarise a scripts/profile.sh output directory into one markdown file (for profiles/)."""
import collections
import csv
import json
import os
import sys


def main(d, out, title):
    lines = [f"# {title}", ""]
    ks = os.path.join(d, "kt", "kt_kernel_stats.csv")
    lines += ["## rocprofv3 --kernel-trace --stats (kernel_stats.csv)", "", "| kernel | calls | avg ns | min ns | max ns | % |",
              "|---|---|---|---|---|---|"]
    for r in csv.DictReader(open(ks)):
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs']):.0f} | {r['MinNs']} | {r['MaxNs']} | "
                     f"{float(r['Percentage']):.2f} |")
    lines.append("")
    kt = os.path.join(d, "kt", "kt_kernel_trace.csv")
    if os.path.exists(kt):
        # per-dispatch distribution of the step kernels: the mean is pulled up by the profiler's per-dispatch
        # completion handling; start-to-start is the profiled launch cadence
        spans = collections.defaultdict(list)
        for r in csv.DictReader(open(kt)):
            if "step" in r["Kernel_Name"] and "rmx::" in r["Kernel_Name"]:
                spans[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        if spans:
            lines += ["## step-kernel dispatch durations under --kernel-trace (ns)", "",
                      "| kernel | dispatches | mean | p10 | median | p90 | median start-to-start |",
                      "|---|---|---|---|---|---|---|"]
            for k, v in spans.items():
                v.sort()
                dur = sorted(e - s for s, e in v)
                s2s = sorted(v[i + 1][0] - v[i][0] for i in range(len(v) - 1)) or [0]
                pct = lambda a, q: a[min(len(a) - 1, int(q * len(a)))]
                lines.append(f"| `{k[:90]}` | {len(v)} | {sum(dur) / len(dur):.0f} | {pct(dur, 0.1)} | "
                             f"{pct(dur, 0.5)} | {pct(dur, 0.9)} | {pct(s2s, 0.5)} |")
            lines.append("")
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = os.path.join(d, f"pmc_{c}", "pmc_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
        lines += [f"## --pmc {c} (KB per dispatch, separate pass)", "", "| kernel | dispatches | mean KB |", "|---|---|---|"]
        for k, v in agg.items():
            if "rmx::" in k:
                lines.append(f"| `{k[:90]}` | {len(v)} | {sum(v) / len(v):.1f} |")
        lines.append("")
    bj = os.path.join(d, "kt_bench.json")
    if os.path.exists(bj):
        txt = [l for l in open(bj).read().splitlines() if l.startswith("{")]
        if txt:
            lines += ["## bench.py line of the profiled (kernel-trace) run", "", "```json", txt[-1], "```", ""]
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
