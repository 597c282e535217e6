"""Summarise a rocprofv3 --kernel-trace run of scripts/trace_window.py (K-step windows on the engine's own queue).

    python scripts/summarize_trace.py OUT_DIR CONFIG [--md profiles/x.md] [--json profiles/trace_times.json]

Reads OUT_DIR/kt/kt_kernel_trace.csv (and kt_kernel_stats.csv) and OUT_DIR/tw.json (the probe's own line).  The
step-kernel dispatches are split into windows where a start-to-start gap exceeds 4x the median; per window the first
dispatch (which follows the doorbell on an idle queue) is set apart.  Reported per config, in ns:
  - duration: End - Start of each steady-state dispatch (the CP's timestamps of that packet: the kernel's own time,
    without the boundary to the next dependent dispatch);
  - period: median start-to-start of consecutive dispatches inside a window (the profiled time per step at the bench's
    back-to-back cadence: duration + the dependent-launch boundary), and the windows' (last end - first start) / K;
  - the probe's wall clock per step of the same windows (host clock around each blocking rmx_step_seq).
The JSON entry (per config) feeds bench.py's roofline.avg_launch_us_profile.
"""
import argparse
import csv
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("config", type=int)
    ap.add_argument("--md", default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--commit", default=None)
    ap.add_argument("--kern", default=None)
    a = ap.parse_args()
    rows = []
    name = None
    for r in csv.DictReader(open(os.path.join(a.d, "kt", "kt_kernel_trace.csv"))):
        if "step_fast_kernel" in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            name = r["Kernel_Name"]
    rows.sort()
    s2s = [rows[i + 1][0] - rows[i][0] for i in range(len(rows) - 1)]
    med = statistics.median(s2s)
    windows, cur = [], [rows[0]]
    for i, g in enumerate(s2s):
        if g > 4 * med:
            windows.append(cur)
            cur = []
        cur.append(rows[i + 1])
    windows.append(cur)
    windows = [w for w in windows if len(w) >= 10]
    steady = [e - s for w in windows for s, e in w[1:]]
    first = [w[0][1] - w[0][0] for w in windows]
    period = [w[i + 1][0] - w[i][0] for w in windows for i in range(len(w) - 1)]
    span = [(w[-1][1] - w[0][0]) / len(w) for w in windows]
    pct = lambda v, q: sorted(v)[min(len(v) - 1, int(q * len(v)))]  # noqa: E731
    probe = {}
    pj = os.path.join(a.d, "tw.json")
    if os.path.exists(pj):
        txt = [ln for ln in open(pj).read().splitlines() if ln.startswith("{")]
        probe = json.loads(txt[-1]) if txt else {}
    out = {"config": a.config, "n_envs": probe.get("n_envs", 65536), "kernel": name, "windows": len(windows),
           "dispatches": sum(len(w) for w in windows), "k": probe.get("k"),
           "duration_ns_mean": statistics.mean(steady), "duration_ns_median": statistics.median(steady),
           "duration_ns_p10": pct(steady, 0.1), "duration_ns_p90": pct(steady, 0.9),
           "first_dispatch_ns_median": statistics.median(first),
           "period_ns_median": statistics.median(period), "period_ns_mean": statistics.mean(period),
           "window_span_ns_per_step_median": statistics.median(span),
           "probe_wall_us_per_step_median": probe.get("us_per_step_wall_median"),
           "source": a.md, "commit": a.commit, "kern": a.kern}
    if a.md:
        L = [f"# Kernel trace of K-step queue windows, config {a.config} (scripts/trace_window.py)", "",
             f"`{name}`", "",
             "rocprofv3 --kernel-trace --stats of `scripts/trace_window.py` (windows of K dependent dispatches on the "
             "engine's own AQL queue, one doorbell each, after a 1-s spin-up).", "",
             "| quantity | ns |", "|---|---|"]
        for k in ("duration_ns_mean", "duration_ns_median", "duration_ns_p10", "duration_ns_p90",
                  "first_dispatch_ns_median", "period_ns_median", "period_ns_mean", "window_span_ns_per_step_median"):
            L.append(f"| {k} | {out[k]:.0f} |")
        L += ["", f"windows {out['windows']}, dispatches {out['dispatches']}, K {out['k']}; the probe's own wall clock "
              f"per step of the same windows (no tracer inside the timing, host clock around each blocking call): "
              f"{out['probe_wall_us_per_step_median']} us", ""]
        ks = os.path.join(a.d, "kt", "kt_kernel_stats.csv")
        if os.path.exists(ks):
            L += ["## kernel_stats.csv", "", "| kernel | calls | avg ns | min ns | max ns |", "|---|---|---|---|---|"]
            for r in csv.DictReader(open(ks)):
                L.append(f"| `{r['Name'][:100]}` | {r['Calls']} | {float(r['AverageNs']):.0f} | {r['MinNs']} | "
                         f"{r['MaxNs']} |")
        os.makedirs(os.path.dirname(os.path.abspath(a.md)), exist_ok=True)
        open(a.md, "w").write("\n".join(L) + "\n")
    if a.json:
        allj = json.load(open(a.json)) if os.path.exists(a.json) else {}
        allj[f"config{a.config}"] = out
        json.dump(allj, open(a.json, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
