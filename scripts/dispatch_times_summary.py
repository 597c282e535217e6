"""profiles/ summary of a bench detail file's per-dispatch times: the HIP-event time per step beside the command
processor's own dispatch stamps of the same run's queue windows (bench.py cp_dispatch_times) and the committed
counter pass's wave residency, for every config the line timed.

    python scripts/dispatch_times_summary.py gpurun_out/r06k/bench_detail_n1.json --md profiles/r06k_dispatch_times.md
"""
import argparse
import json


def rows(d):
    yield "2", d
    for k, v in (d.get("configs") or {}).items():
        if k != "1":
            yield k, v
    for k, v in (d.get("configs_random_starts") or {}).items():
        yield f"rs{k}", v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("detail")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    d = json.load(open(a.detail))
    L = ["# Per-dispatch time of the step kernel: events, command-processor stamps, counter residency", "",
         f"From `{a.detail}` (`bench.py`, N = 1, K = {d.get('steps')}; build {d.get('build')}).  Events: HIP events over "
         "a K-step graph of plain steps (the roofline's `avg_launch_us`).  CP stamps: three more K-step queue windows "
         "after the timed ones with `rmx_queue_timing(50)` on — packets 0, 50, ... and the last stamped by the command "
         "processor — the span from packet 0's start to the last packet's start / (K - 1) (`avg_launch_us_profile`), "
         "and a stamped dispatch's own end - start (it carries a completion signal: ~1.2 us more).  SQ: the committed counter pass's waves-resident time (`profiles/profile_times.json`).",
         "",
         "| config | wall per step, timed windows | wall per step, CP-timed windows | events per step | CP span per dispatch "
         "| a stamped dispatch (end - start) | SQ residency | frac (events) | frac_profile (CP) | frac_sq | frac_profile / frac |",
         "|---|---|---|---|---|---|---|---|---|---|---|"]
    out = []
    for name, v in rows(d):
        r = v.get("roofline") or {}
        cp = r.get("cp_timing") or {}
        f, fp = r.get("frac"), r.get("frac_profile")
        out.append({"config": name, "ms_per_step": v.get("ms_per_step"), "cp": cp, "roofline": {
            k: r.get(k) for k in ("avg_launch_us", "avg_launch_us_profile", "avg_launch_us_sq",
                                  "frac", "frac_profile", "frac_sq")}})

        def fmt(x, p=3):
            return "—" if x is None else f"{x:.{p}f}"
        L.append(f"| {name} | {fmt(v.get('ms_per_step') and v['ms_per_step'] * 1e3)} | "
                 f"{fmt(cp.get('wall_us_per_step_timed'))} | {fmt(r.get('avg_launch_us'))} | "
                 f"{fmt(r.get('avg_launch_us_profile'))} | {fmt(cp.get('stamped_dispatch_us'))} | "
                 f"{fmt(r.get('avg_launch_us_sq'))} | {fmt(f)} | {fmt(fp)} | {fmt(r.get('frac_sq'))} | "
                 f"{fmt(fp / f if f and fp else None, 2)} |")
    L.append("")
    if a.md:
        open(a.md, "w").write("\n".join(L) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
