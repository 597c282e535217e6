"""Per-dispatch time of the default step kernel from a counter pass, for profiles/ and bench.py's roofline.

    python scripts/profile_times.py gpurun_out/r06d --md profiles/r06d_profile_time.md --json profiles/profile_times.json

Reads, per BASELINE config N in 2..5, OUT/ctrN/pmc/**/pmc_counter_collection.csv and pmc_kernel_trace.csv (one
`rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVES` run of
`bench.py --config N`, eager launches, scripts/r06d.sh) and OUT/stamps_edges_N.json (the shader clock measured in-kernel,
s_memtime / s_memrealtime x 100 MHz, on a back-to-back graph: scripts/stamps.py --edges 1).  Per dispatch of the
config's plain step kernel (`step_fast_kernel<..., RPT = false, ...>`):
  - sq_busy_us: SQ_BUSY_CYCLES / the shader engines (rocprofv3's agent info: Array_Count) / the shader clock — the
    time the kernel's waves occupy the shader engines, without the command processor's dispatch set-up and
    end-of-pipe;
  - trace_us: End - Start of the same dispatch in the kernel trace — the profiled dispatch, which under the counter
    pass runs alone on an idle GPU (each dispatch serialized, its counters sampled around it);
  - gui_active_us: GRBM_GUI_ACTIVE / XCDs / clock (equal to GRBM_COUNT here: the counter window, profiler overhead
    included; kept for completeness, not used).
"""
import argparse
import csv
import glob
import json
import os
import statistics

BYTES = {2: 52.5 * 2, 3: 57.0 * 1, 4: 50.25 * 4, 5: 55.0 * 3}  # SURVEY §8(d) B per env-step (x A), bench.py


def one(d, c):
    ctr = os.path.join(d, f"ctr{c}", "pmc")
    vals, dur, name = {}, [], None
    for f in glob.glob(os.path.join(ctr, "**", "pmc_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "step_fast_kernel" in r["Kernel_Name"] and ", false, 0>" in r["Kernel_Name"]:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
                name = r["Kernel_Name"]
    for f in glob.glob(os.path.join(ctr, "**", "pmc_kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"] == name:
                dur.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    agents = [r for r in csv.DictReader(open(glob.glob(os.path.join(ctr, "**", "pmc_agent_info.csv"),
                                                        recursive=True)[0])) if int(r.get("Array_Count") or 0) > 0]
    info = agents[0]  # the GPU agent (the CPU agents report no shader arrays)
    n_se, n_xcc = int(info["Array_Count"]), int(info["Num_Xcc"])
    st = json.load(open(os.path.join(d, f"stamps_edges_{c}.json")))
    ghz = st["shader_clock_ghz_median"]
    sq = statistics.mean(vals["SQ_BUSY_CYCLES"]) / n_se / ghz / 1e3
    return {"config": c, "n_envs": 65536, "kernel": name.split("(")[0] if name else None,
            "dispatches": len(dur), "shader_engines": n_se, "xcc": n_xcc, "shader_clock_ghz": ghz,
            "sq_busy_cycles_per_dispatch": statistics.mean(vals["SQ_BUSY_CYCLES"]),
            "sq_busy_us": sq, "trace_us_median": statistics.median(dur) / 1e3,
            "gui_active_us": statistics.mean(vals["GRBM_GUI_ACTIVE"]) / n_xcc / ghz / 1e3,
            "bytes_per_launch": 65536 * BYTES[c], "frac_sq_busy": 65536 * BYTES[c] / (sq * 1e-6) / 8e12}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--md", default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--commit", default=None)
    ap.add_argument("--kern", default=None)
    a = ap.parse_args()
    rows = [one(a.d, c) for c in (2, 3, 4, 5)]
    for r in rows:
        r.update(source=a.md, commit=a.commit, kern=a.kern)
    if a.json:
        out = {f"config{r['config']}": r for r in rows}
        json.dump(out, open(a.json, "w"), indent=1)
    if a.md:
        L = ["# Per-dispatch time of the default step kernel from a counter pass (configs 2-5, 65,536 envs)", "",
             "`rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVES` of "
             "`bench.py --config N` (eager launches; `scripts/r06d.sh`), the plain step kernel's dispatches; the shader "
             "clock measured in-kernel on a back-to-back graph (`scripts/stamps.py --edges 1`, s_memtime / "
             "s_memrealtime).  `scripts/profile_times.py` wrote this file and `profiles/profile_times.json`.", "",
             "| config | dispatches | shader clock GHz | SQ_BUSY_CYCLES / dispatch | ÷ 32 SEs ÷ clock = waves resident, µs "
             "| traced dispatch (alone on an idle GPU), median µs | algorithmic B / launch | frac of 8 TB/s on the SQ-busy time |",
             "|---|---|---|---|---|---|---|---|"]
        for r in rows:
            L.append(f"| {r['config']} | {r['dispatches']} | {r['shader_clock_ghz']:.3f} | {r['sq_busy_cycles_per_dispatch']:,.0f} | "
                     f"{r['sq_busy_us']:.3f} | {r['trace_us_median']:.3f} | {r['bytes_per_launch']:,.0f} | "
                     f"{r['frac_sq_busy']:.3f} |")
        L += ["", f"Kernel: `{rows[0]['kernel']}` (config 2; the others their own instantiations).  GRBM_GUI_ACTIVE equals "
              "GRBM_COUNT on every dispatch (the counter window, profiler overhead included), so it times the profiler, "
              "not the kernel, and is not used.", ""]
        open(a.md, "w").write("\n".join(L) + "\n")
    print(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
