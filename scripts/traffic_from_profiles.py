"""profiles/traffic.json entries and per-config summaries from the passes of `bash scripts/gpu.sh profile OUT SUB ...`
(SUB: cfg2..cfg5, hbm, slip2, slip3, rs2, rs4 — one directory per leg).

HBM bytes per step-kernel launch = FETCH_SIZE x 2 + WRITE_SIZE (KB = 1024 B), each the mean over the step
kernel's dispatches of its own --pmc pass (gfx950 counts coalesced reads at half: MI355X_MICROARCH.md, HBM
section; calibrated on this kernel at the HBM-resident size, profiles/traffic.json _doc).
    python scripts/traffic_from_profiles.py PROFDIR TAG
"""
import collections
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import summarize_profile as SP  # noqa: E402

B_PER_INSTANCE = {2: 52.5, 3: 57.0, 4: 50.25, 5: 55.0}
AGENTS = {2: 2, 3: 1, 4: 4, 5: 3}


def pmc_mean(d, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, f"pmc_{counter}", "pmc_counter_collection.csv"))):
        if "rmx::step" in r["Kernel_Name"]:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    # the step kernel proper: the most dispatched one (the window's last step, rmx_step_report's RPT
    # instantiation, runs once per window)
    name, vals = max(agg.items(), key=lambda kv: len(kv[1]))
    return name, sum(vals) / len(vals), len(vals)


def main(prof, tag):
    head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                          text=True).stdout.strip()
    tfile = os.path.join(ROOT, "profiles", "traffic.json")
    traffic = json.load(open(tfile))
    for sub, cfg, n in (("cfg2", 2, 65536), ("cfg3", 3, 65536), ("cfg4", 4, 65536), ("cfg5", 5, 65536),
                        ("hbm", 2, 8388608), ("slip2", 2, 65536), ("slip3", 3, 65536), ("rs2", 2, 65536),
                        ("rs4", 4, 65536)):
        d = os.path.join(prof, sub)
        if not os.path.isdir(d):
            continue
        name, fetch_kb, nd = pmc_mean(d, "FETCH_SIZE")
        _, write_kb, _ = pmc_mean(d, "WRITE_SIZE")
        rd, wr = fetch_kb * 2 * 1024, write_kb * 1024
        alg = n * AGENTS[cfg] * B_PER_INSTANCE[cfg]
        if sub.startswith("slip"):  # + the env's PCG64 state: 32 B read, 16 B (state words) written per env-step
            alg += n * 48
        if sub.startswith("rs"):  # random starts (fixed-start cache): + the cached start cells, 4 B per 2 agents per env
            alg += n * 4 * ((AGENTS[cfg] + 1) // 2)
        key = {"hbm": "hbm_diag", "slip2": "config2_slip", "slip3": "config3_slip", "rs2": "config2_randstart",
               "rs4": "config4_randstart"}.get(sub, f"config{cfg}")
        # keep the previous HEAD entry under a round-tagged name
        if key in traffic and traffic[key].get("source", "").split("/")[-1].split("_")[0] != tag:
            traffic[f"{key}_{traffic[key].get('source', 'prev').split('/')[-1].split('_')[0]}"] = traffic[key]
        summary = f"profiles/{tag}_{sub}_step_kernel.md"
        try:  # the source and kernel digests of the library that was profiled (bench.py's "build")
            bi = json.load(open(os.path.join(d, "kt_bench.json"))).get("build", {})
            src, kern = bi.get("src"), bi.get("kern")
        except (OSError, ValueError):
            src = kern = None
        traffic[key] = {"n_envs": n, "bytes_per_launch": rd + wr, "read_bytes": rd, "write_bytes": wr,
                        "algorithmic_bytes": alg, "traffic_over_algorithmic": (rd + wr) / alg, "dispatches": nd,
                        "source": summary, "config": cfg, "kernel": name, "commit": head, "src": src, "kern": kern}
        SP.main(d, os.path.join(ROOT, summary),
                f"{tag} (commit {head}) - default step kernel, BASELINE config {cfg}, {n:,} envs, MI355X")
        print(key, round((rd + wr) / 1e6, 3), "MB", round((rd + wr) / alg, 3))
    json.dump(traffic, open(tfile, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
