"""In-kernel stamp breakdown of the fast step kernel (diagnostic build only).

Runs K graph-replayed steps of BASELINE config C with RMX_LIB = the RMX_DIAG build and RMX_DIAG_STAMPS set,
then reads the per-wave stamps of the LAST launch (s_memtime shader clocks + s_memrealtime 100 MHz):
  S0 entry | S1 blob granules landed (LDS variant) | S2 staged + block barrier | S3 state loads landed |
  S4 move-word lookups landed | S5 RM lookups landed | S6 step logic done | S7 outputs stored | S8 all
  memory operations of the wave complete
Every stamp waits for all outstanding memory operations first, so the segments are upper bounds of an
un-instrumented wave's phases."""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--n-envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--random-starts", type=int, default=0, help="FrozenLake random_start_positions on the scenario")
    ap.add_argument("--edges", type=int, default=0,
                    help="entry and exit stamps only (diag bit 0x100000): the dispatch span at the graph's cadence")
    ap.add_argument("--samples", type=int, default=1, help="graph replays, the last launch of each read (median)")
    ap.add_argument("--spin-s", type=float, default=1.0, help="untimed replays first (clocks up)")
    args = ap.parse_args()
    os.environ.setdefault("RMX_LIB", os.path.join(ROOT, "multiagent-rl-rm_amd/csrc/build/librmx_diag.so"))
    os.environ["RMX_DIAG_STAMPS"] = "1"
    if args.edges:
        os.environ["RMX_DIAG_BITS"] = str(int(os.environ.get("RMX_DIAG_BITS", "0")) | 0x100000)
    import numpy as np
    import torch

    from rmx import tables as T
    from rmx.engine import VecRMEnv

    desc = dict(T.baseline_scenario(args.config))
    if args.random_starts:
        desc["random_start_positions"] = True
    tab = T.compile_scenario(desc)
    env = VecRMEnv(tab, args.n_envs, with_renv=False)
    assert env.step_variant == "fast", env.step_variant
    out_variant = os.environ.get("RMX_FAST_TABLES", "default")
    K = args.steps
    acts = env.fill_actions(0, 0, K)
    g = torch.cuda.CUDAGraph()
    s0 = torch.cuda.Stream()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        with torch.cuda.graph(g, stream=s0):
            for s in range(K):
                env.step(acts[s])
    torch.cuda.current_stream().wait_stream(s0)
    env.reset()
    import time
    lib = env.lib
    lib.rmx_diag_stamps.restype = C.c_int
    lib.rmx_diag_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    n_waves = (args.n_envs + 255) // 256 * 4
    t_end = time.perf_counter() + args.spin_s
    while time.perf_counter() < t_end:
        g.replay()
        torch.cuda.synchronize()
    spans, clocks, uss, bufs = [], [], [], []
    for _ in range(max(1, args.samples)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        uss.append(e0.elapsed_time(e1) * 1e3 / K)
        buf = np.zeros((n_waves, 18), dtype=np.uint64)
        n = lib.rmx_diag_stamps(env._h, buf.ctypes.data, buf.size)
        assert n == buf.size, n
        clk = buf[:, :9].astype(np.int64)
        rt = buf[:, 9:].astype(np.int64)
        live = rt[:, 8] > 0
        spans.append(float(rt[live, 8].max() - rt[live, 0].min()) * 10.0)  # ns: first wave entry -> last wave done
        clocks.append(float(np.median((clk[live, 8] - clk[live, 0]) / np.maximum(rt[live, 8] - rt[live, 0], 1))) * 0.1)
        bufs.append(buf)
    us = float(np.median(uss))
    buf = bufs[-1]
    clk = buf[:, :9].astype(np.int64)
    rt = buf[:, 9:].astype(np.int64)
    seg = np.diff(clk, axis=1)
    names = ["blob_landed", "stage+barrier", "state_landed", "mv_lookup", "rm_lookup", "compute", "stores",
             "stats+drain"]
    out = {"config": args.config, "tables": out_variant, "n_envs": args.n_envs, "us_per_step_instrumented": us,
           "edges_only": bool(args.edges), "samples": len(spans),
           "dispatch_span_ns_median": float(np.median(spans)), "dispatch_span_ns_min": float(min(spans)),
           "shader_clock_ghz_median": float(np.median(clocks)),
           "realtime_10ns": {"entry_spread_p50": float(np.median(rt[:, 0] - rt[:, 0].min())),
                             "entry_spread_max": float(rt[:, 0].max() - rt[:, 0].min()),
                             "wave_span_median": float(np.median(rt[:, 8] - rt[:, 0])),
                             "first_entry_to_last_exit": float(rt[:, 8].max() - rt[:, 0].min())}}
    if not args.edges:
        out.update({"cycles_median": {k: float(np.median(seg[:, i])) for i, k in enumerate(names)},
                    "cycles_p90": {k: float(np.percentile(seg[:, i], 90)) for i, k in enumerate(names)},
                    "wave_total_cycles_median": float(np.median(clk[:, 8] - clk[:, 0]))})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
