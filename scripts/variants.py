"""Sweep engine launch variants (layout x block size) on the GPU; prints per-step times.

Each variant is a separate handle (RMX_LAYOUT / RMX_BLOCK are read at rmx_create).  Also checks
that every variant ends in the identical state (same actions, same steps).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3,4,5")
    ap.add_argument("--n-envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="fast:64,tpe:256,lpe:256")
    ap.add_argument("--rollout", type=int, default=1)
    ap.add_argument("--qrm", type=int, default=0, help="bind the QRM counterfactual outputs")
    ap.add_argument("--diag", default="", help="comma list of RMX_DIAG_BITS (needs RMX_LIB=diag build)")
    ap.add_argument("--stochastic", type=int, default=0, help="slip dynamics on the BASELINE scenario (generic kernel)")
    ap.add_argument("--random-starts", type=int, default=0, help="FrozenLake random_start_positions on the BASELINE scenario")
    ap.add_argument("--seed-episode-stride", type=int, default=None,
                    help="random starts: the reset-seed schedule's episode stride (0 = the fixed-start cache)")
    ap.add_argument("--rollout-lds", default="", help="RMX_ROLLOUT_LDS for the fast rollout (default: library default)")
    args = ap.parse_args()
    if args.rollout_lds:
        os.environ["RMX_ROLLOUT_LDS"] = args.rollout_lds
    import torch

    from rmx import tables as T
    from rmx.engine import VecRMEnv

    res = []
    for cfg in [int(c) for c in args.configs.split(",")]:
        desc = dict(T.baseline_scenario(cfg))
        if args.stochastic:
            desc["stochastic"] = True
        if args.random_starts:
            desc["random_start_positions"] = True
        if args.seed_episode_stride is not None:
            desc["seed_schedule"] = (1, 1, args.seed_episode_stride)
        tab = T.compile_scenario(desc)
        ref_state = None
        variants = args.variants.split(",")
        if args.diag:
            variants = [f"tpe:256:{d}" for d in args.diag.split(",")]
        for v in variants:
            parts = v.split(":")
            layout, block = parts[0], parts[1]
            # "fast" = the fast step kernel (its workgroup size is the library's default: the block field is ignored);
            # "tpe"/"lpe" = the generic kernels (RMX_FAST=0) at that block size
            # table-mode suffix on "fast": "G" global blob, "M" merged 16-B records, "Q" merged 4-B records; none = the
            # default mode.  Trailing "R" / "T": store mode 2 (rm_q / ep_ret skipped when unchanged) / 3 (the same with
            # non-temporal stores); "S" on a generic variant: skip every unchanged word (RMX_GENERIC_SKIP=1)
            fast = layout.startswith("fast")
            os.environ.pop("RMX_FAST_SKIP", None)
            os.environ.pop("RMX_GENERIC_SKIP", None)
            if fast and layout[-1] in "RT" and len(layout) > 4:
                os.environ["RMX_FAST_SKIP"] = {"R": "2", "T": "3"}[layout[-1]]
                layout = layout[:-1]
            elif not fast and layout.endswith("S"):
                os.environ["RMX_GENERIC_SKIP"] = "1"
                layout = layout[:-1]
            os.environ["RMX_FAST"] = "1" if fast else "0"
            mode = {"G": "global", "M": "merged", "Q": "merged4"}.get(layout[-1] if fast else "", "")
            if mode:
                os.environ["RMX_FAST_TABLES"] = mode
            else:
                os.environ.pop("RMX_FAST_TABLES", None)
            os.environ["RMX_LAYOUT"], os.environ["RMX_BLOCK"] = ("tpe" if fast else layout), block
            if len(parts) > 2:
                os.environ["RMX_DIAG_BITS"] = parts[2]
            env = VecRMEnv(tab, args.n_envs, with_renv=False, with_qrm=bool(args.qrm))
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
            times = []
            for r in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) * 1e3 / K)
            st = env.snapshot()
            if args.diag or (len(parts) > 2 and parts[2] != "0"):
                ref_state = st  # ablated diagnostic kernels compute garbage by design
            if ref_state is None:
                ref_state = st
            else:
                for k in ("pos_x", "pos_y", "rm_q", "flags", "t"):
                    assert (st[k] == ref_state[k]).all(), (cfg, v, k)
            rt = None
            if args.rollout:
                env.reset()
                env.rollout(0, 0, 10)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                env.rollout(0, 10, K)
                e1.record()
                torch.cuda.synchronize()
                rt = e0.elapsed_time(e1) * 1e3 / K
            best = min(times)
            row = {"config": cfg, "variant": v, "us_per_step": best, "median": sorted(times)[len(times) // 2],
                   "Gsteps": args.n_envs * tab.n_agents / best / 1e3, "rollout_us_per_step": rt,
                   "rollout_Gsteps": (args.n_envs * tab.n_agents / rt / 1e3) if rt else None}
            print(json.dumps(row), flush=True)
            res.append(row)
            env.close()
            del g


if __name__ == "__main__":
    main()
