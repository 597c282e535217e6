"""Diagnostic (not product): one rmx_step_seq window with the process map written first, so that a crash under a
profiler's queue interception can be placed (frames -> mapped objects).  gpurun_out/<dir>/maps.txt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))
out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
import torch  # noqa: E402
from rmx import tables as T  # noqa: E402
from rmx.engine import VecRMEnv  # noqa: E402

env = VecRMEnv(T.compile_scenario(T.baseline_scenario(2)), 65536)
acts = env.fill_actions(0, 0, 20)
env.step(acts[0])
torch.cuda.synchronize()
with open("/proc/self/maps") as f, open(os.path.join(out, "maps.txt"), "w") as g:
    g.write(f.read())
print("maps written", flush=True)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1
for w in range(n):
    print("window", w, flush=True)
    env.step_seq(acts)
print("windows done", env.queue_counters(), flush=True)
