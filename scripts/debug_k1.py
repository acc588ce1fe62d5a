"""Ad-hoc GPU check: K1 totals vs the C oracle across group counts / modes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import escalator_amd as esc  # noqa: E402
from oracle import soa  # noqa: E402

for (P, N, G, cfg) in [(2_000_000, 20_000, 10_000, 4), (2_000_000, 20_000, 100, 4), (500_000, 20_000, 10_000, 4)]:
    s = esc.Synth(P, N, G, config=cfg, seed=0xE5CA1A7E00000000 + cfg)
    otot = soa.totals(s.pods(), s.nodes(), s.groups)
    for mode, reps in (("plain", 1), ("plain", 2), ("graph", 1), ("graph", 2), ("wide", 1)):
        ctx = esc.Context(s)
        ctx.load_synth(s, replicas=reps)
        ctx.set_state(s.states)
        if mode == "graph":
            ctx.use_graph(True)
        if mode == "wide":
            ctx.force_wide(True)
        for it in range(3):
            ctx.run()
            tot, dec = ctx.results()
            bad = np.nonzero(tot["pod_cpu_m"] != otot[:, 0])[0]
            badn = np.nonzero(tot["n_pods"] != otot[:, 2])[0]
            print(P, G, cfg, mode, reps, it, "bad cpu", len(bad), "bad n", len(badn), "nblk", ctx.lib and "",
                  tot["pod_cpu_m"][:2].tolist(), otot[:2, 0].tolist(), tot["n_pods"][:2].tolist(), otot[:2, 2].tolist(),
                  flush=True)
