"""Debug: config 2 decisions vs the C oracle, per run mode; prints mismatching groups."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import escalator_amd as esc
from oracle import soa
s = esc.Synth(1_000_000, 10_000, 100, config=2, seed=0xE5CA1A7E00000002)
otot = soa.totals(s.pods(), s.nodes(), s.groups)
odf, odi = soa.decide(s.groups, s.states, otot)
for graph in (False, True):
    ctx = esc.Context(s)
    ctx.load_synth(s, replicas=2)
    ctx.use_graph(graph)
    ctx.set_state(s.states)
    for it in range(3):
        ctx.run()
        tot, dec = ctx.results()
        bad = np.nonzero(dec["cpu_pct"].view(np.uint64) != odf[:, 0].view(np.uint64))[0]
        badt = np.nonzero(tot["pod_cpu_m"] != otot[:, 0])[0]
        print("graph", graph, "it", it, "bad dec", bad[:20].tolist(), "bad tot", badt[:10].tolist(), flush=True)
        for g in bad[:5]:
            print("  g", g, "gpu", dec[g], "oracle", odf[g], odi[g], "tot", tot[g], flush=True)
