"""The B-opt CPU baseline (orc_totals_par, OpenMP) equals the single-thread oracle pass
for any thread count, including shards of the node range and tiny inputs."""
import numpy as np
import pytest

from oracle import soa


@pytest.mark.parametrize("threads", [1, 2, 3, 7])
@pytest.mark.parametrize("P,N,G,cfg", [(50_000, 2_000, 64, 2), (20_000, 3_000, 100, 3), (5, 3, 8, 4)])
def test_totals_par_equals_single_pass(threads, P, N, G, cfg):
    import escalator_amd as esc
    s = esc.Synth(P, N, G, config=cfg, seed=0xE5CA1A7E00000000 + cfg, threads=2)
    a = soa.totals(s.pods(), s.nodes(), s.groups)
    b = soa.totals(s.pods(), s.nodes(), s.groups, threads=threads)
    assert np.array_equal(a, b)
    lo, hi = N // 3, N - N // 5
    a = soa.totals(s.pods(), s.nodes(), s.groups, node_lo=lo, node_hi=hi)
    b = soa.totals(s.pods(), s.nodes(), s.groups, node_lo=lo, node_hi=hi, threads=threads)
    assert np.array_equal(a, b)
