"""CPU: the controller's taint / untaint walks over a delivered selection (controller.py
_walk / _scale_down_taint / _scale_up) with a stand-in context — the walk reads past the
selection (esc_group_order) only when failed writes used up its slack, never to fetch a node
past the last one it needs."""
import numpy as np

from escalator_amd.controller import Controller


class _Ctx:
    def __init__(self, order):
        self.order, self.calls = order, 0

    def group_order(self, g, which):
        self.calls += 1
        return np.asarray(self.order, np.int64)


class _Act:
    def __init__(self, bad):
        self.bad, self.calls = set(bad), []

    def taint(self, g, j):
        self.calls.append(j)
        return j not in self.bad

    untaint = taint


def _ctl(sel, order, bad, which):
    c = Controller.__new__(Controller)
    c.groups = [{"dry_mode": False}]
    c.ctx, c.actuator = _Ctx(order), _Act(bad)
    c._sel = (np.array([which], np.int32), np.array([0, len(sel)], np.int64), np.asarray(sel, np.int64))
    return c


def test_walk_stops_at_last_needed_node():
    order = [5, 3, 9, 1, 7, 2, 8]
    for slack, bad, fb in ((1, [5], False), (1, [], False), (0, [3], True), (2, [5, 9], False), (1, [5, 9], True)):
        for which in (0, 1):
            c = _ctl(order[:4 + slack], order, bad, which)
            out = {"walk_fallback": False}
            if which == 0:
                c._scale_down_taint(0, 4, len(order), ["n%d" % j for j in range(10)], out)
                got = out["tainted_now"]
            else:
                c._scale_up(0, 4, len(order), ["n%d" % j for j in range(10)], out)
                got = out["untainted_now"]
            want = [j for j in order if j not in set(bad)][:4]
            assert got == want, (slack, bad, which)
            assert c.actuator.calls == order[:order.index(want[-1]) + 1]
            assert out["walk_fallback"] == fb and c.ctx.calls == int(fb), (slack, bad, which)


def test_walk_zero_count_reads_nothing():
    c = _ctl([], [4, 2], [], 0)
    out = {"walk_fallback": False}
    c._scale_down_taint(0, 0, 2, ["a"] * 5, out)
    assert out["tainted_now"] == [] and not out["walk_fallback"] and c.actuator.calls == []
