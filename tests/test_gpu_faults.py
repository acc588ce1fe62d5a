"""GPU: forced failures fail loudly and recover.

The measurement library (make -C escalator_amd/csrc ABLATIONS=1) carries fault-injection
entry points the product library lacks (esc_debug_lookback_fail, esc_debug_fail_patches); each
scenario runs in a child process on it (tests/fault_child.py):
  - order: a split ordering's bounded look-back gives up -> esc_sync returns ESC_E_ORDER
    once, esc_group_order refuses that ordering, totals / decisions stay exact, and the next
    ordering (in the step or esc_sort_nodes) is exact — the error word does not stick;
  - listing: the age index's listing gives up -> the build returns ESC_E_HIP, the next
    build is exact;
  - patch: node events whose device writes fail after the host mirrors changed ->
    decisions refused (ESC_E_STATE) until esc_load_nodes, exact after it."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
MEASURE = os.path.join(ROOT, "escalator_amd", "libescalator_hip_measure.so")
ESC_E_HIP, ESC_E_STATE, ESC_E_ORDER = -2, -5, -8


def run_child(mode):
    assert os.path.exists(MEASURE), "build the measurement library: make -C escalator_amd/csrc ABLATIONS=1"
    env = dict(os.environ, ESC_LIB_PATH=MEASURE)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "fault_child.py"), mode], capture_output=True,
                       text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])


def test_ordering_lookback_give_up_reported_and_recovered():
    r = run_child("order")
    assert r["sync_rc"] == ESC_E_ORDER and r["sync_again_rc"] == 0, r
    assert r["group_order_rc"] == ESC_E_ORDER, r
    assert r["results_exact"], r
    assert r["next_sync_rc"] == 0 and r["next_orders_exact"], r
    assert r["sort_sync_rc"] == ESC_E_ORDER and r["sort_next_rc"] == 0 and r["sort_orders_exact"], r


def test_listing_lookback_give_up_fails_the_build():
    r = run_child("listing")
    assert r["build_rc"] == ESC_E_HIP and r["build_again_rc"] == 0, r
    assert r["sync_rc"] == 0 and r["orders_exact"], r


def test_node_events_failed_apply_mark_stale_until_reload():
    r = run_child("patch")
    for tag in ("update", "add", "delete"):
        assert r[tag + "_rc"] == ESC_E_HIP, (tag, r)                 # the failed apply
        assert r[tag + "_refused_rc"] == ESC_E_STATE, (tag, r)       # stale: no decision on it
        assert r[tag + "_reload_rc"] == 0 and r[tag + "_after_rc"] == 0, (tag, r)
        assert r[tag + "_exact"], (tag, r)
