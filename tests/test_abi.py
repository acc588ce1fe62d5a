"""CPU: the C-ABI library loads, exports every symbol the header declares, and its
host-only pieces (packer, generator, scalar decision math) work without a GPU."""
import ctypes as C

import numpy as np

from oracle import soa


def test_library_exports_every_header_symbol():
    from escalator_amd import _lib as L
    lib = L.load()
    fns = L.header_functions()
    assert len(fns) >= 40
    assert [f for f in fns if not hasattr(lib, f)] == []
    assert sorted(set(fns) - set(L._SIGS)) == []
    assert lib.esc_abi_version() == 6


def test_product_library_reads_no_result_changing_knob():
    """The product library's results depend on its inputs alone: the
    only environment variables it names are this allow-list, none of which changes a result
    — host thread counts (ESC_HOST_THREADS, ESC_PACK_PAR_MIN: the packer's and the load's
    parallel passes give identical arrays, test_parallel_packer_equals_sequential), an extra
    self-check of the age index (ESC_CHECK_INDEX) and the multi-device exchange transport
    (ESC_EXCHANGE=peer: the same integer SUM).  The measurement knobs (ESC_K1_VARIANT,
    ESC_K3_ABLATE, ESC_K1_FULL_FLUSH, ESC_POD_SORT, ESC_NO_ZEROCOPY) live in the separate
    measurement library only (Makefile ABLATIONS=1)."""
    import re
    from escalator_amd import _lib as L
    with open(L.LIB_PATH, "rb") as f:
        data = f.read()
    # NUL-terminated literals (what getenv takes), not pieces of mangled names or debug info
    names = set(m.decode() for m in re.findall(rb"(?<![A-Za-z0-9_])(ESC_[A-Z0-9_]{3,})\x00", data))
    assert names <= {"ESC_HOST_THREADS", "ESC_PACK_PAR_MIN", "ESC_CHECK_INDEX", "ESC_EXCHANGE"}, names
    for knob in ("ESC_K1_VARIANT", "ESC_K3_ABLATE", "ESC_ORDER_ABLATE", "ESC_ORDER_FUSED", "ESC_K1_FULL_FLUSH",
                 "ESC_POD_SORT", "ESC_NO_ZEROCOPY", "ESC_ORDER_CHUNK"):
        assert knob.encode() not in data, knob
    # the measurement-only K1 ablations are not linked into the product library
    assert b"launch_pod_reduce_ablation" not in data or not hasattr(L.load(), "launch_pod_reduce_ablation")


def test_status_strings_verbatim():
    from escalator_amd import _lib as L
    lib = L.load()
    assert lib.esc_status_string(1) == b"node count less than the minimum"
    assert lib.esc_status_string(2) == b"node count larger than the maximum"
    assert lib.esc_status_string(3) == b"cannot divide by zero in percent calculation"
    assert lib.esc_status_string(4) == b"negative scale up delta"
    assert lib.esc_status_string(7) == b"decided on the group's owner rank"       # world > 1, not a reference status
    buf = C.create_string_buffer(200)
    lib.esc_taint_error(2, 3, buf, 200)
    assert buf.value == b"the number of nodes(2) is less than specified minimum of 3. Taking no action"


def test_no_device_is_reported_not_faked():
    from escalator_amd import _lib as L
    from escalator_amd.context import Context
    ctx = Context([{"name": "a", "label_key": "k", "label_value": "v"}], device=-1)
    assert ctx.lib.esc_run(ctx.handle) == L.ESC_E_NODEV
    assert ctx.lib.esc_sort_nodes(ctx.handle) == L.ESC_E_NODEV
    assert ctx.lib.esc_set_selections(ctx.handle, 0, 0) == L.ESC_E_NODEV
    import pytest
    with pytest.raises(L.EscError):
        ctx.set_selections(2, 0)


def test_group_interning_matches_oracle_tables():
    from escalator_amd.context import Context
    groups = [{"name": "x", "label_key": "customer", "label_value": "a"},
              {"name": "default", "label_key": "customer", "label_value": "a"},
              {"name": "y", "label_key": "customer", "label_value": "a"},
              {"name": "z", "label_key": "pool", "label_value": "a"}]
    ctx = Context(groups, device=-1)
    t = soa.group_tables(groups)
    assert t["n_gp"] == 2 and list(t["gpair"]) == [0, 0, 0, 1]
    assert ctx.lib.esc_ctx_num_group_pairs(ctx.handle) == t["n_gp"]
    for (k, v), i in t["pair_ids"].items():
        assert ctx.lib.esc_ctx_pair_id(ctx.handle, k.encode(), v.encode()) == i
    assert ctx.lib.esc_ctx_pair_id(ctx.handle, b"customer", b"zz") == 0xFFFFFFFF


def test_synth_shards_are_slices_and_single_pass_equals_reference_shaped():
    from escalator_amd.context import Synth
    full = Synth(200_000, 2_000, 40, config=4, seed=7)
    part = Synth(200_000, 2_000, 40, config=4, seed=7, p_lo=50_000, p_hi=130_000)
    fp, pp = full.pods(), part.pods()
    for k in ("flags", "cpu0", "mem0", "pair0"):
        assert np.array_equal(fp[k][50_000:130_000], pp[k]), k
    for k, v in full.nodes().items():
        assert np.array_equal(v, part.nodes()[k]), k
    tot = soa.totals(fp, full.nodes(), full.groups)
    assert np.array_equal(soa.totals(fp, full.nodes(), full.groups, reference_shaped=True), tot)
    df, di = soa.decide(full.groups, full.states, tot)
    assert len(set(di[:, 5].tolist())) >= 3          # several decision branches exercised
    assert tot[:, 2].sum() > 0 and (tot[:, 12] == 0).all()


def test_synth_mem_milli_within_int64():
    """every bit-exact config keeps each group's mem_sum*1000 < 2^63 (the
    MilliValue() wrap is unpinned).  Checked on a 1/100..1/1000 sample, scaled up."""
    from escalator_amd.context import Synth
    for cfg, P, N, G, full_p, full_n in [(2, 100_000, 1_000, 100, 1_000_000, 10_000),
                                         (3, 100_000, 1_000, 100, 10_000_000, 100_000),
                                         (4, 100_000, 10_000, 10_000, 100_000_000, 1_000_000)]:
        s = Synth(P, N, G, config=cfg, seed=cfg)
        tot = soa.totals(s.pods(), s.nodes(), s.groups)
        pod_scale, node_scale = full_p // P, full_n // N
        # 2x margin for sampling noise on small groups
        assert max(int(x) for x in tot[:, 1]) * pod_scale * 1000 * 2 < 2 ** 63, cfg
        assert max(int(x) for x in tot[:, 4]) * node_scale * 1000 * 2 < 2 ** 63, cfg
