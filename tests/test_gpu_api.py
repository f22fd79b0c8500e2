"""C-ABI contract details through the HIP engine (include/svtrek_gpu.h): gather records,
launch ordering across streams, multi-device contexts, device selection, and the event
walk's work counters (the roofline's algorithmic bytes)."""
import numpy as np
import oracle_ffi as O
import pytest
import torch

from svtrek_amd import Engine, Params, sim
from svtrek_amd._lib import LOCUS_DTYPE, RECORD_DTYPE, RESULT_DTYPE

pytestmark = pytest.mark.gpu


def _workload(n_loci=3000, seed=61):
    cfg = sim.SimConfig(seed=seed, n_targets=2, n_loci=n_loci, del_frac=0.5, coverage=25.0)
    return sim.generate(cfg)


def _same(got, want):
    bad = np.nonzero((got["start"] != want["start"]) | (got["end"] != want["end"]))[0]
    assert len(bad) == 0, f"{len(bad)} loci differ; first #{bad[0]}: {got[bad[0]]} vs {want[bad[0]]}"


def test_records_output(engine_factory):
    """svt_refine_device_records: {row index, start, end, 0} per locus, same results."""
    r = _workload()
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    n = len(r.loci)
    want = eng.refine(r.loci)
    d_loci = torch.from_numpy(r.loci.view(np.uint8).copy()).cuda()
    idx = np.random.default_rng(0).permutation(n).astype(np.uint32)
    d_idx = torch.from_numpy(idx.view(np.int32)).cuda()
    d_rec = torch.full((n * 4,), -1, dtype=torch.int32, device="cuda")
    eng.refine_device_records(d_loci.data_ptr(), n, d_rec.data_ptr(), d_idx.data_ptr())
    eng.sync()
    rec = d_rec.cpu().numpy().view(RECORD_DTYPE)
    assert np.array_equal(rec["index"], idx) and (rec["pad"] == 0).all()
    _same(rec, want)
    eng.refine_device_records(d_loci.data_ptr(), n, d_rec.data_ptr(), None, 1000)
    eng.sync()
    rec = d_rec.cpu().numpy().view(RECORD_DTYPE)
    assert np.array_equal(rec["index"], np.arange(1000, 1000 + n, dtype=np.uint32))
    _same(rec, want)


def test_launches_on_two_streams_stay_ordered(engine_factory):
    """Launches of one context on two streams share its spill pool: the context orders them
    (a window with > 256 candidates spills in every launch here), so both stay exact."""
    from fuzz import cluster_pileup
    from svtrek_amd import make_loci
    vals = [500000 + (i * 37) % 600 for i in range(2000)]
    pl = cluster_pileup(vals)
    eng = engine_factory()
    eng.load_pileup(pl)
    loci = make_loci([(2, 1, 500100 + k, 510000 + k) for k in range(64)] + [(1, 1, 500300, 500300)] * 8)
    want = O.refine_batch(pl, loci)
    d_loci = torch.from_numpy(loci.view(np.uint8).copy()).cuda()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [torch.empty(len(loci) * 8, dtype=torch.uint8, device="cuda") for _ in range(6)]
    for k, o in enumerate(outs):
        eng.refine_device(d_loci.data_ptr(), len(loci), o.data_ptr(), (s1 if k % 2 else s2).cuda_stream)
    eng.sync(s1.cuda_stream)
    eng.sync(s2.cuda_stream)
    torch.cuda.synchronize()
    for o in outs:
        _same(o.cpu().numpy().view(RESULT_DTYPE), want)


def test_multi_device_context_splits_batches():
    """svt_open_multi: the pileup is replicated, host batches are split into contiguous
    slices, one per device, results in input order.  On a one-GPU box both contexts sit on
    device 0 (independent contexts), which exercises the same split/merge path."""
    ndev = torch.cuda.device_count()
    devices = list(range(min(ndev, 4))) if ndev > 1 else [0, 0]
    r = _workload(n_loci=2501, seed=62)
    want = O.refine_batch(r.pileup, r.loci, threads=8)
    with Engine(Params(), devices=devices) as eng:
        assert eng.n_devices == len(devices)
        eng.load_pileup(r.pileup)
        _same(eng.refine(r.loci), want)
        w = eng.count_work(r.loci)
        _, ow = O.refine_batch(r.pileup, r.loci, threads=8, with_work=True)
        assert (w["windows"], w["reads"], w["ops_walked"], w["candidates"]) == \
            (ow["windows"], ow["reads"], ow["ops_walked"], ow["candidates"])
        _same(eng.refine(r.loci[:3]), want[:3])   # fewer loci than devices


def test_entry_points_restore_current_device(engine_factory):
    """Every svt_* call selects its context's device and gives the thread its device back."""
    r = _workload(n_loci=200, seed=63)
    eng = engine_factory()
    torch.cuda.set_device(0)
    before = torch.cuda.current_device()
    eng.load_pileup(r.pileup)
    eng.refine(r.loci)
    assert torch.cuda.current_device() == before


def test_span_walk_counters(engine_factory):
    """svt_work's span-walk counters (the default gather): event_bytes = their sum at the
    documented sizes, the reference work equals the oracle's."""
    r = _workload(n_loci=4000, seed=65)
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    w = eng.count_work(r.loci)
    n = len(r.loci)
    _, ow = O.refine_batch(r.pileup, r.loci, threads=8, with_work=True)
    assert (w["windows"], w["reads"], w["ops_walked"], w["candidates"]) == \
        (ow["windows"], ow["reads"], ow["ops_walked"], ow["candidates"])
    assert 0 < w["span_bounds"] <= w["queries"] <= w["windows"]
    assert w["span_events"] >= w["candidates"] * 0.5
    assert w["range_reads"] == 0 and w["list_entries"] == 0
    assert eng.load_stats()["bucket_index"] == 1
    # the value buckets (the default): every window of the default parameters is answered from them,
    # reading its band's buckets (and, when the vote needs ABOVE, the bounded walks) -- a fraction of
    # the span walk's events
    assert 0.99 * w["queries"] <= w["bucket_queries"] <= w["queries"]
    assert 0 < w["bucket_events"] < w["span_events"]
    assert w["event_bytes"] == 24 * n + 12 * w["bucket_queries"] + 16 * w["bucket_events"]
    assert w["event_bytes"] < 24 * n + 12 * w["reads"] + 4 * w["ops_walked"]
    _same(eng.refine(r.loci), O.refine_batch(r.pileup, r.loci, threads=8))


def test_span_list_counters(engine_factory):
    """SVTREK_INDEX=lists (the span lists alone, rounds 1-5): no bucket counters, event_bytes the
    span walk's own bytes, same results."""
    r = _workload(n_loci=4000, seed=65)
    eng = engine_factory(env={"SVTREK_INDEX": "lists"})
    eng.load_pileup(r.pileup)
    assert eng.load_stats()["bucket_index"] == 0
    w = eng.count_work(r.loci)
    n = len(r.loci)
    assert w["bucket_queries"] == 0 and w["bucket_events"] == 0
    exp = (24 * n + 32 * w["queries"] + 4 * w["probe_entries"] + 36 * w["stop_searches"]
           + 4 * w["stop_chunk_words"] + 16 * w["span_bounds"] + 16 * w["span_events"])
    assert w["event_bytes"] == exp
    _same(eng.refine(r.loci), O.refine_batch(r.pileup, r.loci, threads=8))


def test_lane_count_lane_redo_counters(engine_factory):
    """a lane launch, a counting launch, then a smaller lane launch -- the
    third must start its left-over list from zero (two counters alternating on lane launches
    only), so no stale window of the first batch is re-run out of bounds.  Forced lane kernel
    (SVTREK_LANE_W) at both sizes; every result checked against the oracle."""
    r = _workload(n_loci=6000, seed=66)
    prm = Params(consensus_min_count=1)   # more windows with big bands -> left-overs in every launch
    eng = engine_factory(prm, gather="span")   # lane kernel<32> at every batch size
    eng.load_pileup(r.pileup)
    big, small = r.loci, r.loci[: len(r.loci) // 5]
    want_big = O.refine_batch(r.pileup, big, prm, threads=8)
    want_small = O.refine_batch(r.pileup, small, prm, threads=8)
    for _ in range(2):
        _same(eng.refine(big), want_big)
        eng.count_work(big)
        _same(eng.refine(small), want_small)
        eng.count_work(small)
        eng.count_work(big)
        _same(eng.refine(small), want_small)


def test_reindex_keeps_results(engine_factory):
    """svt_reindex rebuilds the device index in place (bench.py's step): results before and
    after, and after several rebuilds interleaved with refines, equal the oracle's."""
    import torch
    r = _workload(n_loci=3000, seed=67)
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    want = O.refine_batch(r.pileup, r.loci, threads=8)
    _same(eng.refine(r.loci), want)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        eng.reindex(s)
    eng.sync(s)
    _same(eng.refine(r.loci), want)
    eng.reindex()
    _same(eng.refine(r.loci), want)


def test_graph_replay_reindex(engine_factory):
    """svt_reindex + svt_refine_device captured into a HIP graph (torch.cuda.graph) replay with
    the oracle's results every time: the capture takes the two-pass index build (a replayed
    single-pass build would carry its capture's epoch) and the refine resets its own counters."""
    r = _workload(n_loci=3000, seed=71)
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    want = O.refine_batch(r.pileup, r.loci, threads=8)
    n = len(r.loci)
    d_loci = torch.from_numpy(r.loci.view(np.uint8).copy()).cuda()
    d_out = torch.zeros(n * RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):   # warm-up: a single-pass rebuild outside the capture
        eng.reindex(s.cuda_stream)
        eng.refine_device(d_loci.data_ptr(), n, d_out.data_ptr(), s.cuda_stream)
    s.synchronize()
    _same(d_out.cpu().numpy().view(RESULT_DTYPE), want)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        eng.reindex(s.cuda_stream)
        eng.refine_device(d_loci.data_ptr(), n, d_out.data_ptr(), s.cuda_stream)
    for _ in range(3):
        d_out.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        _same(d_out.cpu().numpy().view(RESULT_DTYPE), want)
    eng.reindex()   # and single-pass rebuilds after the replays
    _same(eng.refine(r.loci), want)


def test_locus_dtype_layout():
    assert LOCUS_DTYPE.itemsize == 16 and RECORD_DTYPE.itemsize == 16


def test_graph_replays_between_direct_lane_launches(engine_factory):
    """a captured lane launch replays with its capture's redo-counter parity
    while direct launches in between flip it; the replay must leave both left-over counters zero,
    or the next direct launch of the same parity appends after a stale count and re-runs windows
    of the graph's batch.  Lane kernel forced, min_count 1 (left-overs in every launch); direct and
    replayed launches alternate as direct, replay, direct, direct, replay, replay, direct."""
    r = _workload(n_loci=4000, seed=72)
    prm = Params(consensus_min_count=1)
    eng = engine_factory(prm, gather="span")
    eng.load_pileup(r.pileup)
    want = O.refine_batch(r.pileup, r.loci, prm, threads=8)
    n = len(r.loci)
    small = r.loci[: n // 3]
    want_small = want[: n // 3]
    d_loci = torch.from_numpy(r.loci.view(np.uint8).copy()).cuda()
    d_out = torch.zeros(n * RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        eng.refine_device(d_loci.data_ptr(), n, d_out.data_ptr(), s.cuda_stream)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        eng.refine_device(d_loci.data_ptr(), n, d_out.data_ptr(), s.cuda_stream)

    def replay():
        d_out.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        _same(d_out.cpu().numpy().view(RESULT_DTYPE), want)

    def direct():
        _same(eng.refine(small), want_small)

    for f in (direct, replay, direct, direct, replay, replay, direct):
        f()
