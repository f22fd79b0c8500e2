"""HIP engine vs CPU oracle: bit-exact refined breakpoints (integer path, no tolerance).

All calls go through the C ABI (libsvtrek_hip.so via svtrek_amd.Engine).
"""
import numpy as np
import oracle_ffi as O
import pytest

from svtrek_amd import SVT_NA, Engine, Params, make_loci, sim
from svtrek_amd._lib import LOCUS_DTYPE

from fuzz import cluster_pileup, random_loci, random_pileup

pytestmark = pytest.mark.gpu


def _assert_same(got, want, loci):
    bad = np.nonzero((got["start"] != want["start"]) | (got["end"] != want["end"]))[0]
    if len(bad):
        i = int(bad[0])
        raise AssertionError(f"{len(bad)} of {len(loci)} loci differ; first #{i} locus={loci[i]} "
                             f"gpu={got[i]} oracle={want[i]}")


def test_consensus_vectors_through_kernel(engine_factory):
    """SURVEY A10 vectors routed through a DEL-start window of a synthetic pileup."""
    from test_oracle_consensus import SURVEY_VECTORS
    eng = engine_factory()
    base = 100000
    for locs, pos, want in SURVEY_VECTORS:
        vals = [base + v for v in locs]
        pl = cluster_pileup(vals)
        eng.load_pileup(pl)
        loci = make_loci([(2, 1, base + pos, base + pos + 5000)])
        got = eng.refine(loci)
        exp = SVT_NA if want == -1 else base + want
        assert int(got["start"][0]) == exp, (locs, pos, want, int(got["start"][0]))
        assert int(O.refine_batch(pl, loci)["start"][0]) == exp


@pytest.mark.parametrize("gather", ["span", "span1"])
@pytest.mark.parametrize("seed", range(6))
def test_random_consensus_windows(engine_factory, seed, gather):
    rng = np.random.default_rng(seed)
    eng = engine_factory(Params(consensus_interval=int(rng.choice([0, 1, 5, 12])),
                                consensus_interval_range=int(rng.choice([50, 500, 900])),
                                consensus_min_count=int(rng.choice([1, 2, 3, 5]))), gather=gather)
    base = 200000
    rows, vals = [], []
    for k in range(40):
        c = base + k * 60000
        n = int(rng.integers(0, 40))
        centers = c + rng.integers(-400, 400, size=3)
        v = [int(rng.choice(centers)) + int(rng.integers(-8, 9)) for _ in range(n)]
        vals.extend(v)
        rows.append((2, 1, c + int(rng.integers(-30, 30)), c + 20000))
    pl = cluster_pileup(vals)
    eng.load_pileup(pl)
    loci = make_loci(rows)
    got = eng.refine(loci)
    want = O.refine_batch(pl, loci, eng.params)
    _assert_same(got, want, loci)


@pytest.mark.parametrize("gather", ["span", "span1"])
@pytest.mark.parametrize("seed", range(10))
def test_fuzz_pileups(engine_factory, seed, gather):
    rng = np.random.default_rng(1000 + seed)
    hot = [int(x) for x in rng.integers(5000, 55000, size=6)]
    pl = random_pileup(rng, n_targets=2, contig_len=60000, n_reads=int(rng.integers(50, 700)),
                       max_ops=int(rng.choice([3, 40, 150, 400])), hot=hot)
    prm = Params(wider_interval=int(rng.choice([20000, 3000])), median_interval=int(rng.choice([10000, 500])),
                 narrow_interval=int(rng.choice([2000, 100])), consensus_interval_range=int(rng.choice([500, 80])),
                 consensus_interval=int(rng.choice([5, 0, 30])), consensus_min_count=int(rng.choice([1, 2, 3])))
    eng = engine_factory(prm, gather=gather)
    eng.load_pileup(pl)
    loci = random_loci(rng, 300, 2, 60000, hot)
    got = eng.refine(loci)
    want = O.refine_batch(pl, loci, prm)
    _assert_same(got, want, loci)


def test_spill_path(engine_factory):
    """> SVT_LDS_CANDS candidates in one window: the device spill pool keeps it exact."""
    rng = np.random.default_rng(7)
    base = 300000
    vals = [base + int(x) for x in rng.integers(-300, 300, size=1500)] + [base + 3] * 40
    pl = cluster_pileup(vals)
    eng = engine_factory()
    eng.load_pileup(pl)
    loci = make_loci([(2, 1, base, base + 10000), (2, 1, base + 150, base + 9000), (1, 1, base, base)])
    w = eng.count_work(loci)
    assert w["spilled_windows"] >= 2
    got = eng.refine(loci)
    want = O.refine_batch(pl, loci)
    _assert_same(got, want, loci)


def test_spill_pool_grows_on_demand(engine_factory):
    """A 1 KiB pool cannot hold a 3000-candidate window: the synchronous call grows the pool
    to what the launch asked for and re-runs (the reference reallocs its candidate arrays,
    refinement.c:125-133), so the result is still exact; the asynchronous call reports
    EOVERFLOW once through svt_sync, after which the same launch fits."""
    import torch

    from svtrek_amd import SvtError
    from svtrek_amd._lib import RESULT_DTYPE
    vals = [400000 + i % 700 for i in range(3000)]
    pl = cluster_pileup(vals)
    eng = engine_factory(Params(spill_bytes=1024))
    eng.load_pileup(pl)
    loci = make_loci([(2, 1, 400100, 410000), (1, 1, 400300, 400300)])
    _assert_same(eng.refine(loci), O.refine_batch(pl, loci), loci)

    eng2 = engine_factory(Params(spill_bytes=1024))
    eng2.load_pileup(pl)
    d_loci = torch.from_numpy(loci.view(np.uint8).copy()).cuda()
    d_out = torch.empty(len(loci) * RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    eng2.refine_device(d_loci.data_ptr(), len(loci), d_out.data_ptr())
    with pytest.raises(SvtError) as ei:
        eng2.sync()
    assert ei.value.code == -5
    eng2.refine_device(d_loci.data_ptr(), len(loci), d_out.data_ptr())
    eng2.sync()
    got = d_out.cpu().numpy().view(RESULT_DTYPE)
    _assert_same(got, O.refine_batch(pl, loci), loci)


def test_long_cigars(engine_factory):
    """Reads with thousands of ops (multi-chunk scans, break deep inside a chunk)."""
    rng = np.random.default_rng(3)
    rows = []
    for k in range(120):
        pos = int(rng.integers(0, 20000))
        ops = []
        for j in range(int(rng.integers(500, 5000))):
            ops.append((int(rng.choice([0, 0, 1, 2, 8])), int(rng.integers(1, 9))))
        if rng.random() < 0.6:
            cut = int(rng.integers(0, len(ops)))
            ops.insert(cut, (2, int(rng.choice([51, 300]))))
        rows.append((0, pos, ops))
    from svtrek_amd.pileup import from_reads
    pl = from_reads(1, rows)
    eng = engine_factory()
    eng.load_pileup(pl)
    loci = make_loci([(2, 1, int(p), int(p) + int(e)) for p, e in
                      zip(rng.integers(0, 40000, 200), rng.integers(51, 20000, 200))] +
                     [(1, 1, int(p), int(p) + 1) for p in rng.integers(0, 40000, 100)])
    got = eng.refine(loci)
    want = O.refine_batch(pl, loci)
    _assert_same(got, want, loci)


def test_inv_and_unknown_types(engine_factory):
    pl = cluster_pileup([10000] * 10)
    eng = engine_factory()
    eng.load_pileup(pl)
    loci = make_loci([(3, 1, 10000, 20000), (4, 1, 10000, 20000), (0, 1, 10000, 10100)])
    got = eng.refine(loci)
    assert (got["start"] == SVT_NA).all() and (got["end"] == SVT_NA).all()
    want = O.refine_batch(pl, loci)
    _assert_same(got, want, loci)


def test_empty_inputs(engine_factory):
    from svtrek_amd.pileup import from_reads
    eng = engine_factory()
    eng.load_pileup(from_reads(3, []))
    assert len(eng.refine(np.zeros(0, dtype=LOCUS_DTYPE))) == 0
    loci = make_loci([(2, 1, 100000, 101000), (1, 3, 5, 6)])
    got = eng.refine(loci)
    assert (got["start"] == SVT_NA).all() and (got["end"] == SVT_NA).all()


def test_load_stats(engine_factory):
    """svt_last_load_stats: the split of svt_load_pileup's time (host pass, H2D, device index)."""
    from svtrek_amd.pileup import from_reads
    eng = engine_factory()
    eng.load_pileup(from_reads(3, []))
    st = eng.load_stats()
    assert st["index_ms"] == 0.0 and st["total_ms"] >= st["host_ms"] >= 0.0
    r = sim.generate(sim.SimConfig(seed=5, n_targets=2, n_loci=32, coverage=10.0))
    eng.load_pileup(r.pileup)
    st = eng.load_stats()
    assert st["index_ms"] > 0.0 and st["upload_ms"] > 0.0
    assert st["host_ms"] + st["upload_ms"] <= st["total_ms"] + 1e-3


@pytest.mark.parametrize("name", ["cfg1_100del_10x"])
def test_workload_cfg1_full(engine_factory, name):
    r = sim.generate(sim.WORKLOADS[name])
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    got = eng.refine(r.loci)
    want = O.refine_batch(r.pileup, r.loci)
    _assert_same(got, want, r.loci)
    assert (got["start"] != SVT_NA).mean() > 0.5


def test_workload_exotic_ops(engine_factory):
    cfg = sim.SimConfig(seed=9, n_targets=2, n_loci=400, del_frac=0.5, coverage=20, p_exotic=0.05,
                        p_clip_ends=0.3, p_noise_sv=0.3)
    r = sim.generate(cfg)
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    got = eng.refine(r.loci)
    want = O.refine_batch(r.pileup, r.loci, threads=4)
    _assert_same(got, want, r.loci)


def test_workload_cfg2_full_parity(engine_factory):
    """BASELINE config 2 at full size (10k DEL, 30x ONT-like): every locus bit-exact."""
    r = sim.generate(sim.WORKLOADS["cfg2_10kdel_30x_ont"])
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    got = eng.refine(r.loci)
    want, ow = O.refine_batch(r.pileup, r.loci, threads=8, with_work=True)
    _assert_same(got, want, r.loci)
    w = eng.count_work(r.loci)
    assert (w["windows"], w["reads"], w["ops_walked"], w["candidates"]) == \
        (ow["windows"], ow["reads"], ow["ops_walked"], ow["candidates"])


def test_repeatability_and_batch_split(engine_factory):
    """Order/batching independence (loci are independent, audit.c:50-248)."""
    r = sim.generate(sim.SimConfig(seed=77, n_loci=500, n_targets=2, del_frac=0.6))
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    a = eng.refine(r.loci)
    perm = np.random.default_rng(0).permutation(len(r.loci))
    b = eng.refine(r.loci[perm])
    assert (b == a[perm]).all()
    c = np.concatenate([eng.refine(r.loci[:123]), eng.refine(r.loci[123:])])
    assert (c == a).all()


@pytest.mark.parametrize("gather", ["span", "span1"])
def test_hifi_short_cigars(engine_factory, gather):
    """HiFi-like: ~30 ops per read, many reads per 256-op index slot (read starts mid-lane)."""
    cfg = sim.SimConfig(seed=12, n_targets=2, n_loci=600, del_frac=0.5, coverage=30, read_len_mean=15000,
                        read_len_sd=3000, read_len_min=500, rho=1 / 500, spacing=6000, sv_max_len=1500,
                        p_clip_ends=0.3, p_noise_sv=0.2)
    r = sim.generate(cfg)
    eng = engine_factory(gather=gather)
    eng.load_pileup(r.pileup)
    got = eng.refine(r.loci)
    want, ow = O.refine_batch(r.pileup, r.loci, threads=8, with_work=True)
    _assert_same(got, want, r.loci)
    w = eng.count_work(r.loci)
    assert (w["reads"], w["ops_walked"], w["candidates"]) == (ow["reads"], ow["ops_walked"], ow["candidates"])


def test_tiny_reads_and_empty_cigars(engine_factory):
    """1-op and 0-op reads (n_cigar == 0 keeps only the soft-clip tests, with the clip
    bits ingest recorded from the bytes the reference reads)."""
    from svtrek_amd.pileup import from_reads
    rng = np.random.default_rng(5)
    rows, clip = [], {}
    for i in range(3000):
        pos = int(rng.integers(0, 30000))
        kind = rng.random()
        if kind < 0.25:
            ops = []
            clip[i] = int(rng.integers(0, 4))
        elif kind < 0.6:
            ops = [(int(rng.choice([0, 2, 4, 1, 5])), int(rng.choice([1, 3, 51, 60, 120])))]
        else:
            ops = [(int(rng.choice([0, 2, 4, 1, 8, 3])), int(rng.choice([1, 2, 51, 300]))) for _ in range(int(rng.integers(2, 9)))]
        rows.append((0, pos, ops))
    pl = from_reads(1, rows, clip=clip)
    for gather in ("span", "span1"):
        eng = engine_factory(Params(consensus_min_count=1), gather=gather)
        eng.load_pileup(pl)
        loci = make_loci([(int(rng.choice([1, 2])), 1, int(p), int(p) + int(d)) for p, d in
                          zip(rng.integers(0, 32000, 400), rng.integers(51, 3000, 400))])
        got = eng.refine(loci)
        want = O.refine_batch(pl, loci, Params(consensus_min_count=1))
        _assert_same(got, want, loci)


def test_wrapping_walks_take_exact_path(engine_factory):
    """Reads whose walk position passes 2^31 (huge H/P/N ops advance rp, refinement.c:141)
    and windows ending past 2^31: exact uint32 replay, same as the oracle."""
    from svtrek_amd.pileup import from_reads
    big = (1 << 28) - 1
    rows = []
    for i in range(200):
        pos = 10000 + 37 * i
        ops = [(0, 500), (2, 80), (0, 300)]
        if i % 3 == 0:
            ops += [(5, big)] * 9 + [(2, 70), (0, 10)]
        if i % 5 == 0:
            ops = [(4, 20)] + ops + [(4, 30)]
        rows.append((0, pos, ops))
    pl = from_reads(1, rows)
    loci = make_loci([(2, 1, 10000 + 500 + 37 * k, 10000 + 580 + 37 * k) for k in range(0, 200, 7)] +
                     [(2, 1, (1 << 31) - 1000, (1 << 31) + 5000), (1, 1, 10600, 10601)])
    for gather in ("span", "span1"):
        eng = engine_factory(gather=gather)
        eng.load_pileup(pl)
        got = eng.refine(loci)
        want = O.refine_batch(pl, loci)
        _assert_same(got, want, loci)


@pytest.mark.parametrize("ncand", [63, 64, 65, 100, 128, 129, 200, 256])
def test_register_sort_sizes(engine_factory, ncand):
    """Candidate counts around the register-sort tiers (64 / 128 / 256 per window) and the
    LDS capacity: same votes as the oracle."""
    rng = np.random.default_rng(ncand)
    base = 500000
    rows, vals = [], []
    for k in range(30):
        c = base + k * 80000
        centers = c + rng.integers(-300, 300, size=4)
        vals.extend(int(rng.choice(centers)) + int(rng.integers(-6, 7)) for _ in range(ncand))
        rows.append((2, 1, c + int(rng.integers(-20, 20)), c + 30000))
    pl = cluster_pileup(vals)
    eng = engine_factory(Params(consensus_min_count=2))
    eng.load_pileup(pl)
    loci = make_loci(rows)
    w = eng.count_work(loci)
    assert w["spilled_windows"] == 0
    got = eng.refine(loci)
    want = O.refine_batch(pl, loci, eng.params)
    _assert_same(got, want, loci)


@pytest.mark.parametrize("seed", range(8))
def test_vote_band_edges(engine_factory, seed):
    """The vote's band filter (svt_engine.hip band_filter) against the full-multiset oracle:
    candidates exactly at / next to pos +- (range + ci), at pos+25 +- 1, far-left and far-right
    noise (the upper_bound A[0] and the max), clusters straddling the band edge, and parameter
    sets where the band is off (range <= 25, negative ci)."""
    rng = np.random.default_rng(7000 + seed)
    rows, vals = [], []
    ci = int(rng.choice([-3, 0, 1, 5, 12]))
    rng_ = int(rng.choice([10, 25, 26, 60, 500]))
    mc = int(rng.choice([1, 2, 3, 4]))
    eng = engine_factory(Params(consensus_interval=ci, consensus_interval_range=rng_, consensus_min_count=mc))
    base = 300000
    w = rng_ + max(ci, 0)
    for k in range(60):
        c = base + k * 60000
        pos = c + int(rng.integers(-30, 30))
        edge = [pos - w - 1, pos - w, pos - w + 1, pos + w - 1, pos + w, pos + w + 1,
                pos + 24, pos + 25, pos + 26, pos - 24, pos - 25, pos - 26,
                pos - rng_, pos - rng_ + 1, pos + rng_ - 1, pos + rng_]
        v = []
        for _ in range(int(rng.integers(0, 30))):
            r = rng.random()
            if r < 0.4:
                v.append(int(rng.choice(edge)) + int(rng.integers(-1, 2)))
            elif r < 0.6:
                v.append(pos + int(rng.integers(-15000, -w)))     # far left noise (A[0])
            elif r < 0.7:
                v.append(pos + int(rng.integers(w, 1900)))        # far right noise (the max)
            else:
                v.append(pos + int(rng.integers(-w - 10, w + 10)))
        if rng.random() < 0.3:   # a tight cluster straddling an edge
            e0 = int(rng.choice(edge))
            v.extend([e0 + int(d) for d in rng.integers(-abs(ci) - 2, abs(ci) + 3, size=int(rng.integers(2, 8)))])
        vals.extend(v)
        rows.append((2, 1, pos, c + 20000))
    pl = cluster_pileup(vals)
    eng.load_pileup(pl)
    loci = make_loci(rows)
    got = eng.refine(loci)
    want = O.refine_batch(pl, loci, eng.params)
    _assert_same(got, want, loci)


@pytest.mark.parametrize("seed", range(3))
def test_hip_and_cpu_backends_through_one_abi(engine_factory, seed):
    """The same svt_open / svt_load_pileup / svt_refine_batch / svt_count_work calls on the
    HIP engine and on oracle/libsvtrek_cpu.so (the CPU restatement behind include/svtrek_gpu.h)."""
    import ctypes as C
    import os

    from svtrek_amd._lib import bind_abi
    cpu_lib = bind_abi(C.CDLL(os.path.join(os.path.dirname(O.__file__), "libsvtrek_cpu.so")))
    rng = np.random.default_rng(900 + seed)
    hot = [int(x) for x in rng.integers(5000, 55000, size=6)]
    pl = random_pileup(rng, n_targets=2, contig_len=60000, n_reads=int(rng.integers(100, 600)), max_ops=120, hot=hot)
    loci = random_loci(rng, 400, 2, 60000, hot)
    gpu = engine_factory()
    gpu.load_pileup(pl)
    with Engine(Params(), device=0, lib=cpu_lib) as cpu:
        cpu.load_pileup(pl)
        _assert_same(gpu.refine(loci), cpu.refine(loci), loci)
        nv = loci[loci["type"] != 3]   # the engine issues no INV queries (refine_point never collects)
        wc, wg = cpu.count_work(nv), gpu.count_work(nv)
        assert (wc["windows"], wc["reads"], wc["ops_walked"], wc["candidates"]) == \
            (wg["windows"], wg["reads"], wg["ops_walked"], wg["candidates"])


@pytest.mark.parametrize("gather", ["span", "span1"])
@pytest.mark.parametrize("nsplit", [20, 90, 300])
def test_lane_kernel_split_reads_bands_and_left_overs(engine_factory, nsplit, gather):
    """refine_end over many split reads (leading S, walk past the window end: the LEAD/TRAIL
    sentinel events) at DEL ends, next to windows whose bands exceed 32 members (left over to
    refine_redo_kernel) and a window with > 256 candidates (spill slab), all against the oracle."""
    from svtrek_amd.pileup import from_reads
    rng = np.random.default_rng(nsplit)
    rows, loci = [], []
    for k in range(40):
        c = 50000 + k * 30000
        end = c + 3000
        loci.append((2, 1, c, end))
        for _ in range(int(rng.integers(0, 12))):   # DEL-start support
            p0 = c - int(rng.integers(500, 4000))
            rows.append((0, p0, [(0, c - p0 + int(rng.integers(-6, 7))), (2, 3000), (0, 2000)]))
        for _ in range(nsplit // 10 if k % 3 else nsplit):   # split reads at the DEL end: S, then a long M
            p0 = end + int(rng.integers(-1900, 1900))
            rows.append((0, p0, [(4, 500), (0, int(rng.integers(1, 40))), (1, 60), (0, 6000)]))
        if k == 7:   # a dense band: 60 candidates within a few bp of pos
            for _ in range(60):
                p0 = c - 1000
                rows.append((0, p0, [(0, 1000 + int(rng.integers(-3, 4))), (2, 3000), (0, 500)]))
        if k == 11:  # > 256 candidates in one window
            for _ in range(300):
                p0 = c - int(rng.integers(2000, 15000))
                rows.append((0, p0, [(0, c - p0 + int(rng.integers(-400, 400))), (2, 80), (0, 300)]))
    pl = from_reads(1, rows, clip=None)
    eng = engine_factory(gather=gather)
    eng.load_pileup(pl)
    lc = make_loci(loci)
    _assert_same(eng.refine(lc), O.refine_batch(pl, lc), lc)


def test_size_based_kernel_pick_alternating(engine_factory):
    """The product's own pick: batches below 64K windows run refine_span_kernel, larger ones
    refine_lane_kernel<32> + refine_redo_kernel, whose left-over counters alternate by launch;
    interleaving small and large batches on one context (and a device-side stream of launches
    without host syncs between them) must keep every result equal to the oracle's."""
    import torch
    rng = np.random.default_rng(77)
    hot = [int(x) for x in rng.integers(5000, 55000, size=8)]
    pl = random_pileup(rng, n_targets=2, contig_len=60000, n_reads=600, max_ops=150, hot=hot)
    eng = engine_factory(gather="auto")
    eng.load_pileup(pl)
    big = random_loci(rng, 40000, 2, 60000, hot)     # 80K windows: lane kernel
    small = random_loci(rng, 3000, 2, 60000, hot)    # 6K windows: span kernel
    want_b, want_s = O.refine_batch(pl, big), O.refine_batch(pl, small)
    for batch, want in ((big, want_b), (small, want_s), (big, want_b), (big, want_b), (small, want_s),
                        (small, want_s), (big, want_b)):
        _assert_same(eng.refine(batch), want, batch)
    # the same sequence queued on one stream, checked after a single sync
    from svtrek_amd._lib import LOCUS_DTYPE, RESULT_DTYPE
    seq = [big, small, small, big, small, big, big]
    dev = [torch.from_numpy(np.ascontiguousarray(b, dtype=LOCUS_DTYPE).view(np.uint8)).cuda() for b in seq]
    outs = [torch.empty(len(b) * RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda") for b in seq]
    s = torch.cuda.current_stream().cuda_stream
    for b, d, o in zip(seq, dev, outs):
        eng.refine_device(d.data_ptr(), len(b), o.data_ptr(), s)
    eng.sync(s)
    torch.cuda.synchronize()
    for b, o in zip(seq, outs):
        got = o.cpu().numpy().view(RESULT_DTYPE)
        _assert_same(got, want_b if b is big else want_s, b)


@pytest.mark.parametrize("seed", range(4))
def test_index_kinds_agree_with_saturating_walks(engine_factory, seed):
    """The two index builds agree: lane per read (the product's pick for short reads; also
    forced, SVTREK_IX=lane) and the stream walk (SVTREK_IX=stream), with and without the stream
    walk's quiet slots (long reads, SVTREK_IX_RANGES=1: a few huge ranges).  The pileup has reads
    whose walks pass 2^28 and 2^30 (huge H ops, refinement.c:141 advances on H): the index
    saturates their walk positions at 2^30, windows ending below 2^30 stay exact on them, and
    windows ending past 2^30 take the per-read replay.  Same index sizes, same results as the
    oracle, also after a rebuild from the resident pileup."""
    from svtrek_amd.pileup import from_reads
    rng = np.random.default_rng(50 + seed)
    rows = []
    big = (1 << 28) - 1
    pos = 5000
    far = []   # (walk position, endpos) regions reached through huge N ops
    for i in range(4000):
        pos += int(rng.integers(0, 40))
        if i % 50:
            ops = [(int(rng.choice([0, 1, 2, 4, 5, 0, 0, 8])), int(rng.integers(1, 120)))
                   for _ in range(int(rng.integers(1, 30)))]
        else:   # a long read with few candidates: quiet slots of the stream walk
            ops = [(int(rng.choice([0, 0, 0, 8, 1, 2, 7])), int(rng.integers(1, 20)))
                   for _ in range(int(rng.integers(300, 3000)))]
            for _ in range(int(rng.integers(0, 3))):
                ops.insert(int(rng.integers(0, len(ops))), (int(rng.choice([1, 2])), int(rng.integers(50, 400))))
        if i % 997 == 3:     # a walk past 2^28 / 2^30 on huge H ops (the walk runs ahead of endpos)
            ops += [(5, big)] * (1 if i % 2 else 5) + [(2, 60), (0, 5)]
        if i % 991 == 5:     # ... and on huge N ops (endpos follows: windows out there see the read)
            k = 3 if i % 2 else 4
            ops = [(0, 100)] + [(3, big)] * k + [(2, 60), (0, 50), (4, 30)]
            far.append(pos + 100 + k * big)
        if rng.random() < 0.3:
            ops = [(4, int(rng.integers(1, 40)))] + ops
        if rng.random() < 0.3:
            ops = ops + [(4, int(rng.integers(1, 40)))]
        rows.append((0, pos, ops))
    pl = from_reads(1, rows)
    hot = [int(x) for x in rng.integers(6000, pos, size=8)]
    loci = random_loci(rng, 400, 1, pos + 2000, hot)
    extra = [(2, 1, (1 << 30) - 3000, (1 << 30) + 100), (1, 1, (1 << 30) - 50, 0)]
    for f in far:   # DEL / INS calls at the far D ops: below and past 2^30
        extra += [(2, 1, f + int(d), f + 60 + int(d)) for d in rng.integers(-5, 5, 3)] + [(1, 1, f, 0)]
    loci = np.concatenate([loci, make_loci(extra)])
    want = O.refine_batch(pl, loci)
    stats = []
    for env in (None, {"SVTREK_IX": "lane"}, {"SVTREK_IX": "stream"},
                {"SVTREK_IX": "stream", "SVTREK_IX_RANGES": "1"}):
        eng = engine_factory(env=env)
        eng.load_pileup(pl)
        st = eng.load_stats()
        stats.append(st["span_events"])
        _assert_same(eng.refine(loci), want, loci)
        for _ in range(2):   # rebuilds from the resident pileup
            eng.reindex()
            _assert_same(eng.refine(loci), want, loci)
    assert all(x == stats[0] for x in stats)


@pytest.mark.parametrize("seed", range(2))
def test_lane_filing_stage_overflow(engine_factory, seed):
    """The short-read filing pass stages a group's events in LDS (256 of them, svt_bucket_build.inc
    IXB_EVCAP); a group with more -- here reads with ~8 D > 50 / I >= 50 ops each, ~500 events a
    group -- files the rest through a second walk of the group, and a group whose reads lie in two
    contigs files all of its events that way.  Lane index forced (SVTREK_IX=lane); same results as
    the oracle, also after rebuilds (the cursors' epochs)."""
    from svtrek_amd.pileup import from_reads
    rng = np.random.default_rng(90 + seed)
    rows = []
    for t in range(2):
        pos = 3000
        for i in range(1500):
            pos += int(rng.integers(0, 12))
            ops = []
            for _ in range(int(rng.integers(4, 12))):
                ops.append((0, int(rng.integers(20, 300))))
                ops.append((int(rng.choice([1, 2])), int(rng.integers(45, 200))))
            ops.append((0, int(rng.integers(10, 200))))
            if rng.random() < 0.4:
                ops = [(4, int(rng.integers(1, 40)))] + ops
            if rng.random() < 0.4:
                ops = ops + [(4, int(rng.integers(1, 40)))]
            rows.append((t, pos, ops))
    pl = from_reads(2, rows)
    hot = [int(x) for x in rng.integers(4000, 12000, size=8)]
    loci = random_loci(rng, 600, 2, 15000, hot)
    want = O.refine_batch(pl, loci)
    eng = engine_factory(env={"SVTREK_IX": "lane"})
    eng.load_pileup(pl)
    assert eng.load_stats()["index_kind"] == 1
    _assert_same(eng.refine(loci), want, loci)
    for _ in range(2):
        eng.reindex()
        _assert_same(eng.refine(loci), want, loci)
