"""Seeded synthetic pileups (libsvtrek_sim.so) and the BASELINE.json workload presets.

Workloads follow SURVEY.md §8(d).  Each preset is deterministic (one seed per
config) so the GPU box and this container generate identical inputs.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, fields

import numpy as np

from ._lib import LOCUS_DTYPE, load_sim
from .pileup import Pileup


class _SimConfig(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("n_targets", C.c_int32),
        ("n_loci", C.c_int32),
        ("del_frac", C.c_double),
        ("sv_min_len", C.c_int32),
        ("sv_max_len", C.c_int32),
        ("spacing", C.c_int32),
        ("first_offset", C.c_int32),
        ("coverage", C.c_double),
        ("read_len_mean", C.c_int32),
        ("read_len_sd", C.c_int32),
        ("read_len_min", C.c_int32),
        ("rho", C.c_double),
        ("p_carry", C.c_double),
        ("p_split", C.c_double),
        ("bp_jitter", C.c_int32),
        ("report_jitter", C.c_int32),
        ("p_noise_sv", C.c_double),
        ("p_clip_ends", C.c_double),
        ("p_exotic", C.c_double),
        ("par_contigs", C.c_int32),
    ]


@dataclass
class SimConfig:
    seed: int = 1
    n_targets: int = 1
    n_loci: int = 100
    del_frac: float = 1.0
    sv_min_len: int = 50
    sv_max_len: int = 10000
    spacing: int = 40000
    first_offset: int = 25000
    coverage: float = 30.0
    read_len_mean: int = 10000
    read_len_sd: int = 2000
    read_len_min: int = 1000
    rho: float = 1.0 / 25.0
    p_carry: float = 0.70
    p_split: float = 0.15
    bp_jitter: int = 10
    report_jitter: int = 40
    p_noise_sv: float = 0.05
    p_clip_ends: float = 0.10
    p_exotic: float = 0.0
    par_contigs: int = 0

    def to_c(self) -> _SimConfig:
        return _SimConfig(**{f.name: getattr(self, f.name) for f in fields(self)})


# BASELINE.json configs.  Contig count keeps every contig < 2^29 bp
# (the BAI limit the reference's region queries live under).
WORKLOADS = {
    "cfg1_100del_10x": SimConfig(seed=101, n_targets=1, n_loci=100, del_frac=1.0, coverage=10.0,
                                 read_len_mean=10000, read_len_sd=2000, rho=1 / 25, spacing=40000),
    "cfg2_10kdel_30x_ont": SimConfig(seed=202, n_targets=4, n_loci=10000, del_frac=1.0, coverage=30.0,
                                     read_len_mean=10000, read_len_sd=2000, rho=1 / 25, spacing=40000),
    "cfg3_50k_delins_30x_ont": SimConfig(seed=303, n_targets=16, n_loci=50000, del_frac=0.5, coverage=30.0,
                                         read_len_mean=10000, read_len_sd=2000, rho=1 / 25, spacing=40000),
    "cfg4_1m_delins_30x_hifi": SimConfig(seed=404, n_targets=22, n_loci=1000000, del_frac=0.5, coverage=30.0,
                                         read_len_mean=15000, read_len_sd=2000, read_len_min=2000,
                                         rho=1 / 500, spacing=3100, sv_max_len=1000, first_offset=25000),
    "cfg5_100k_60x_ul_ont": SimConfig(seed=505, n_targets=8, n_loci=100000, del_frac=0.5, coverage=60.0,
                                      read_len_mean=50000, read_len_sd=10000, read_len_min=5000, rho=1 / 25,
                                      spacing=40000, par_contigs=2),
}


@dataclass
class SimResult:
    pileup: Pileup
    loci: np.ndarray        # LOCUS_DTYPE (reported, jittered breakpoints)
    truth: np.ndarray       # int32 [n, 2] true bp1, bp2
    handle: object = None   # keeps the C allocation alive for write_bam


class _Handle:
    def __init__(self, lib, h):
        self.lib, self.h = lib, h

    def __del__(self):
        if self.h:
            self.lib.sim_free(self.h)
            self.h = None


def generate(cfg: SimConfig, keep_handle: bool = False) -> SimResult:
    lib = load_sim()
    c = cfg.to_c()
    h = lib.sim_generate(C.byref(c))
    if not h:
        raise MemoryError("sim_generate failed")
    hd = _Handle(lib, h)
    nt = lib.sim_n_targets(h)
    nr = lib.sim_n_reads(h)
    nops = lib.sim_n_ops(h)
    nl = lib.sim_n_loci(h)

    def arr(fn, dtype, n):
        """The C array as numpy: a zero-copy view when the handle is kept (the Pileup keeps it
        alive; cfg5's 9.6 G CIGAR words are never copied), else a copy."""
        p = getattr(lib, fn)(h)
        if n == 0:
            return np.zeros(0, dtype=dtype)
        buf = (C.c_char * (n * np.dtype(dtype).itemsize)).from_address(p)
        a = np.frombuffer(buf, dtype=dtype, count=n)
        return a if keep_handle else a.copy()

    pile = Pileup(
        tid_off=arr("sim_tid_off", np.int64, nt + 1),
        pos=arr("sim_pos", np.int32, nr),
        endpos=arr("sim_endpos", np.int32, nr),
        cig_off=arr("sim_cig_off", np.uint64, nr + 1),
        cigar=arr("sim_cigar", np.uint32, nops),
        flag=arr("sim_flag", np.uint16, nr),
        contig_len=np.array([lib.sim_contig_len(h, t) for t in range(nt)], dtype=np.int32),
    )
    raw = arr("sim_loci", np.int32, nl * 4).reshape(-1, 4)
    loci = np.zeros(nl, dtype=LOCUS_DTYPE)
    loci["type"] = raw[:, 0]
    loci["chrom"] = raw[:, 1]
    loci["pos"] = raw[:, 2].astype(np.uint32)
    loci["end"] = raw[:, 3].astype(np.uint32)
    truth = arr("sim_truth", np.int32, nl * 2).reshape(-1, 2).copy()
    if keep_handle:
        pile._keepalive.append(hd)
    return SimResult(pile, loci, truth, hd if keep_handle else None)


def insertion_sequences(res: SimResult, cfg: SimConfig, err_permille: int = 50) -> tuple[np.ndarray, np.ndarray]:
    """(off uint64 [n+1], bases uint8 nt4) for every I >= 50 op of the pileup in (read, op)
    order -- svt_load_insseq's input.  Ops carrying an INS locus get that locus's allele with
    per-base substitutions (err_permille / 1000); others random bases.  Seeded by cfg.seed."""
    if res.handle is None:
        raise ValueError("generate(..., keep_handle=True) is required")
    lib = load_sim()
    n = C.c_uint64(0)
    po, pb = C.c_void_p(), C.c_void_p()
    if lib.sim_insseq(res.handle.h, cfg.seed, cfg.bp_jitter, err_permille, C.byref(n), C.byref(po), C.byref(pb)):
        raise MemoryError("sim_insseq")
    try:
        nn = int(n.value)
        off = np.frombuffer((C.c_char * (8 * (nn + 1))).from_address(po.value), dtype=np.uint64).copy()
        nb = int(off[-1])
        bases = (np.frombuffer((C.c_char * nb).from_address(pb.value), dtype=np.uint8).copy() if nb
                 else np.zeros(0, dtype=np.uint8))
    finally:
        lib.sim_free_buf(po)
        lib.sim_free_buf(pb)
    return off, bases


def write_bam(res: SimResult, path: str, with_seq: bool = False, level: int = 6, bai: bool = True,
              region: tuple[int, int, int] | None = None) -> None:
    """Coordinate-sorted BAM of the pileup (+ `path`.bai unless bai=False; the reference needs
    one, audit.c:271).  region = (tid, beg, end): only the records of that contig overlapping
    [beg, end) -- every query inside the region yields the same reads as on the full file."""
    if res.handle is None:
        raise ValueError("generate(..., keep_handle=True) is required to write a BAM")
    lib = load_sim()
    t, b, e = region if region is not None else (-1, 0, 0)
    if lib.sim_write_bam_region(res.handle.h, path.encode(), 1 if with_seq else 0, level, t, b, e,
                                1 if bai else 0) != 0:
        raise OSError(f"sim_write_bam failed: {path}")


def write_bam_regions(res: SimResult, path: str, regions: list[tuple[int, int, int]], with_seq: bool = False,
                      level: int = 6, bai: bool = True) -> None:
    """Like write_bam, with the records overlapping any of several (tid, beg, end) regions: one
    shard's halo over the contigs its loci span (every query of the shard yields the same reads
    as on the full file)."""
    if res.handle is None:
        raise ValueError("generate(..., keep_handle=True) is required to write a BAM")
    lib = load_sim()
    tid = np.ascontiguousarray([r[0] for r in regions], dtype=np.int32)
    beg = np.ascontiguousarray([r[1] for r in regions], dtype=np.int64)
    end = np.ascontiguousarray([r[2] for r in regions], dtype=np.int64)
    if lib.sim_write_bam_regions(res.handle.h, path.encode(), 1 if with_seq else 0, level, len(regions),
                                 tid.ctypes.data, beg.ctypes.data, end.ctypes.data, 1 if bai else 0) != 0:
        raise OSError(f"sim_write_bam_regions failed: {path}")


def write_vcf(loci: np.ndarray, path: str, chrom_prefix: str = "") -> None:
    """Plain `SVTYPE=..;END=..` VCF (the layout BASELINE configs 2-5 use)."""
    names = {1: "INS", 2: "DEL", 3: "INV"}
    with open(path, "w") as f:
        f.write("##fileformat=VCFv4.2\n")
        f.write('##INFO=<ID=SVTYPE,Number=1,Type=String,Description="Type of structural variant">\n')
        f.write('##INFO=<ID=END,Number=1,Type=Integer,Description="End position">\n')
        f.write("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n")
        for i, l in enumerate(loci):
            t = names.get(int(l["type"]), "DUP")
            f.write(f"{chrom_prefix}{int(l['chrom'])}\t{int(l['pos'])}\tsv{i}\tN\t<{t}>\t60\tPASS\t"
                    f"SVTYPE={t};END={int(l['end'])}\n")
