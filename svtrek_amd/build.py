"""In-tree build of every native artefact (gfx950 HIP engine, host tools, CLI).

Outputs land next to their sources inside the repo so they travel to the GPU box
with the gpurun snapshot (they are git-ignored, not gpurun-ignored):

    svtrek_amd/libsvtrek_hip.so   HIP kernels + C ABI (include/svtrek_gpu.h)   [product]
    svtrek_amd/libsvtrek_host.so  BAM ingest + VCF parse/format (C++)          [product]
    svtrek_amd/svtrek             `svtrek audt` drop-in CLI                     [product]
    svtrek_amd/libsvtrek_sim.so   seeded synthetic pileups + BAM writer         [test/bench data]
    oracle/liboracle.so           CPU parity oracle                             [test infra]
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "svtrek_amd")
CSRC = os.path.join(PKG, "csrc")
INC = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SVT_OFFLOAD_ARCH", "gfx950")


def _run(cmd: list[str], cwd: str | None = None) -> None:
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")


def _stale(out: str, deps: list[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build_engine(force: bool = False) -> str:
    out = os.path.join(PKG, "libsvtrek_hip.so")
    deps = [os.path.join(CSRC, "svt_engine.hip"), os.path.join(INC, "svtrek_gpu.h"), os.path.join(CSRC, "svt_poa.inc"),
            os.path.join(CSRC, "svt_index.inc"), os.path.join(CSRC, "svt_index2.inc"),
            os.path.join(CSRC, "svt_inflate.inc"), os.path.join(CSRC, "svt_bamrec.h"), os.path.join(CSRC, "svt_bam.inc"),
            os.path.join(CSRC, "svt_bucket.inc"), os.path.join(CSRC, "svt_bucket_build.inc")]
    if force or _stale(out, deps):
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
              "-Wall", "-I", INC, "-o", out, deps[0]])
    return out


def build_test_engine(force: bool = False) -> str:
    """Test artefact: the engine with a 2-row POA ring (svt_poa.inc SVT_POA_RING), so nearly
    every predecessor is read from a spill row -- tests/test_gpu_poa.py runs parity on it."""
    out = os.path.join(PKG, "variants", "libsvtrek_hip_ring2.so")
    deps = [os.path.join(CSRC, "svt_engine.hip"), os.path.join(INC, "svtrek_gpu.h"), os.path.join(CSRC, "svt_poa.inc"),
            os.path.join(CSRC, "svt_index.inc"), os.path.join(CSRC, "svt_index2.inc"),
            os.path.join(CSRC, "svt_inflate.inc"), os.path.join(CSRC, "svt_bamrec.h"), os.path.join(CSRC, "svt_bam.inc"),
            os.path.join(CSRC, "svt_bucket.inc"), os.path.join(CSRC, "svt_bucket_build.inc")]
    if force or _stale(out, deps):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-DSVT_POA_RING=2",
              "-I", INC, "-o", out, deps[0]])
    return out


def build_host(force: bool = False) -> str:
    out = os.path.join(PKG, "libsvtrek_host.so")
    srcs = [os.path.join(CSRC, f) for f in ("bam_ingest.cpp", "vcf_audit.cpp")]
    hdrs = [os.path.join(CSRC, "svtrek_host.h"), os.path.join(INC, "svtrek_gpu.h"), os.path.join(CSRC, "svt_bamrec.h")]
    if all(os.path.exists(s) for s in srcs) and (force or _stale(out, srcs + hdrs)):
        _run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra", "-pthread",
              "-I", INC, "-o", out] + srcs + ["-lz", "-ldl"])
    return out


def build_cli(force: bool = False) -> str:
    out = os.path.join(PKG, "svtrek")
    main = os.path.join(CSRC, "svtrek_main.cpp")
    srcs = [main] + [os.path.join(CSRC, f) for f in ("bam_ingest.cpp", "vcf_audit.cpp")]
    hdrs = [os.path.join(CSRC, "svtrek_host.h"), os.path.join(INC, "svtrek_gpu.h"), os.path.join(CSRC, "svt_bamrec.h")]
    eng = os.path.join(PKG, "libsvtrek_hip.so")
    if all(os.path.exists(s) for s in srcs) and (force or _stale(out, srcs + hdrs + [eng])):
        _run(["g++", "-O3", "-std=c++17", "-Wall", "-Wextra", "-pthread", "-I", INC, "-o", out] + srcs +
             ["-L", PKG, "-lsvtrek_hip", "-Wl,-rpath,$ORIGIN", "-lz", "-ldl"])
    return out


def build_sim(force: bool = False) -> str:
    out = os.path.join(PKG, "libsvtrek_sim.so")
    deps = [os.path.join(CSRC, "simpileup.c"), os.path.join(CSRC, "simpileup.h")]
    if force or _stale(out, deps):
        _run(["gcc", "-O3", "-std=gnu11", "-fPIC", "-shared", "-Wall", "-Wextra", "-o", out, deps[0],
              "-lz", "-lm"])
    return out


def build_oracle(force: bool = False) -> str:
    """Test infrastructure: the CPU parity oracle (oracle/Makefile)."""
    out = os.path.join(ROOT, "oracle", "liboracle.so")
    src = [os.path.join(ROOT, "oracle", f) for f in ("svtrek_oracle.c", "poa_oracle.c", "bgzf_ref.c", "svtrek_oracle.h",
                                                      "svtrek_cpu.c", "Makefile")] + [os.path.join(INC, "svtrek_gpu.h")]
    cpu = os.path.join(ROOT, "oracle", "libsvtrek_cpu.so")
    if force or _stale(out, src) or _stale(cpu, src):
        _run(["make", "-s", "-C", os.path.join(ROOT, "oracle")] + (["-B"] if force else []))
    # the product's CLI (svtrek_main.cpp) linked against the CPU backend: CPU-side CLI tests
    cli = os.path.join(ROOT, "oracle", "_cpu", "svtrek_cpu")
    csrc = [os.path.join(CSRC, f) for f in ("svtrek_main.cpp", "bam_ingest.cpp", "vcf_audit.cpp")]
    if os.path.exists(csrc[0]) and (force or _stale(cli, csrc + [cpu, os.path.join(CSRC, "svtrek_host.h")])):
        os.makedirs(os.path.dirname(cli), exist_ok=True)
        _run(["g++", "-O2", "-std=c++17", "-pthread", "-I", INC, "-o", cli] + csrc +
             ["-L", os.path.join(ROOT, "oracle"), "-lsvtrek_cpu", "-Wl,-rpath,$ORIGIN/..", "-lz", "-ldl"])
    return out


SAN_FLAGS = {"asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"],
             "tsan": ["-fsanitize=thread"]}


def build_sanitizers(force: bool = False) -> dict[str, str]:
    """Test artefacts (host code only, tests/test_sanitizers.py): the product's host C++
    (bam_ingest.cpp, vcf_audit.cpp) and the oracle's threaded paths, each under ASan+UBSan
    and under TSan, as standalone drivers (tests/san/) in build/san/."""
    out_dir = os.path.join(ROOT, "build", "san")
    os.makedirs(out_dir, exist_ok=True)
    host_src = [os.path.join(ROOT, "tests", "san", "host_san.cpp")] + \
        [os.path.join(CSRC, f) for f in ("bam_ingest.cpp", "vcf_audit.cpp")]
    orc_src = [os.path.join(ROOT, "tests", "san", "oracle_san.c"), os.path.join(CSRC, "simpileup.c")] + \
        [os.path.join(ROOT, "oracle", f) for f in ("svtrek_oracle.c", "poa_oracle.c", "bgzf_ref.c")]
    hdrs = [os.path.join(CSRC, "svtrek_host.h"), os.path.join(INC, "svtrek_gpu.h"), os.path.join(CSRC, "simpileup.h"),
            os.path.join(ROOT, "oracle", "svtrek_oracle.h")]
    arts = {}
    for kind, fl in SAN_FLAGS.items():
        out = os.path.join(out_dir, f"host_{kind}")
        if force or _stale(out, host_src + hdrs):
            _run(["g++", "-O1", "-g", "-std=c++17", "-pthread", *fl, "-I", INC, "-I", CSRC, "-o", out] + host_src +
                 ["-lz", "-ldl"])
        arts[f"host_{kind}"] = out
        out = os.path.join(out_dir, f"oracle_{kind}")
        if force or _stale(out, orc_src + hdrs):
            _run(["gcc", "-O1", "-g", "-std=gnu11", "-pthread", *fl, "-I", CSRC, "-I", os.path.join(ROOT, "oracle"),
                  "-o", out] + orc_src + ["-lz", "-lm"])
        arts[f"oracle_{kind}"] = out
    return arts


def build_all(force: bool = False) -> dict[str, str]:
    arts = {
        "engine": build_engine(force),
        "engine_ring2": build_test_engine(force),
        "sim": build_sim(force),
        "oracle": build_oracle(force),
    }
    if os.path.exists(os.path.join(CSRC, "svtrek_main.cpp")):
        arts["host"] = build_host(force)
        arts["cli"] = build_cli(force)
    return arts


if __name__ == "__main__":
    force = "--force" in sys.argv
    for k, v in build_all(force).items():
        print(f"{k:7s} {v} {'ok' if os.path.exists(v) else 'MISSING'}")
    if shutil.which(HIPCC) is None and not os.path.exists(HIPCC):
        print("warning: hipcc not found", file=sys.stderr)
