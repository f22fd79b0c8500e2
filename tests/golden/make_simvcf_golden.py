"""Generate the simvcf golden fixtures (run in the build container only).

Runs the reference's own test-data generator, /root/reference/utils/simvcf.py
(stdlib-only Python, reference utils/simvcf.py:24-196), under a fixed
`random.seed`, on a small sequence-resolved input VCF written here, and stores
input + output as data fixtures under tests/golden/.  The reference file itself
is executed from its read-only location; nothing of it is copied.

    python tests/golden/make_simvcf_golden.py

Fixtures written:
    simvcf_input.vcf            the sequence-resolved input (>= 9 columns, simvcf.py:112
                                appends INFO text after column 8, so 8-column input breaks)
    simvcf_seed<S>.sim.vcf      simvcf.py output with random.seed(S) before it runs
"""
import os
import random
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/utils/simvcf.py"
SEEDS = (1, 7, 2024)


def make_input(path: str) -> None:
    rng = random.Random(12345)
    bases = "ACGT"
    lines = [
        "##fileformat=VCFv4.2\n",
        "##source=svtrek_amd golden generator\n",
        '##INFO=<ID=AF,Number=A,Type=Float,Description="Allele Frequency">\n',
        "##contig=<ID=chr1,length=248956422>\n",
        "##contig=<ID=chr2,length=242193529>\n",
        "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tSAMPLE\n",
    ]
    pos = 30000
    for k in range(40):
        chrom = "chr1" if k < 25 else "chr2"
        kind = k % 5
        if kind in (0, 1):      # deletion, 50..3000 bp
            n = rng.choice([49, 50, 51, 60, 120, 800, 2999])
            ref = "".join(rng.choice(bases) for _ in range(n + 1))
            alt = ref[0]
        elif kind in (2, 3):    # insertion
            n = rng.choice([49, 50, 51, 75, 300, 1500])
            ref = rng.choice(bases)
            alt = ref + "".join(rng.choice(bases) for _ in range(n))
        else:                   # SNV / MNV left untouched by simvcf
            ref = rng.choice(bases)
            alt = rng.choice([b for b in bases if b != ref])
        vid = "." if k % 3 else f"var{k}"
        lines.append(f"{chrom}\t{pos}\t{vid}\t{ref}\t{alt}\t60\tPASS\tAF=0.5\tGT\t0/1\n")
        pos += rng.randint(31000, 60000)
    with open(path, "w") as f:
        f.writelines(lines)


def main() -> int:
    if not os.path.exists(REF):
        print("reference simvcf.py not present; fixtures are committed", file=sys.stderr)
        return 0
    inp = os.path.join(HERE, "simvcf_input.vcf")
    make_input(inp)
    for seed in SEEDS:
        out = os.path.join(HERE, f"simvcf_seed{seed}.sim.vcf")
        code = (
            "import random, runpy, sys\n"
            f"random.seed({seed})\n"
            f"sys.argv = ['simvcf.py', '-i', {inp!r}, '-o', {out!r}]\n"
            f"runpy.run_path({REF!r}, run_name='__main__')\n"
        )
        subprocess.run([sys.executable, "-c", code], check=True)
        print("wrote", out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
