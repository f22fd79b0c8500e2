"""The seeded simvcf restatement reproduces the reference simvcf.py output byte for byte
(fixtures made by running the reference itself: tests/golden/make_simvcf_golden.py)."""
import os
import random

import pytest

from svtrek_amd.simvcf import simulate

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("seed", [1, 7, 2024])
def test_matches_reference_output(seed):
    with open(os.path.join(GOLD, "simvcf_input.vcf")) as f:
        lines = f.readlines()
    with open(os.path.join(GOLD, f"simvcf_seed{seed}.sim.vcf")) as f:
        want = f.read()
    got = "".join(simulate(lines, random.Random(seed)))
    assert got == want
