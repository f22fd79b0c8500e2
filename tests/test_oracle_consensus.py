"""Oracle pinning: consensus_pos / lower_bound / upper_bound known-answer vectors.

Every vector below was produced by the reference's own object code
(refinement.c:3-101 compiled in the survey session) and is recorded in
SURVEY.md §8 A9/A10 -- these are reference outputs, not restatements.
"""
import oracle_ffi as O
import pytest

# (locations, pos, expected)  -- SURVEY.md §8 A10 step 6, min_count 3, ci 5, range 500
SURVEY_VECTORS = [
    ([1100, 1100, 1101, 1102, 1099], 1000, -1),
    ([1100, 1100, 1101, 1102, 1099, 800], 1000, 1100),
    ([900, 900, 901, 899, 902], 1000, 900),
    ([1003, 1003, 1004, 1100, 1100, 1100, 1100], 1000, 1003),
    ([940, 941, 942, 1080, 1081, 1082, 1083], 1000, 941),
    ([950, 950, 950, 1050, 1050, 1050], 1000, 950),
    ([1010, 1012, 1014, 1015], 1000, 1013),
    ([1000, 1000], 1000, -1),
]


@pytest.mark.parametrize("locs,pos,want", SURVEY_VECTORS)
def test_consensus_survey_vectors(locs, pos, want):
    assert O.consensus_pos(locs, pos) == want


def test_a9_asymmetry():
    # a cluster only at pos+100 -> -1; one noise read at pos-200 -> 1100
    assert O.consensus_pos([1100] * 5, 1000) == -1
    assert O.consensus_pos([1100] * 5 + [800], 1000) == 1100


def test_bounds_semantics():
    import ctypes as C
    import numpy as np
    L = O.lib()
    a = np.array([1, 3, 3, 7], dtype=np.int32)
    p = a.ctypes.data
    # lower_bound: first i with a[i] > x -> i-1 (0 if i==0); none -> n-1
    assert L.orc_lower_bound(C.c_void_p(p), 4, 0) == 0
    assert L.orc_lower_bound(C.c_void_p(p), 4, 3) == 2
    assert L.orc_lower_bound(C.c_void_p(p), 4, 100) == 3
    # upper_bound: first i with a[i] < x; none -> n-1
    assert L.orc_upper_bound(C.c_void_p(p), 4, 2) == 0
    assert L.orc_upper_bound(C.c_void_p(p), 4, 1) == 3
    assert L.orc_upper_bound(C.c_void_p(p), 4, 0) == 3


def test_min_count_gate():
    assert O.consensus_pos([1000, 1000], 1000, min_count=3) == -1
    assert O.consensus_pos([1000, 1000], 1000, min_count=2) == 1000
