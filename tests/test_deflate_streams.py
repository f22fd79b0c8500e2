"""The hand-built DEFLATE streams of tests/deflate_streams.py are what zlib says they are: the
GPU inflater's accept / reject cases (tests/test_gpu_inflate.py) are judged against zlib's own
verdict on each, so the streams themselves are checked here on the CPU."""
import random
import zlib

import deflate_streams as D


def test_zlib_round_trips_every_kind():
    rng = random.Random(1)
    for kind in D.KINDS:
        d = D.data(kind, rng)
        for level in (0, 1, 6, 9):
            for strat in D.STRATEGIES:
                assert zlib.decompressobj(-15).decompress(D.deflate(d, level, strat)) == d


def test_hand_built_blocks_match_zlib_verdicts():
    data = b"SVTrek"
    lit_ok = [9] * 256 + [1]
    for cl, lit, dist, valid in [({9: 1, 1: 2, 2: 2}, lit_ok, [1], True),
                                 ({9: 1, 1: 2}, lit_ok, [1], False),
                                 ({9: 1, 2: 2, 1: 2}, [9] * 256 + [2], [1], False)]:
        comp = D.dynamic_block(cl, lit, dist, data)
        assert D.zlib_ok(comp, len(data)) == valid


def test_crafted_streams_decode_as_written():
    """The crafted multi-block streams (far-edge matches, stored after dynamic blocks, chunk-end
    outputs, long codes) inflate under zlib to exactly the bytes the writer expanded."""
    import random
    import zlib
    for comp, plain, name in D.crafted_streams(random.Random(17)):
        assert zlib.decompressobj(-15).decompress(comp) == plain, name
        assert 0 < len(plain) <= 65536, name
