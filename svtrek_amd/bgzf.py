"""BGZF block tables (SAM spec 4.1) for svt_bgzf_inflate: where each block's raw DEFLATE data
lies in the compressed bytes and where its ISIZE bytes go in the output."""
from __future__ import annotations

import numpy as np

from ._lib import BGZF_BLOCK_DTYPE


def block_table(comp) -> np.ndarray:
    """Walk the BGZF headers of `comp` (bytes / uint8 array holding whole blocks) and return
    BGZF_BLOCK_DTYPE rows, outputs packed back to back.  Raises on a malformed header."""
    buf = memoryview(comp).cast("B")
    n = len(buf)
    rows = []
    p = u = 0
    while p < n:
        if n - p < 18 or buf[p] != 31 or buf[p + 1] != 139 or buf[p + 2] != 8 or not buf[p + 3] & 4:
            raise ValueError(f"not a BGZF block at byte {p}")
        xlen = buf[p + 10] | buf[p + 11] << 8
        bsize, x = 0, 0
        while x + 4 <= xlen:
            si1, si2, slen = buf[p + 12 + x], buf[p + 13 + x], buf[p + 14 + x] | buf[p + 15 + x] << 8
            if si1 == 66 and si2 == 67 and slen == 2:
                bsize = (buf[p + 16 + x] | buf[p + 17 + x] << 8) + 1
            x += 4 + slen
        if not bsize or p + bsize > n:
            raise ValueError(f"BGZF block at byte {p}: no BC subfield or truncated")
        isize = int.from_bytes(buf[p + bsize - 4:p + bsize], "little")
        rows.append((p + 12 + xlen, u, bsize - xlen - 20, isize))
        u += isize
        p += bsize
    return np.array(rows, dtype=BGZF_BLOCK_DTYPE)
