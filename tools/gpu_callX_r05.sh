#!/bin/bash
# Round 5, call X: the BGZF inflate's remaining costs -- variants of engine 0.23.3 on
# tools/bench_inflate.py: x_nofar (diagnostic: far matches read the ring, wrong bytes: what the
# far loads cost), x_small (9-bit literal/length root, 1 KiB ring: 4.5 KB of LDS a wave), x_small8
# (the same at 8 waves per SIMD), x_w7 (7 waves per SIMD), against the in-tree build.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/${CALL_TAG:-r05_X}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for v in ${VARS:-new x_nofar x_small x_small8 x_w7}; do
    lib=""; [ $v != new ] && lib=$PWD/variants/$v.so
    SVTREK_ENGINE_LIB=$lib timeout -k 10 300 python tools/bench_inflate.py --scale 0.1 --reps 3 > "$OUT/inf_${v}_$rep.log" 2>&1
    rc=$?   # (1: output differs from zlib -- expected of the diagnostic x_nofar only)
    if [ $rc -ne 0 ] && ! { [ $rc -eq 1 ] && [ $v = x_nofar ]; }; then echo "inf $v failed rc=$rc"; tail -5 "$OUT/inf_${v}_$rep.log"; exit 1; fi
    python - "$v $rep" "$OUT/inf_${v}_$rep.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], d["kernel_ms"], "ms", d["kernel_gbs"], "GB/s identical", d["identical_to_zlib"])
PY
  done
done
echo done
