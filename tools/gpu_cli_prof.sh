#!/bin/bash
# Run ON THE GPU BOX: write a workload's BAM (with SEQ/QUAL) + VCF once, then a rocprofv3 kernel +
# memory-copy trace of one `svtrek audt --inflate gpu` run on it (the device ingest's stage split).
#   tools/gpu_cli_prof.sh TAG [workload]
set -u
TAG=${1:?tag}; WL=${2:-cfg2_10kdel_30x_ont}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
D=$(mktemp -d /tmp/svt_cli_XXXX)
timeout -k 10 600 python -u tools/e2e_bench.py --workload "$WL" --with-seq -t 16 --reps 1 --inflate gpu --dir "$D" \
  > "$OUT/e2e.log" 2>&1 || { tail -5 "$OUT/e2e.log"; exit 1; }
tail -1 "$OUT/e2e.log" | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  svtrek_amd/svtrek audt -b "$D/w.bam" -v "$D/w.vcf" -t 16 --verbose --inflate gpu > "$OUT/cli.out" 2> "$OUT/cli.err"
rc=$?
tail -3 "$OUT/cli.err"
rm -rf "$D"
exit $rc
