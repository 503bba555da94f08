#!/bin/bash
# Wave-state counters of the C2 bench's kernels (one SQ pass): where the
# waves of the pair-table GEMMs and the aggregations spend their cycles.
#   scripts/pmc_stalls.sh <tag> [extra bench flags...]
# WAIT_ANY = parked on s_waitcnt / barrier; WAIT_INST_ANY = issue stalls
# (MFMA dependency, pipe busy); WAIT_INST_LDS = LDS issue stalls; all in
# quad-cycles like WAVE_CYCLES (MI355X_MICROARCH.md, rocprofv3 PMC slots).
set -o pipefail
TAG=${1:-stalls}
shift
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG}
mkdir -p $OUT
B="--steps 10 --warmup 3 --no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0 --no-interference-probe"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS --kernel-trace -d $OUT/sq -o run --output-format csv -- \
  python3 bench.py $B "$@" > $OUT/sq.log 2>&1 || { echo "sq pass failed"; tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/sq2 -o run --output-format csv -- \
  python3 bench.py $B "$@" > $OUT/sq2.log 2>&1 || { echo "sq2 pass failed"; tail -5 $OUT/sq2.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for p in ("sq", "sq2"):
    f = glob.glob(f"{out}/{p}/**/*counter_collection.csv", recursive=True)
    if not f:
        print("no counter csv for", p); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if not any(s in k for s in ("k_h2_", "k_spmm_gather", "k_top", "k_gemm", "k_s3")):
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
    for k, d in acc.items():
        short = k.split("(")[0][-70:]
        cnt = max(n[(k, c)] for c in d)
        print(short, {c: round(v / max(n[(k, c)], 1)) for c, v in sorted(d.items())})
PY
echo done
