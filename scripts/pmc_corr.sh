#!/bin/bash
# Counter study of the all-pairs volume + pyramid kernel (corr_flat_kernel) at
# the training shape (8 x 46 x 62, C = 256): one rocprofv3 run per counter
# pass (SQ <= 8, TCC <= 4 per pass), then a per-kernel mean of every counter.
set -o pipefail
OUT=gpurun_out/pmc_corr
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
PASSES=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
        "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
        "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum")
timeout -k 10 120 python3 scripts/bench_corr.py --hw 46 62 --batch 8 --reps 20 > $OUT/timing.log 2>&1 || { tail -5 $OUT/timing.log; exit 1; }
cat $OUT/timing.log | grep -v amdgpu
for i in 0 1 2; do
  timeout -s KILL 90 rocprofv3 --pmc ${PASSES[$i]} --output-format csv -d /tmp/pmccorr_$i -o pmc -- \
    python3 scripts/bench_corr.py --hw 46 62 --batch 8 --reps 3 > $OUT/p$i.log 2>&1 || { echo "FAILED pass $i"; tail -5 $OUT/p$i.log; exit 1; }
  find /tmp/pmccorr_$i -name "*counter_collection.csv" -exec cp {} $OUT/p$i.csv \;
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/pmc_corr/p*.csv")):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if "corr_flat" not in name:
            continue
        key = name.split("(")[0][-40:]
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open("gpurun_out/pmc_corr/summary.txt", "w") as out:
    for k, d in acc.items():
        out.write(k + "\n")
        for c, v in sorted(d.items()):
            out.write(f"  {c:32s} {sum(v) / len(v):14.1f}  (n={len(v)})\n")
print(open("gpurun_out/pmc_corr/summary.txt").read())
PY
