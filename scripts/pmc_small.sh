#!/bin/bash
# PMC counters of the small VALU kernels (one rocprofv3 pass per counter set).
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
for k in wgrad fwd enc; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d /tmp/pmc_$k -o p -- python3 scripts/pmc_small.py $k > gpurun_out/pmc/$k.log 2>&1 || exit 1
  find /tmp/pmc_$k -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc/$k.csv \;
done
