#!/bin/bash
# Round-4 first GPU session: the tests changed by the advisor fixes, the
# default bench, the update-block conv counter study, the data-feed bench.
set -o pipefail
mkdir -p gpurun_out/s1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_enc_geo_gpu.py::test_graphed_inference_sees_weight_updates tests/test_norm_gpu.py tests/test_ddp_gpu.py \
  > gpurun_out/s1/pytest.log 2>&1; rc=$?
tail -n 3 gpurun_out/s1/pytest.log
if [[ $rc -ne 0 && $rc -ne 1 ]]; then echo "pytest rc=$rc: stop"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/s1/bench.log 2>&1 || { tail -20 gpurun_out/s1/bench.log; exit 1; }
tail -n 1 gpurun_out/s1/bench.log
bash scripts/pmc_update_conv.sh > gpurun_out/s1/pmc.log 2>&1 || { tail -20 gpurun_out/s1/pmc.log; exit 1; }
tail -n 40 gpurun_out/s1/pmc.log
for w in 4 8 16; do timeout -k 10 300 python scripts/bench_dataloader.py --workers $w --batches 40 2>&1 | tail -1; done > gpurun_out/s1/feed.log
cat gpurun_out/s1/feed.log
