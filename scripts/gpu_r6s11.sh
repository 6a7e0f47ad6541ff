set -o pipefail
OUT=gpurun_out/r6s11
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py -k "conv1x1 or v3_epilogues" > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -3 $OUT/test.log
timeout -k 10 300 python scripts/bench_1x1.py > $OUT/b1x1.log 2>&1 || { tail -20 $OUT/b1x1.log; exit 1; }
cat $OUT/b1x1.log
timeout -k 10 300 python scripts/bench_1x1.py --scan > $OUT/scan.log 2>&1 || { tail -20 $OUT/scan.log; exit 1; }
cat $OUT/scan.log
