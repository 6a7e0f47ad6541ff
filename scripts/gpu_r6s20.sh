set -o pipefail
OUT=gpurun_out/r6s20
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_v3f_gpu.py tests/test_fused_gpu.py tests/test_enc_conv_gpu.py > $OUT/test.log 2>&1 || { tail -40 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
cd scripts && timeout -k 10 300 python bench_v3f.py > ../$OUT/bv3f.log 2>&1 || { tail -20 ../$OUT/bv3f.log; exit 1; }
cat ../$OUT/bv3f.log
