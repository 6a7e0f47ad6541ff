set -o pipefail
OUT=gpurun_out/r6s2
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_fused_gpu.py -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider -k "bf16_training_grads or segment_offsets or v3_tiles" > $OUT/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.txt; exit 1; }
grep "bf16 vs fp32" $OUT/pytest.txt; tail -1 $OUT/pytest.txt
timeout -k 10 300 python scripts/bench_encoders.py > $OUT/enc.log 2>&1 || { tail -20 $OUT/enc.log; exit 1; }
cat $OUT/enc.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/pe_e -o enc -- python3 scripts/bench_encoders.py --graph-only --reps 5 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
f=$(find /tmp/pe_e -name "*kernel_trace.csv" | head -1); gzip -c $f > $OUT/enc_trace.csv.gz
echo done
