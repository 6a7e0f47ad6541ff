set -o pipefail
OUT=gpurun_out/r6s27d
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_v3f_gpu.py tests/test_enc_f32_train_gpu.py tests/test_conv_f32_gpu.py > $OUT/test.log 2>&1 || { tail -40 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
for r in 1 2; do
timeout -k 10 300 python bench.py --fp32 --steps 12 --warmup 3 --infer-reps 30 > $OUT/b_fp32.$r.log 2>&1 || { tail -20 $OUT/b_fp32.$r.log; exit 1; }
tail -1 $OUT/b_fp32.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fp32", d["value"], d["ms_per_step"], d["inference"]["ms_per_pair"])'
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf -o train -- python3 bench.py --fp32 --steps 5 --warmup 3 --no-infer > $OUT/prof_fp32.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_fp32.log; exit 1; }
find /tmp/pf -name "*kernel_stats.csv" -exec cp {} $OUT/train_fp32_kernel_stats.csv \;
