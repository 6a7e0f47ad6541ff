set -o pipefail
mkdir -p gpurun_out/trace
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr -o t -- python3 bench.py --steps 1 --warmup 2 --no-infer > gpurun_out/trace/log 2>&1 || exit 1
find /tmp/tr -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace/kt.csv \;
