set -o pipefail
OUT=gpurun_out/r6s16
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python scripts/host_profile.py --steps 20 > $OUT/host.log 2>&1 || { tail -20 $OUT/host.log; exit 1; }
cat $OUT/host.log
